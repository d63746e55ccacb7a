"""MuJoCo's soft-constraint model pinned by closed forms (not by either restatement).

The solref/solimp -> impedance -> efc_D / efc_aref arithmetic is written twice
in this repo (oracle/oracle.c efc_row_params and csrc/mjh_step.hip), so a
shared error would pass every oracle-vs-HIP parity test. These tests pin it to
MuJoCo's DOCUMENTED soft-constraint model instead, restated here in a few lines
of numpy from the published definitions (MuJoCo documentation, Computation ->
"Soft constraints" / "Solver parameters"; the reference sets these parameters
through ``spec_config.py:159-161,230-231`` and the MJCF defaults):

* solref = (timeconst, dampratio), with timeconst raised to 2*timestep
  ("refsafe"); solimp = (dmin, dmax, width, midpoint, power);
* impedance d(r): x = |r| / width; d = dmax for x >= 1, else
  d = dmin + y(x) (dmax - dmin) with y = x^p / mid^(p-1) below the midpoint and
  1 - (1-x)^p / (1-mid)^(p-1) above it;
* stiffness and damping b = 2 / (dmax tc), k = d(r) / (dmax^2 tc^2 zeta^2);
* reference acceleration aref = -b v - k r (v = J qvel, r = the constraint
  violation: the contact distance), regulariser R = (1-d)/d * A with A the
  diagonal approximation of J M^-1 J^T (a contact's body invweight0);
* the constrained acceleration of a single active row then obeys
  a1 + d (b v + k r) = (1 - d) a0 (a0 the unconstrained acceleration).

For a free sphere of mass m on a plane (condim 1: one normal row, J = the
normal, A = 1/m exactly because the contact point lies on the line through the
centre) everything reduces to a scalar recurrence in the penetration r and
velocity v, which these tests iterate in numpy:

  a1 = (1 - d) (-g) + d (-b v - k r)   while the row is active (a1 > -g),
  v' = v + dt a1,  z' = z + dt v'      (semi-implicit Euler).

Known answers derived from it:
* the resting penetration r* solves (1 - d(r*)) g = -d(r*) k(r*) r*, i.e.
  r* = -(1 - d) g / (d^2 K) with K = 1 / (dmax^2 tc^2 zeta^2);
* with dmin = dmax (constant d) the penetration error e = r - r* obeys
  e'' + (2/tc) e' + e / (tc zeta)^2 = 0: critically damped at zeta = 1, decaying
  with time constant tc: e(t) = (e0 + (v0 + e0/tc) t) exp(-t/tc);
* pyramidal condim 3 (friction mu, impratio 1): four edge rows n +/- mu t with
  A = (1 + mu^2) * 2 mu^2 / m each (MuJoCo's pyramidal diagApprox); at rest their
  summed normal force carries m g, so r* = -(1 - d) g (1 + mu^2) mu^2 / (2 d^2 K).

Tolerances: float64 oracle 1e-6 relative on r* (the solver's own tolerance
sets the floor) and 1e-9 m along trajectories; the HIP step (float32):
efc_D and efc_aref 2e-4 relative, r* 2e-3 relative.
"""

import numpy as np
import pytest
from scipy.optimize import brentq

from mjlab_amd.spec.compiler import compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from oracle.oracle import Oracle

G = 9.81
MASS, RAD = 2.0, 0.1

# (solref, solimp) sets: the default, one where d(r) varies across the resting
# penetration (wide sigmoid, underdamped), and a refsafe case (tc < 2 dt)
PARAMS = {
  "default": ((0.02, 1.0), (0.9, 0.95, 0.001, 0.5, 2.0)),
  "soft": ((0.05, 0.5), (0.8, 0.99, 0.01, 0.3, 3.0)),
  "refsafe": ((0.004, 1.0), (0.85, 0.95, 0.002, 0.6, 1.0)),
}


def ball_xml(solref, solimp, condim=1, friction=1.0, dt=0.005):
  ref = " ".join(str(x) for x in solref)
  imp = " ".join(str(x) for x in solimp)
  attr = f'condim="{condim}" friction="{friction} 0.005 0.0001" solref="{ref}" solimp="{imp}"'
  return f"""<mujoco><option timestep="{dt}"/><worldbody>
  <geom name="floor" type="plane" size="5 5 0.1" {attr}/>
  <body name="ball" pos="0 0 1"><freejoint/><geom type="sphere" size="{RAD}" mass="{MASS}" {attr}/></body>
  </worldbody></mujoco>"""


def ball_model(solref, solimp, condim=1, friction=1.0, dt=0.005, **opt):
  m = compile_spec(read_mjcf_string(ball_xml(solref, solimp, condim, friction, dt)), 8, 32)
  m.iterations, m.tolerance = 50, 1e-12
  for k, v in opt.items():
    setattr(m, k, v)
  return m


# ---------------------------------------------------------------- the closed form (MuJoCo docs)
def impedance(r, solimp):
  dmin, dmax, width, mid, p = solimp
  x = abs(r) / width
  if x >= 1:
    return dmax
  y = x**p / mid ** (p - 1) if x < mid else 1 - (1 - x) ** p / (1 - mid) ** (p - 1)
  return dmin + y * (dmax - dmin)


def kb(solref, solimp, dt):
  tc, zeta = max(solref[0], 2 * dt), solref[1]
  dmax = solimp[1]
  return 1.0 / (dmax**2 * tc**2 * zeta**2), 2.0 / (dmax * tc)  # K (k = d K), b


def efc_closed_form(r, v, solref, solimp, dt, A):
  """(efc_D, efc_aref) of a contact row at distance r < 0 and normal velocity v."""
  K, b = kb(solref, solimp, dt)
  d = impedance(r, solimp)
  return d / ((1 - d) * A), -b * v - K * d * r


def rest_penetration(solref, solimp, dt, factor=1.0):
  """r* < 0 with factor (1 - d) g = -d^2 K r (factor = 1 for one normal row)."""
  K, _ = kb(solref, solimp, dt)
  f = lambda r: factor * (1 - impedance(r, solimp)) * G + impedance(r, solimp) ** 2 * K * r
  return brentq(f, -1.0, -1e-15, xtol=1e-18, rtol=1e-14)


def recurrence(z0, v0, nstep, solref, solimp, dt):
  """The scalar soft-contact recurrence of a condim-1 ball: heights after each step."""
  K, b = kb(solref, solimp, dt)
  z, v, out = z0, v0, []
  for _ in range(nstep):
    r = z - RAD
    a = -G
    if r < 0:
      d = impedance(r, solimp)
      a1 = (1 - d) * (-G) + d * (-b * v - K * d * r)
      a = max(a, a1)  # the row only pushes (inactive when the unconstrained a0 already exceeds it)
    v = v + dt * a
    z = z + dt * v
    out.append(z)
  return np.array(out)


def rollout(orc, z0, v0, nstep):
  st = {"qpos": np.array([[0, 0, z0, 1, 0, 0, 0]], float), "qvel": np.array([[0, 0, v0, 0, 0, 0]], float)}
  zs, out = [], None
  for _ in range(nstep):
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    zs.append(st["qpos"][0, 2])
  return np.array(zs), out


# ---------------------------------------------------------------- oracle (float64)
def test_closed_form_is_self_consistent():
  """The numpy restatement: r* is a fixed point of the recurrence, and the
  decay closed form is the continuous limit of the recurrence (dt -> 0)."""
  for solref, solimp in PARAMS.values():
    rs = rest_penetration(solref, solimp, 0.005)
    zs = recurrence(RAD + rs, 0.0, 5, solref, solimp, 0.005)
    np.testing.assert_allclose(zs - RAD, rs, rtol=1e-9)
  tc = 0.05
  e0 = -0.004
  for dt, tol in ((1e-3, 0.03), (1e-4, 0.003)):
    solimp = (0.9, 0.9, 0.001, 0.5, 2.0)
    rs = rest_penetration((tc, 1.0), solimp, dt)
    n = int(0.3 / dt)
    e = recurrence(RAD + rs + e0, 0.0, n, (tc, 1.0), solimp, dt) - RAD - rs
    t = dt * np.arange(1, n + 1)
    exact = (e0 + e0 / tc * t) * np.exp(-t / tc)
    assert np.abs(e - exact).max() < tol * abs(e0)


@pytest.mark.parametrize("name", sorted(PARAMS))
@pytest.mark.parametrize("ls_parallel", [0, 1])
def test_oracle_efc_rows_match_closed_form(name, ls_parallel):
  """efc_D and efc_aref of the contact row at a range of penetrations and
  approach/separation velocities: the oracle's row parameters equal the
  documented formulas (A = the ball's invweight0 = 1/m)."""
  solref, solimp = PARAMS[name]
  m = ball_model(solref, solimp, ls_parallel=ls_parallel)
  assert m.body_invweight0[1, 0] == pytest.approx(1 / MASS, rel=1e-12)
  rng = np.random.default_rng(7)
  n = 32
  r = -rng.uniform(1e-5, 0.02, n)
  v = rng.uniform(-0.5, 0.5, n)
  q = np.tile([0, 0, 0, 1, 0, 0, 0], (n, 1)).astype(float)
  q[:, 2] = RAD + r
  qv = np.zeros((n, 6))
  qv[:, 2] = v
  out = Oracle(m).run(n, {"qpos": q, "qvel": qv}, integrate=False)
  assert (out["nefc"][:, 0] == 1).all()
  for w in range(n):
    D, aref = efc_closed_form(r[w], v[w], solref, solimp, m.timestep, 1 / MASS)
    assert out["efc_D"][w, 0] == pytest.approx(D, rel=1e-12)
    assert out["efc_aref"][w, 0] == pytest.approx(aref, rel=1e-12, abs=1e-12)


@pytest.mark.parametrize("name", sorted(PARAMS))
def test_oracle_trajectory_follows_soft_contact_recurrence(name):
  """Dropped from 5 mm above the floor: the oracle's whole trajectory (impact,
  approach, rest) equals the scalar recurrence of the documented model."""
  solref, solimp = PARAMS[name]
  m = ball_model(solref, solimp)
  zs, _ = rollout(Oracle(m), RAD + 0.005, 0.0, 300)
  ref = recurrence(RAD + 0.005, 0.0, 300, solref, solimp, m.timestep)
  np.testing.assert_allclose(zs, ref, atol=1e-9, rtol=0)


@pytest.mark.parametrize("name", sorted(PARAMS))
def test_oracle_rest_penetration(name):
  """The ball comes to rest at r* = -(1 - d(r*)) g / (d(r*)^2 K) (1e-6
  relative), with the vertical constraint force m g."""
  solref, solimp = PARAMS[name]
  m = ball_model(solref, solimp)
  zs, out = rollout(Oracle(m), RAD + 0.002, 0.0, 800)  # 4 s
  rs = rest_penetration(solref, solimp, m.timestep)
  assert zs[-1] - RAD == pytest.approx(rs, rel=1e-6)
  assert abs(out["qvel"][0]).max() < 1e-8
  assert out["qfrc_constraint"][0, 2] == pytest.approx(MASS * G, rel=1e-8)


@pytest.mark.parametrize("mu", [1.0, 0.5])
def test_oracle_rest_penetration_pyramidal(mu):
  """condim 3, pyramidal cone: four edge rows at rest, r* with the pyramidal
  diagApprox factor (1 + mu^2) mu^2 / 2 (= 1 at MuJoCo's default mu = 1)."""
  solref, solimp = PARAMS["default"]
  m = ball_model(solref, solimp, condim=3, friction=mu)
  zs, out = rollout(Oracle(m), RAD + 0.002, 0.0, 800)
  assert int(out["nefc"][0, 0]) == 4
  rs = rest_penetration(solref, solimp, m.timestep, factor=(1 + mu * mu) * mu * mu / 2)
  assert zs[-1] - RAD == pytest.approx(rs, rel=1e-6)


@pytest.mark.parametrize("zeta", [1.0, 0.5])
def test_oracle_penetration_error_decays_with_timeconst(zeta):
  """Constant impedance (dmin = dmax = 0.9), small time step (1 ms, tc 50 ms):
  the penetration error follows the continuous mass-spring-damper of the
  documented model, e'' + (2/tc) e' + e/(tc zeta)^2 = 0 (critically damped at
  zeta = 1), to 3 % of the initial error. The start (2 mm below rest) keeps
  the underdamped overshoot in contact."""
  tc, dt, e0 = 0.05, 0.0005, -0.002
  solimp = (0.9, 0.9, 0.001, 0.5, 2.0)
  m = ball_model((tc, zeta), solimp, dt=dt)
  rs = rest_penetration((tc, zeta), solimp, dt)
  n = 600
  zs, _ = rollout(Oracle(m), RAD + rs + e0, 0.0, n)
  e = zs - RAD - rs
  t = dt * np.arange(1, n + 1)
  if zeta == 1.0:
    exact = (e0 + e0 / tc * t) * np.exp(-t / tc)
  else:  # underdamped: e = exp(-t/tc) (e0 cos(wd t) + e0/(tc wd) sin(wd t))
    wd = np.sqrt(1 / (tc * zeta) ** 2 - 1 / tc**2)
    exact = np.exp(-t / tc) * (e0 * np.cos(wd * t) + e0 / (tc * wd) * np.sin(wd * t))
  assert np.abs(e - exact).max() < 0.03 * abs(e0), np.abs(e - exact).max() / abs(e0)


# ---------------------------------------------------------------- HIP step (float32)
@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PARAMS))
def test_gpu_efc_rows_and_rest_match_closed_form(name):
  """The HIP step's efc_D / efc_aref against the closed form (2e-4 relative),
  and a HIP rollout's resting penetration against r* (2e-3 relative)."""
  import torch

  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg

  dev = "cuda:0"
  solref, solimp = PARAMS[name]
  m = ball_model(solref, solimp)
  n = 64
  sim = Simulation(n, SimulationCfg(nconmax=8, njmax=32, mujoco=MujocoCfg(timestep=m.timestep, iterations=50,
                                                                          tolerance=1e-10)), m, dev)
  rng = np.random.default_rng(11)
  r = -rng.uniform(1e-4, 0.02, n)
  v = rng.uniform(-0.5, 0.5, n)
  q = np.tile([0, 0, 0, 1, 0, 0, 0], (n, 1)).astype(np.float32)
  q[:, 2] = RAD + r
  qv = np.zeros((n, 6), np.float32)
  qv[:, 2] = v
  sim.data.qpos.copy_(torch.as_tensor(q, device=dev))
  sim.data.qvel.copy_(torch.as_tensor(qv, device=dev))
  sim.forward()
  torch.cuda.synchronize()
  nefc = sim.data.nefc.cpu().numpy().reshape(n)
  D = sim.data.efc_D.cpu().numpy().reshape(n, -1)[:, 0]
  aref = sim.data.efc_aref.cpu().numpy().reshape(n, -1)[:, 0]
  assert (nefc == 1).all()
  rz = q[:, 2].astype(np.float64) - float(np.float32(RAD))  # the float32 state the device saw
  for w in range(n):
    Dc, arefc = efc_closed_form(rz[w], float(qv[w, 2]), solref, solimp, m.timestep, 1 / MASS)
    assert D[w] == pytest.approx(Dc, rel=2e-4), (w, rz[w])
    assert aref[w] == pytest.approx(arefc, rel=2e-4, abs=1e-3), (w, rz[w], float(qv[w, 2]))
  # rest: every world from its own start settles at r*
  q[:, 2] = RAD + rng.uniform(0.0, 0.004, n)
  sim.data.qpos.copy_(torch.as_tensor(q, device=dev))
  sim.data.qvel.zero_()
  sim.data.qacc_warmstart.zero_()
  for _ in range(800):
    sim.step()
  torch.cuda.synchronize()
  rs = rest_penetration(solref, solimp, m.timestep)
  z = sim.data.qpos[:, 2].double().cpu().numpy()
  np.testing.assert_allclose(z - RAD, rs, rtol=2e-3)
  fz = sim.data.qfrc_constraint[:, 2].double().cpu().numpy()
  np.testing.assert_allclose(fz, MASS * G, rtol=1e-4)
