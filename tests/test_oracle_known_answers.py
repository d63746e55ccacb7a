"""The oracle (CPU restatement of mj_step) against analytic known answers.

Physics numerics are not pinned by the reference's own tests (MuJoCo / MuJoCo
Warp are absent here: SURVEY.md §8c), so the oracle is pinned by closed-form
results instead: free fall, torque-free momentum conservation, pendulum energy,
a static stance carrying the robot's weight, and PD equilibrium."""

import numpy as np
import pytest

from mjlab_amd.spec.compiler import compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from oracle.oracle import Oracle
from tests.scenes import g1_scene_model

FREE_BALL = """
<mujoco>
  <option timestep="0.005"/>
  <worldbody>
    <geom name="floor" type="plane" size="5 5 0.1"/>
    <body name="ball" pos="0 0 1">
      <freejoint/>
      <geom type="sphere" size="0.1" mass="2"/>
    </body>
  </worldbody>
</mujoco>
"""

PENDULUM = """
<mujoco>
  <option timestep="0.001"/>
  <worldbody>
    <body name="link1" pos="0 0 2">
      <joint name="j1" type="hinge" axis="0 1 0"/>
      <geom type="capsule" fromto="0 0 0 0.5 0 0" size="0.03" mass="1" contype="0" conaffinity="0"/>
      <body name="link2" pos="0.5 0 0">
        <joint name="j2" type="hinge" axis="0 1 0"/>
        <geom type="capsule" fromto="0 0 0 0.5 0 0" size="0.03" mass="1" contype="0" conaffinity="0"/>
      </body>
    </body>
  </worldbody>
</mujoco>
"""


def _model(xml, **opt):
  m = compile_spec(read_mjcf_string(xml), 16, 64)
  for k, v in opt.items():
    setattr(m, k, v)
  return m


def test_free_fall_first_step():
  m = _model(FREE_BALL)
  out = Oracle(m).run(1, {"qpos": m.qpos0[None]}, integrate=True, debug=True)
  g, dt = 9.81, m.timestep
  assert out["ncon"][0, 0] == 0
  # qM of a free solid sphere (mass 2, radius 0.1): diag(m, m, m, 2/5 m r^2 x 3)
  np.testing.assert_allclose(out["qM"][0].reshape(6, 6), np.diag([2.0] * 3 + [0.4 * 2.0 * 0.01] * 3), atol=1e-12)
  np.testing.assert_allclose(out["qacc_smooth"][0], [0, 0, -g, 0, 0, 0], atol=1e-12)
  np.testing.assert_allclose(out["qacc"][0], [0, 0, -g, 0, 0, 0], atol=1e-12)
  assert out["qvel"][0, 2] == pytest.approx(-g * dt, abs=1e-12)
  assert out["qpos"][0, 2] == pytest.approx(1.0 - g * dt * dt, abs=1e-12)  # semi-implicit Euler
  assert out["time"][0, 0] == pytest.approx(dt)


def test_resting_ball_contact_jacobian():
  """Ball touching the floor: one frictional contact (condim 3 -> 4 pyramid
  rows). Each row of efc_J is frame-row combinations of the contact point
  Jacobian of the ball's free joint: translation columns = the pyramid edge
  directions n +/- mu t (frame rows), rotation columns = (c - p) x edge with c
  the contact point and p the ball centre."""
  m = _model(FREE_BALL)
  st = {"qpos": m.qpos0[None].copy()}
  st["qpos"][0, 2] = 0.0999
  out = Oracle(m).run(1, st, integrate=False, debug=True)
  assert out["ncon"][0, 0] == 1 and out["nefc"][0, 0] == 4
  J = out["efc_J"][0].reshape(m.njmax, 6)[:4]
  fr = out["contact_frame"][0, :9].reshape(3, 3)
  mu = out["contact_friction"][0, 0]
  c, p = out["contact_pos"][0, :3], st["qpos"][0, :3]
  for r in range(4):
    edge = fr[0] + (1 if r % 2 == 0 else -1) * mu * fr[1 + r // 2]
    np.testing.assert_allclose(J[r, :3], edge, atol=1e-12)
    np.testing.assert_allclose(J[r, 3:], np.cross(c - p, edge), atol=1e-12)


def test_ball_comes_to_rest_on_floor():
  m = _model(FREE_BALL)
  orc = Oracle(m)
  st = {"qpos": m.qpos0[None].copy()}
  st["qpos"][0, 2] = 0.12
  for _ in range(400):
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
  # resting at MuJoCo's documented soft-contact penetration r* (default
  # solref/solimp, pyramidal condim 3 at mu = 1: tests/test_soft_constraint.py
  # derives r* = -(1 - d) g / (d^2 K) from the published model), normal force = m g
  from tests.test_soft_constraint import rest_penetration
  rs = rest_penetration((0.02, 1.0), (0.9, 0.95, 0.001, 0.5, 2.0), m.timestep)
  assert st["qpos"][0, 2] - 0.1 == pytest.approx(rs, rel=1e-5)
  assert abs(st["qvel"][0]).max() < 1e-6
  fz = out["qfrc_constraint"][0, 2]
  assert fz == pytest.approx(2 * 9.81, rel=1e-3)


def test_momentum_conserved_without_gravity_or_contacts():
  """Free-floating G1, no gravity, contacts off: internal PD torques cannot move
  the centre of mass — subtree_com of the root moves with constant velocity."""
  m = g1_scene_model(1)
  m.gravity = np.zeros(3)
  orc = Oracle(m)
  st = {"qpos": m.key_qpos[None].copy(), "ctrl": m.key_ctrl[None] + 0.3}
  st["qpos"][0, 2] += 5.0  # far above the floor
  coms = []
  for _ in range(40):
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    st["ctrl"] = m.key_ctrl[None] + 0.3
    coms.append(out["subtree_com"][0, 6:9].copy())  # body 2 = robot root (0 world, 1 terrain)
  # self-contacts may occur: internal forces, momentum still conserved
  world_com = np.array(coms)
  # zero initial momentum: the COM stays put (to the O(dt^2) error of
  # integrating in generalized coordinates) while the limbs swing
  assert np.abs(world_com - world_com[0]).max() < 1e-4
  assert np.abs(st["qpos"][0, 7:] - m.key_qpos[7:]).max() > 0.05


def test_pendulum_energy_bounded():
  m = _model(PENDULUM)
  orc = Oracle(m)
  st = {"qpos": np.array([[0.3, 0.2]])}
  mass = m.body_mass
  g = 9.81

  def energy(o):
    # potential from body COM heights; kinetic from cvel (spatial velocity at com frame)
    pe = sum(mass[b] * g * o["xipos"][0, 3 * b + 2] for b in range(1, m.nbody))
    ke = 0.0
    for b in range(1, m.nbody):
      cv = o["cvel"][0, 6 * b : 6 * b + 6]
      w, v0 = cv[:3], cv[3:]
      r = o["xipos"][0, 3 * b : 3 * b + 3] - o["subtree_com"][0, 0:3]
      v = v0 + np.cross(w, r)
      R = o["ximat"][0, 9 * b : 9 * b + 9].reshape(3, 3)
      I = R @ np.diag(m.body_inertia[b]) @ R.T
      ke += 0.5 * mass[b] * v @ v + 0.5 * w @ I @ w
    return pe, ke

  es, kes = [], []
  for _ in range(500):
    out = orc.run(1, st, integrate=False)
    pe_ke = energy(out)
    es.append(pe_ke[0] + pe_ke[1])
    kes.append(pe_ke[1])
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
  es = np.array(es)
  # semi-implicit Euler at dt=1ms: total energy drifts < 1% of the swing's kinetic energy
  assert max(kes) > 1.0
  assert np.ptp(es) / max(kes) < 1e-2


def test_g1_static_stance_carries_weight():
  """G1 dropped at its keyframe under PD hold: once the landing transient has
  died out (1 s), the vertical constraint force on the free joint carries the
  robot's weight m_total * g and the base has barely moved."""
  m = g1_scene_model(1)
  orc = Oracle(m)
  st = {"qpos": m.key_qpos[None].copy(), "ctrl": m.key_ctrl[None].copy()}
  fz = []
  for _ in range(200):
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    st["ctrl"] = m.key_ctrl[None].copy()
    fz.append(out["qfrc_constraint"][0, 2])
  mtot = m.body_mass.sum()
  assert np.mean(fz[150:]) == pytest.approx(mtot * 9.81, rel=0.02)
  assert out["ncon"][0, 0] >= 4
  assert abs(st["qpos"][0, 0]) < 0.1 and abs(st["qpos"][0, 2] - m.key_qpos[2]) < 0.05


def test_pd_actuator_force_law():
  """force = kp*(clamp(ctrl, range) - q) - kd*qdot, clamped to forcerange."""
  m = g1_scene_model(1)
  rng = np.random.default_rng(1)
  st = {"qpos": m.key_qpos[None].copy(), "qvel": rng.normal(0, 1, (1, m.nv)), "ctrl": m.key_ctrl[None] + rng.uniform(-3, 3, (1, m.nu))}
  st["qpos"][0, 2] += 2.0
  out = Oracle(m).run(1, st, integrate=False)
  for i in range(m.nu):
    j = int(m.actuator_trnid[i, 0]) if m.actuator_trnid.ndim == 2 else int(m.actuator_trnid[i])
    qa, va = int(m.jnt_qposadr[j]), int(m.jnt_dofadr[j])
    kp, kd = m.actuator_gainprm[i, 0], -m.actuator_biasprm[i, 2]
    lo, hi = m.actuator_ctrlrange[i]
    c = np.clip(st["ctrl"][0, i], lo, hi)
    f = kp * c - kp * st["qpos"][0, qa] - kd * st["qvel"][0, va]
    flo, fhi = m.actuator_forcerange[i]
    assert out["actuator_force"][0, i] == pytest.approx(np.clip(f, flo, fhi), rel=1e-9, abs=1e-9)


def test_oracle_struct_layouts_both_precisions():
  """The ctypes mirrors of or_model/or_data match the compiled oracle in both
  precisions (bench.py's cpu_baseline times float64 and float32)."""
  import ctypes

  from oracle.oracle import ORACLE_DIR, abi, build

  build()
  for prec, real in (("f64", ctypes.c_double), ("f32", ctypes.c_float)):
    lib = ctypes.CDLL(str(ORACLE_DIR / f"liboracle_{prec}.so"))
    lib.oracle_sizeof_model.restype = ctypes.c_size_t
    lib.oracle_sizeof_data.restype = ctypes.c_size_t
    assert ctypes.sizeof(abi.model_struct(real, device=False)) == lib.oracle_sizeof_model(), prec
    assert ctypes.sizeof(abi.data_struct(real, device=False)) == lib.oracle_sizeof_data(), prec


def test_compare_step_oracle_f32_vs_f64():
  """The parity checker itself (tests/scenes.py compare_step): the oracle's
  float32 build passes against its float64 build with integer outputs
  identical, so the tolerances are attainable by a correct float32 step."""
  import numpy as np

  from oracle.oracle import Oracle
  from tests.scenes import compare_step, g1_sensor_scene, random_states

  n = 64
  m = g1_sensor_scene(n).compile(50, 300)
  st = random_states(m, n, np.random.default_rng(12))
  rep = compare_step(Oracle(m, "f32").run(n, st, integrate=True, debug=True),
                     Oracle(m).run(n, st, integrate=True, debug=True))
  assert not rep["failures"], rep["failures"]
  assert "qM" in rep["maxerr"] and "efc_J" in rep["maxerr"]
  assert rep["int_match_rate"] >= 0.98


def _free_body_xml(bodies: str, gravity: str = "0 0 -9.81", plane: str = "") -> str:
  return f"""
<mujoco>
  <option timestep="0.002" gravity="{gravity}"/>
  <worldbody>
    {plane}
    {bodies}
  </worldbody>
</mujoco>
"""


def test_capsule_capsule_crossing_distance_and_frame():
  """Two crossed capsules (x- and y-axis, radius 0.05, centres 0.08 apart in z):
  one contact, dist = 0.08 - 0.1 = -0.02, normal along z, position midway
  between the surfaces on the common normal (MuJoCo's segment-segment test)."""
  xml = _free_body_xml("""
    <body name="a" pos="0 0 0.5"><freejoint/><geom type="capsule" fromto="-0.3 0 0 0.3 0 0" size="0.05"/></body>
    <body name="b" pos="0.1 0.05 0.58"><freejoint/><geom type="capsule" fromto="0 -0.3 0 0 0.3 0" size="0.05"/></body>
  """, gravity="0 0 0")
  m = _model(xml)
  out = Oracle(m).run(1, {"qpos": m.qpos0[None]}, integrate=False)
  assert out["ncon"][0, 0] == 1
  assert out["contact_dist"][0, 0] == pytest.approx(-0.02, abs=1e-12)
  n = out["contact_frame"][0, 0:3]
  assert abs(abs(n[2]) - 1.0) < 1e-12 and abs(n[0]) < 1e-12 and abs(n[1]) < 1e-12
  np.testing.assert_allclose(out["contact_pos"][0, 0:3], [0.1, 0.0, 0.54], atol=1e-12)


def test_capsule_capsule_separated_no_contact():
  xml = _free_body_xml("""
    <body name="a" pos="0 0 0.5"><freejoint/><geom type="capsule" fromto="-0.3 0 0 0.3 0 0" size="0.05"/></body>
    <body name="b" pos="0 0 0.62"><freejoint/><geom type="capsule" fromto="0 -0.3 0 0 0.3 0" size="0.05"/></body>
  """, gravity="0 0 0")
  m = _model(xml)
  out = Oracle(m).run(1, {"qpos": m.qpos0[None]}, integrate=False)
  assert out["ncon"][0, 0] == 0  # surfaces 0.02 apart, zero margin


def test_box_plane_corner_contacts():
  """Box (half sizes 0.2 x 0.1 x 0.05) sunk 0.01 into the floor, axis aligned:
  four corner contacts with dist -0.01 and normal +z (the Go1 trunk's pair)."""
  xml = _free_body_xml("""<body name="box" pos="0 0 0.04"><freejoint/><geom type="box" size="0.2 0.1 0.05"/></body>""",
                       plane='<geom name="floor" type="plane" size="5 5 0.1"/>')
  m = _model(xml)
  out = Oracle(m).run(1, {"qpos": m.qpos0[None]}, integrate=False)
  nc = int(out["ncon"][0, 0])
  assert nc == 4
  dist = out["contact_dist"][0, :nc]
  np.testing.assert_allclose(dist, -0.01, atol=1e-12)
  pos = out["contact_pos"][0, : 3 * nc].reshape(nc, 3)
  corners = {(round(abs(x), 9), round(abs(y), 9)) for x, y in pos[:, :2]}
  assert corners == {(0.2, 0.1)} and len({(np.sign(x), np.sign(y)) for x, y in pos[:, :2]}) == 4
  for i in range(nc):
    np.testing.assert_allclose(out["contact_frame"][0, 9 * i : 9 * i + 3], [0, 0, 1], atol=1e-12)


@pytest.mark.parametrize("tan_theta,slides", [(0.5, False), (0.8, True)])
def test_block_on_incline_stick_slip_threshold(tan_theta, slides):
  """A block on a plane with friction mu = 0.65 under gravity tilted by theta
  (equivalent to an incline): it sticks when tan(theta) < mu and slides with
  a = g (sin(theta) - mu cos(theta)) when tan(theta) > mu (pyramidal cone,
  condim 3)."""
  mu, g = 0.65, 9.81
  th = np.arctan(tan_theta)
  grav = f"{g * np.sin(th)} 0 {-g * np.cos(th)}"
  xml = _free_body_xml(
    f"""<body name="blk" pos="0 0 0.05"><freejoint/><geom type="box" size="0.1 0.1 0.05" mass="1" friction="{mu} 0.005 0.0001"/></body>""",
    gravity=grav, plane=f'<geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>')
  m = _model(xml)
  orc = Oracle(m)
  st = {"qpos": m.qpos0[None].copy()}
  vx = []
  for _ in range(500):  # 1 s
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    vx.append(st["qvel"][0, 0])
  if slides:
    a = (vx[-1] - vx[249]) / (250 * m.timestep)
    assert a == pytest.approx(g * (np.sin(th) - mu * np.cos(th)), rel=0.05)
  else:
    assert abs(vx[-1]) < 5e-3 and abs(st["qpos"][0, 0]) < 5e-3


def test_cg_and_newton_reach_the_same_minimiser():
  """CG (opt.solver = mjSOL_CG, Polak-Ribiere on the M-preconditioned
  gradient) and Newton minimise the same convex cost, so with the iteration cap
  lifted (float64 oracle, exact line search) both reach the same qacc; CG takes
  more iterations (first-order directions)."""
  from tests.scenes import random_states

  n = 16
  m = g1_scene_model(n)
  m.iterations, m.tolerance, m.ls_iterations, m.ls_parallel = 300, 1e-14, 50, 0
  st = random_states(m, n, np.random.default_rng(31))
  m.solver = 2
  newton = Oracle(m).run(n, st, integrate=False)
  m.solver = 1
  cg = Oracle(m).run(n, st, integrate=False)
  assert (newton["nefc"] > 0).mean() > 0.8
  scale = 1 + np.abs(newton["qacc"]).max(axis=1, keepdims=True)
  assert (np.abs(cg["qacc"] - newton["qacc"]) / scale).max() < 1e-6
  assert cg["solver_niter"].mean() > newton["solver_niter"].mean()


@pytest.mark.parametrize("tan_theta,slides", [(0.5, False), (0.8, True)])
def test_elliptic_cone_incline_stick_slip_threshold(tan_theta, slides):
  """The incline of test_block_on_incline_stick_slip_threshold with elliptic
  cones (opt.cone = mjCONE_ELLIPTIC, impratio 1: the regularised cone's
  mu = friction0): the same threshold tan(theta) = mu and sliding acceleration
  g (sin(theta) - mu cos(theta)); the rows are the contact frame's
  components (3 per contact instead of 4 pyramid edges)."""
  mu, g = 0.65, 9.81
  th = np.arctan(tan_theta)
  grav = f"{g * np.sin(th)} 0 {-g * np.cos(th)}"
  xml = _free_body_xml(
    f"""<body name="blk" pos="0 0 0.05"><freejoint/><geom type="box" size="0.1 0.1 0.05" mass="1" friction="{mu} 0.005 0.0001"/></body>""",
    gravity=grav, plane=f'<geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>')
  m = _model(xml, cone=1)
  orc = Oracle(m)
  st = {"qpos": m.qpos0[None].copy()}
  vx = []
  for i in range(500):  # 1 s
    out = orc.run(1, st, integrate=True)
    if i == 10:
      nc = int(out["ncon"][0, 0])
      assert nc == 4 and int(out["nefc"][0, 0]) == 3 * nc
      assert set(out["efc_type"][0, : 3 * nc].tolist()) == {7}
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    vx.append(st["qvel"][0, 0])
  if slides:
    a = (vx[-1] - vx[249]) / (250 * m.timestep)
    assert a == pytest.approx(g * (np.sin(th) - mu * np.cos(th)), rel=0.05)
  else:
    assert abs(vx[-1]) < 5e-3 and abs(st["qpos"][0, 0]) < 5e-3


@pytest.mark.parametrize("cone,factor", [(1, 1.0), (0, 2 ** -0.5)])
def test_diagonal_sliding_by_cone(cone, factor):
  """The incline of test_block_on_incline_stick_slip_threshold (tan(theta) =
  0.8 > mu = 0.65) tilted along the diagonal of the contact frame's tangents:
  an elliptic cone (the friction disc) resists the slide with mu N, the
  pyramidal cone, whose edges lie along the tangents (each direction's
  friction takes a share of the normal force), with mu N / sqrt(2) at most:
  a = g (sin(theta) - factor mu cos(theta)). The two cone types apart."""
  mu, g = 0.65, 9.81
  th = np.arctan(0.8)
  gt = g * np.sin(th) / np.sqrt(2)
  xml = _free_body_xml(
    f"""<body name="blk" pos="0 0 0.05"><freejoint/><geom type="box" size="0.1 0.1 0.05" mass="1" friction="{mu} 0.005 0.0001"/></body>""",
    gravity=f"{gt} {gt} {-g * np.cos(th)}",
    plane=f'<geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>')
  m = _model(xml, cone=cone)
  orc = Oracle(m)
  st = {"qpos": m.qpos0[None].copy()}
  sp = []
  for _ in range(500):  # 1 s
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    sp.append(np.hypot(st["qvel"][0, 0], st["qvel"][0, 1]))
  a = (sp[-1] - sp[249]) / (250 * m.timestep)
  assert a == pytest.approx(g * (np.sin(th) - factor * mu * np.cos(th)), rel=0.05)
  assert abs(st["qvel"][0, 0] - st["qvel"][0, 1]) < 1e-6  # stays on the diagonal


def test_elliptic_newton_converges_fast_and_matches_cg():
  """Elliptic cones on the G1 scene: Newton (with the cone's Hessian blocks)
  and CG reach the same qacc with the iteration cap lifted, Newton in few
  iterations (a wrong cone Hessian would still descend, but slowly)."""
  from tests.scenes import random_states

  n = 16
  m = g1_scene_model(n)
  m.cone = 1
  m.iterations, m.tolerance, m.ls_iterations, m.ls_parallel = 300, 1e-14, 50, 0
  st = random_states(m, n, np.random.default_rng(33))
  m.solver = 2
  newton = Oracle(m).run(n, st, integrate=False)
  m.solver = 1
  cg = Oracle(m).run(n, st, integrate=False)
  assert (newton["ncon"] > 0).mean() > 0.8
  types = {int(t) for w in range(n) for t in newton["efc_type"][w, : int(newton["nefc"][w, 0])]}
  assert 7 in types and 6 not in types
  scale = 1 + np.abs(newton["qacc"]).max(axis=1, keepdims=True)
  assert (np.abs(cg["qacc"] - newton["qacc"]) / scale).max() < 1e-6
  assert newton["solver_niter"].mean() < 20 < cg["solver_niter"].mean()


@pytest.mark.parametrize("scene", ["g1", "box"])
def test_pgs_newton_cg_reach_the_same_minimiser(scene):
  """PGS (opt.solver = mjSOL_PGS: projected Gauss-Seidel on the dual
  0.5 f'AR f + f'b) and Newton / CG (the primal) solve the same convex
  problem, so with the iteration caps lifted the three reach the same qacc
  (float64 oracle). PGS converges linearly: it needs far more iterations."""
  from tests.scenes import random_states

  if scene == "g1":
    n = 8
    m = g1_scene_model(n)
    st = random_states(m, n, np.random.default_rng(35))
  else:
    from tests.test_gpu_parity import BOX_SCENE, _box_states

    n = 16
    m = _model(BOX_SCENE)
    st = _box_states(m, n, np.random.default_rng(36))
  m.tolerance, m.ls_iterations, m.ls_parallel = 1e-15, 50, 0
  out = {}
  for solver, iters in (("newton", 200), ("cg", 3000), ("pgs", 20000)):
    m.solver, m.iterations = {"pgs": 0, "cg": 1, "newton": 2}[solver], iters
    out[solver] = Oracle(m).run(n, st, integrate=False)
  assert (out["newton"]["nefc"] > 0).mean() > 0.5
  scale = 1 + np.abs(out["newton"]["qacc"]).max(axis=1, keepdims=True)
  for s in ("cg", "pgs"):
    err = (np.abs(out[s]["qacc"] - out["newton"]["qacc"]) / scale).max()
    assert err < 1e-5, (s, err)
  # the dual solution's forces satisfy the projections: contact/limit rows >= 0
  f, ty = out["pgs"]["efc_force"], out["pgs"]["efc_type"]
  for w in range(n):
    k = int(out["pgs"]["nefc"][w, 0])
    assert (f[w, :k][ty[w, :k] != 1] >= 0).all()
  assert out["pgs"]["solver_niter"].mean() > out["newton"]["solver_niter"].mean()


def test_pgs_resting_penetration_and_incline_threshold():
  """PGS on the closed-form scenes: the condim-1 ball rests at MuJoCo's
  documented r* (tests/test_soft_constraint.py), and the incline block sticks
  below tan(theta) = mu and slides with a = g (sin - mu cos) above it."""
  from tests.test_soft_constraint import PARAMS, RAD, ball_model, rest_penetration, rollout

  solref, solimp = PARAMS["default"]
  m = ball_model(solref, solimp)
  m.solver, m.iterations, m.tolerance = 0, 200, 1e-14
  zs, _ = rollout(Oracle(m), RAD + 0.002, 0.0, 800)
  assert zs[-1] - RAD == pytest.approx(rest_penetration(solref, solimp, m.timestep), rel=1e-6)
  mu, g = 0.65, 9.81
  for tan_theta, slides in ((0.5, False), (0.8, True)):
    th = np.arctan(tan_theta)
    xml = _free_body_xml(
      f"""<body name="blk" pos="0 0 0.05"><freejoint/><geom type="box" size="0.1 0.1 0.05" mass="1" friction="{mu} 0.005 0.0001"/></body>""",
      gravity=f"{g * np.sin(th)} 0 {-g * np.cos(th)}",
      plane=f'<geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>')
    m = _model(xml, solver=0, iterations=100)
    orc = Oracle(m)
    st = {"qpos": m.qpos0[None].copy()}
    vx = []
    for _ in range(500):
      out = orc.run(1, st, integrate=True)
      st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
      vx.append(st["qvel"][0, 0])
    if slides:
      a = (vx[-1] - vx[249]) / (250 * m.timestep)
      assert a == pytest.approx(g * (np.sin(th) - mu * np.cos(th)), rel=0.05)
    else:
      assert abs(vx[-1]) < 5e-3 and abs(st["qpos"][0, 0]) < 5e-3
