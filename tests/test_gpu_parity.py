"""HIP step (through the C-ABI) vs the float64 oracle, and size-independent
properties at the benchmark size. Tolerances: tests/scenes.py docstring."""

import numpy as np
import pytest
import torch

from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
from oracle.oracle import INPUTS, Oracle
from tests.scenes import check_iteration_counts, compare_step, g1_mocap_scene, g1_scene_model, g1_sensor_scene, go1_scene_model, mocap_states, random_states

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CFG = dict(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.005, iterations=10, ls_iterations=20))
MODELS = {"g1": g1_scene_model, "go1": go1_scene_model}


def make_sim(m, n, expand=(), ls_parallel=True):
  sim = Simulation(n, SimulationCfg(**CFG, ls_parallel=ls_parallel), m, DEV)
  if expand:
    sim.expand_model_fields(tuple(expand))
  return sim


def put(sim, st):
  for k, v in st.items():
    t = getattr(sim.data, k)
    t.copy_(torch.as_tensor(np.asarray(v), dtype=t.dtype, device=DEV).view_as(t))


def get(sim, n):
  torch.cuda.synchronize()
  return {k: getattr(sim.data, k).detach().cpu().numpy().reshape(n, -1) for k in sim.data.fields()}


LIFTED_ITERATIONS = 100


def recheck_capped(m, state, worlds, ls_parallel=True, integrate=True, cfg=None, overrides=None):
  """The worlds a comparison held to the soft bound because the solver stopped
  at the iteration cap (tests/scenes.py: unconverged, so a float32 and a float64
  iterate drift apart) are solved again from the same state with the cap lifted
  (LIFTED_ITERATIONS), device against the oracle (follow mode), and now held to
  every hard bound; both must converge. A world that passes is no longer an
  unverified exemption (the PARITY summary's capped_unverified)."""
  import copy

  from tests.scenes import PARITY_LOG

  worlds = [int(w) for w in worlds]
  k = len(worlds)
  mc = copy.deepcopy(m)
  base = dict(cfg or CFG)
  mj = copy.deepcopy(base["mujoco"])
  mj.iterations = LIFTED_ITERATIONS
  base["mujoco"] = mj
  sim = Simulation(k, SimulationCfg(**base, ls_parallel=ls_parallel), mc, DEV)
  sub_over = None
  if overrides:
    sub_over = {name: np.asarray(a)[worlds] for name, a in overrides.items()}
    sim.expand_model_fields(tuple(sub_over))
    for name, a in sub_over.items():
      t = getattr(sim.model, name)
      t.copy_(torch.as_tensor(a, dtype=t.dtype, device=DEV).view_as(t))
  sub = {f: np.asarray(v)[worlds] for f, v in state.items()}
  put(sim, sub)
  sim.step() if integrate else sim.forward()
  got = get(sim, k)
  ref = Oracle(mc, overrides=sub_over).run(k, sub, integrate=integrate, follow=got if ls_parallel else None)
  rep = compare_step(got, ref, cap_exempt=False)
  PARITY_LOG.pop()  # the re-run is recorded on the original comparison's entry
  conv = got["solver_niter"][:, 0] < LIFTED_ITERATIONS
  assert not rep["failures"] and conv.all(), ("capped worlds re-run with the cap lifted", worlds, rep["failures"],
                                              got["solver_niter"][:, 0])
  PARITY_LOG[-1]["capped_verified"] = k
  return k


def assert_parity(got, ref, n, min_int_rate=0.98, tag="", recheck=None):
  """compare_step must report no failure (every integer mismatch explained by
  a borderline contact/row; floats within tests/scenes.py tolerances), and at
  least `min_int_rate` of the worlds must have bit-identical integer outputs.
  recheck (model, state and the run's options): the capped worlds are solved
  again with the iteration cap lifted and held to the hard bounds."""
  rep = compare_step(got, ref)
  print(f"[parity{tag}] int_match_rate={rep['int_match_rate']:.4f} mismatches={rep['int_mismatch_reasons']} "
        f"maxerr={ {k: f'{v:.2e}' for k, v in rep['maxerr'].items()} }")
  assert not rep["failures"], (rep["failures"], rep["maxerr"])
  assert rep["int_match_rate"] >= min_int_rate, rep["int_mismatch_reasons"]
  capped = [w for w in rep["capped_worlds"] if w not in rep["int_mismatch_reasons"]]
  if recheck is not None and capped:
    recheck_capped(worlds=capped, **recheck)
  return rep


@pytest.mark.parametrize("name", ["g1", "go1"])
@pytest.mark.parametrize("integrate", [True, False])
@pytest.mark.parametrize("ls_parallel", [True, False])
def test_single_step_parity(name, integrate, ls_parallel):
  """Both line searches (SimulationCfg.ls_parallel: MuJoCo Warp's parallel
  search, the reference default, and the exact 1-D Newton search) against the
  oracle running the same one, at the capped iteration count."""
  n = 256
  m = MODELS[name](n)
  st = random_states(m, n, np.random.default_rng(1))
  sim = make_sim(m, n, ls_parallel=ls_parallel)
  assert m.ls_parallel == int(ls_parallel)  # the oracle reads the same model option
  put(sim, st)
  sim.step() if integrate else sim.forward()
  got = get(sim, n)
  got.update({k: v.cpu().numpy().reshape(n, -1) for k, v in sim.debug_fields().items()})
  ref = Oracle(m).run(n, st, integrate=integrate, debug=True, follow=got)
  rep = assert_parity(got, ref, n, tag=f" {name} integrate={integrate}",
                      recheck=dict(m=m, state=st, ls_parallel=ls_parallel, integrate=integrate))
  assert "qM" in rep["maxerr"] and "efc_J" in rep["maxerr"]  # the debug copies were compared
  assert (got["ncon"] > 0).mean() > 0.5  # the states exercise contacts
  it = check_iteration_counts(got, m, st, integrate)
  print(f"[iterations {name}] {it}")
  assert it["ok"], it  # no systematic early stop against the float32 oracle's own test


def test_trajectory_parity_along_gpu_rollout():
  """At every step of a 40-step GPU rollout (warm starts, evolving contacts),
  one oracle step from the GPU's state must match the GPU's next state."""
  n = 64
  m = g1_scene_model(n)
  sim = make_sim(m, n)
  st = random_states(m, n, np.random.default_rng(2), drop=0.03)
  put(sim, st)
  orc = Oracle(m)
  worst = worst32 = 0.0
  for k in range(40):
    cur = get(sim, n)
    state = {f: cur[f] for f in INPUTS if f in cur}
    sim.step()
    nxt = get(sim, n)
    ref = orc.run(n, state, integrate=True, follow=nxt)
    rep = assert_parity(nxt, ref, n, min_int_rate=0.95, tag=f" step {k}", recheck=dict(m=m, state=state))
    worst = max(worst, rep["maxerr"]["qvel"])
    worst32 = max(worst32, float(np.abs(ref["f32"]["qvel"] - ref["qvel"]).max()))
  # 0.05 m/s, or the float32 oracle's own deviation along the same choices (x4,
  # tests/scenes.py F32_SENSITIVITY) where stiff contacts make that larger
  assert worst < max(0.05, 4.0 * worst32), (worst, worst32)


def test_per_world_randomized_friction():
  n = 128
  m = g1_scene_model(n)
  sim = make_sim(m, n, expand=("geom_friction",))
  rng = np.random.default_rng(3)
  fr = sim.model.geom_friction
  fr[:, :, 0] = torch.as_tensor(rng.uniform(0.3, 1.2, (n, fr.shape[1])), dtype=torch.float32, device=DEV)
  st = random_states(m, n, rng)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m, overrides={"geom_friction": fr.cpu().numpy()}).run(n, st, integrate=True, follow=got)
  assert_parity(got, ref, n, recheck=dict(m=m, state=st, overrides={"geom_friction": fr.cpu().numpy()}))


def test_gated_forward():
  n = 32
  m = g1_scene_model(n)
  sim = make_sim(m, n)
  st = random_states(m, n, np.random.default_rng(4))
  put(sim, st)
  sim.forward()
  a = get(sim, n)
  put(sim, random_states(m, n, np.random.default_rng(5)))
  sim.forward_gated(torch.zeros(1, dtype=torch.bool, device=DEV))
  b = get(sim, n)
  for k in ("xpos", "qacc", "sensordata", "efc_force"):
    assert np.array_equal(a[k], b[k]), k  # gate 0: nothing recomputed
  # forward saves qacc into qacc_warmstart (as MuJoCo's solver does), so
  # restore the warm start before each call being compared
  ws = sim.data.qacc_warmstart.clone()
  sim.forward_gated(torch.ones(1, dtype=torch.bool, device=DEV))
  c = get(sim, n)
  sim.data.qacc_warmstart.copy_(ws)
  sim.forward()
  d = get(sim, n)
  for k in ("xpos", "qacc", "sensordata"):
    assert np.array_equal(c[k], d[k]), k


def test_overflow_is_flagged_not_fatal():
  """Contacts beyond a world's slots (max(nconmax, njmax) = 16 here) are dropped
  and flagged; the step stays finite."""
  n = 16
  m = g1_scene_model(n, nconmax=4, njmax=16)
  sim = Simulation(n, SimulationCfg(**dict(CFG, nconmax=4, njmax=16)), m, DEV)
  assert m.nconmax == 16 and m.ncon_share == 4
  st = random_states(m, n, np.random.default_rng(6), drop=0.06)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  assert (got["ncon"] <= 16).all()
  assert ((got["flags"] & 1) != 0).any()
  assert np.isfinite(got["qvel"]).all()
  # surfaced without a sync: sticky flags (OR over launches) counted and
  # cleared on the device by flag_stats
  assert np.array_equal(got["flags_acc"] & got["flags"], got["flags"])
  sim.step()
  f2 = sim.data.flags.clone()
  acc = sim.data.flags_acc.clone()
  assert torch.equal(acc & f2, f2)
  n_or = int(((acc & 1) != 0).sum())
  st = sim.flag_stats().cpu().numpy()
  assert st[0] == n_or and st[3] == n_or and n_or > 0
  assert int(sim.data.flags_acc.abs().sum()) == 0
  st = sim.flag_stats().cpu().numpy()
  assert st[0] == 0 and st[3] == n_or  # running total kept


def test_pooled_contacts_one_world_exceeds_nconmax():
  """SimulationCfg.nconmax sizes a pool shared by the worlds, as the
  reference's ("one world may have more than nconmax contacts",
  /root/reference/src/mjlab/sim/sim.py:81-85): with nconmax 2 and njmax 32 a
  world keeps up to max(2, 32) = 32 contacts, so the G1 worlds lying on the
  floor keep all of theirs (as an uncapped float64 oracle run finds them,
  up to 28) while the airborne ones hold none, and nothing is flagged."""
  n = 8
  m = g1_scene_model(n, nconmax=2, njmax=32)
  st = random_states(m, n, np.random.default_rng(6), drop=0.06)
  full = Oracle(g1_scene_model(n, nconmax=64, njmax=300)).run(n, st, integrate=False)["ncon"][:, 0]
  sim = Simulation(n, SimulationCfg(**dict(CFG, nconmax=2, njmax=32)), m, DEV)
  assert m.nconmax == 32 and m.ncon_share == 2
  put(sim, st)
  sim.forward()
  got = get(sim, n)
  np.testing.assert_array_equal(got["ncon"][:, 0], full)
  assert (full > 2).sum() >= 3 and (full <= 2).any()  # some worlds above their share, some below
  assert ((got["flags"][:, 0] & 1) == 0).all()


def test_full_size_determinism_and_world_independence():
  """N=4096 (the bench size): two runs from one state are bitwise equal, and
  permuting the worlds permutes every output bitwise (no cross-world coupling)."""
  n = 4096
  m = g1_scene_model(n)
  sim = make_sim(m, n)
  st = random_states(m, n, np.random.default_rng(7))
  put(sim, st)
  for _ in range(3):
    sim.step()
  base = {k: getattr(sim.data, k).clone() for k in ("qpos", "qvel", "qacc_warmstart", "ctrl", "time")}
  sim.step()
  a = get(sim, n)
  for k, v in base.items():
    getattr(sim.data, k).copy_(v)
  sim.step()
  b = get(sim, n)
  for k in ("qpos", "qvel", "qacc", "sensordata", "efc_force", "ncon"):
    assert np.array_equal(a[k], b[k]), k
  assert np.isfinite(a["qpos"]).all() and (a["flags"] & 4 == 0).all()
  perm = torch.randperm(n, generator=torch.Generator().manual_seed(0))
  for k, v in base.items():
    getattr(sim.data, k).copy_(v[perm.to(DEV)])
  sim.step()
  c = get(sim, n)
  p = perm.numpy()
  for k in ("qpos", "qvel", "qacc", "sensordata", "ncon"):
    assert np.array_equal(c[k], a[k][p]), k


def test_full_size_integer_parity_rate():
  """N=4096 (the bench size), one step from random stance states against the
  float64 oracle: >= 99.9 % of worlds have bit-identical integer outputs
  (contacts, rows), every mismatch is borderline, and every float check holds."""
  n = 4096
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(11))
  sim = make_sim(m, n)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, nthreads=8, follow=got)
  assert_parity(got, ref, n, min_int_rate=0.999, tag=" N=4096", recheck=dict(m=m, state=st))


def test_contact_sensor_reductions_and_fields():
  """maxforce / mindist (top-k, stable), netforce (net wrench at the
  force-weighted centroid) and none, with found/force/torque/dist/pos/normal/
  tangent, against the oracle (oracle/oracle.c sensors())."""
  n = 256
  m = g1_sensor_scene(n).compile(50, 300)
  st = random_states(m, n, np.random.default_rng(12))
  sim = make_sim(m, n)
  put(sim, st)
  sim.forward()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=False, follow=got)
  rep = assert_parity(got, ref, n, tag=" sensors")
  good = np.array([w for w in range(n) if w not in rep["int_mismatch_reasons"]])
  sd_g, sd_r = got["sensordata"][good], ref["sensordata"][good]
  assert (np.abs(sd_r) > 0).sum(axis=0).min() >= 0  # shape sanity
  assert np.abs(sd_g - sd_r).max() <= 2e-3 * (1 + np.abs(sd_r).max())
  assert (sd_r != 0).any(axis=0).mean() > 0.5  # most sensor entries are exercised


def test_converged_solver_parity():
  """With the iteration cap lifted (iterations 100, tolerance 1e-10) the HIP
  Newton solver and the float64 oracle converge to the same qacc in EVERY
  world (the capped comparisons differ only in where each stops)."""
  n = 512
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(11))
  # the exact line search: the parallel one's discrete steps may stop short of
  # a 1e-10 tolerance on either side (its parity is checked in follow mode)
  cfg = dict(CFG, mujoco=MujocoCfg(timestep=0.005, iterations=100, ls_iterations=50, tolerance=1e-10))
  sim = Simulation(n, SimulationCfg(**cfg, ls_parallel=False), m, DEV)
  put(sim, st)
  sim.forward()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=False)
  # float32 round-off at convergence: measured max 1.4e-5 (qacc), 2.7e-5
  # (qfrc_constraint), 2.2e-5 (sensordata) relative; bound 1e-4 for every world
  rep = compare_step(got, ref, solve_rel=1e-4, solve_frac=1.0, solve_max=1e-4)
  print("[converged]", rep["int_match_rate"], {k: f"{v:.2e}" for k, v in rep["maxerr"].items() if "/" in k})
  assert not rep["failures"], rep["failures"]


def test_converged_solver_parity_parallel_search():
  """The reference default (ls_parallel=True, sim.py:91,117) without follow
  mode: each side takes its own step-size choices, and with the iteration cap
  lifted (iterations 100, tolerance 1e-10) both reach the same qacc in every
  world — the minimiser does not depend on the path."""
  n = 512
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(13))
  cfg = dict(CFG, mujoco=MujocoCfg(timestep=0.005, iterations=100, ls_iterations=20, tolerance=1e-10))
  sim = Simulation(n, SimulationCfg(**cfg, ls_parallel=True), m, DEV)
  assert m.ls_parallel == 1
  put(sim, st)
  sim.forward()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=False)  # no follow: the oracle's own choices
  # the float32 oracle's own converged solve (its own choices and stop): each
  # world's float32 resolution, the per-world floor of the bounds (F32_SENSITIVITY)
  ref["f32"] = Oracle(m, "f32").run(n, st, integrate=False)
  # 3e-4 rather than the exact search's 1e-4: at tolerance 1e-10 the float32
  # stop sits in noise, and a stiff world stops a little short of the float32
  # oracle (measured: 1.8e-4 relative in sensordata, world 271 of seed 13, 112
  # rows, device 7 iterations / float32 oracle 8 / float64 7)
  rep = compare_step(got, ref, solve_rel=3e-4, solve_frac=1.0, solve_max=3e-4)
  print("[converged parallel]", rep["int_match_rate"], {k: f"{v:.2e}" for k, v in rep["maxerr"].items() if "/" in k},
        "niter_differs", rep["decisions"].get("niter_differs"))
  for k in ("sensordata", "qacc", "qfrc_constraint"):
    d = np.abs(got[k] - ref[k]).max(axis=1)
    w = int(np.argmax(d))
    j = int(np.argmax(np.abs(got[k][w] - ref[k][w])))
    print(f"  worst {k}: world {w} entry {j} device {got[k][w, j]:.6e} f64 {ref[k][w, j]:.6e} f32 {ref['f32'][k][w, j]:.6e} "
          f"niter device/f32/f64 {int(got['solver_niter'][w, 0])}/{int(ref['f32']['solver_niter'][w, 0])}/"
          f"{int(ref['solver_niter'][w, 0])} nefc {int(ref['nefc'][w, 0])} max|ref| {np.abs(ref[k][w]).max():.3e}")
  assert not rep["failures"], rep["failures"]


def test_known_answers_on_gpu():
  """The analytic known answers that pin the oracle (test_oracle_known_answers)
  hold for the HIP step too: crossed capsules, box corners on a plane, and the
  incline stick/slip threshold (float32 tolerances)."""
  from tests import test_oracle_known_answers as KA

  def sim_of(xml, n=1):
    m = KA._model(xml)
    # MujocoCfg.apply sets the model's options (sim.py:42-94), gravity included
    opt = MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20, gravity=tuple(float(x) for x in m.gravity))
    sim = Simulation(n, SimulationCfg(nconmax=16, njmax=64, mujoco=opt), m, DEV)
    put(sim, {"qpos": np.tile(m.qpos0[None], (n, 1))})
    return m, sim

  m, sim = sim_of(KA._free_body_xml("""
    <body name="a" pos="0 0 0.5"><freejoint/><geom type="capsule" fromto="-0.3 0 0 0.3 0 0" size="0.05"/></body>
    <body name="b" pos="0.1 0.05 0.58"><freejoint/><geom type="capsule" fromto="0 -0.3 0 0 0.3 0" size="0.05"/></body>
  """, gravity="0 0 0"))
  sim.forward()
  o = get(sim, 1)
  assert o["ncon"][0, 0] == 1
  assert o["contact_dist"][0, 0] == pytest.approx(-0.02, abs=1e-6)
  np.testing.assert_allclose(o["contact_pos"][0, 0:3], [0.1, 0.0, 0.54], atol=1e-6)

  m, sim = sim_of(KA._free_body_xml("""<body name="box" pos="0 0 0.04"><freejoint/><geom type="box" size="0.2 0.1 0.05"/></body>""",
                                    plane='<geom name="floor" type="plane" size="5 5 0.1"/>'))
  sim.forward()
  o = get(sim, 1)
  assert o["ncon"][0, 0] == 4
  np.testing.assert_allclose(o["contact_dist"][0, :4], -0.01, atol=1e-6)
  np.testing.assert_allclose(np.abs(o["contact_pos"][0, :12].reshape(4, 3)[:, :2]), [[0.2, 0.1]] * 4, atol=1e-6)

  mu, g = 0.65, 9.81
  for tan_theta, slides in ((0.5, False), (0.8, True)):
    th = np.arctan(tan_theta)
    m, sim = sim_of(KA._free_body_xml(
      f"""<body name="blk" pos="0 0 0.05"><freejoint/><geom type="box" size="0.1 0.1 0.05" mass="1" friction="{mu} 0.005 0.0001"/></body>""",
      gravity=f"{g * np.sin(th)} 0 {-g * np.cos(th)}",
      plane=f'<geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>'))
    vx = []
    for _ in range(500):
      sim.step()
      vx.append(sim.data.qvel[0, 0].item())
    if slides:
      a = (vx[-1] - vx[249]) / (250 * m.timestep)
      assert a == pytest.approx(g * (np.sin(th) - mu * np.cos(th)), rel=0.05)
    else:
      assert abs(vx[-1]) < 5e-3 and abs(sim.data.qpos[0, 0].item()) < 5e-3


@pytest.mark.parametrize("integrate", [True, False])
def test_mocap_body_parity(integrate):
  """A mocap sphere (pose from mocap_pos / unnormalised mocap_quat) moved into
  the robot: kinematics, contacts and the solve against the oracle."""
  n = 256
  m = g1_mocap_scene(n).compile(50, 300)
  st = mocap_states(m, n, np.random.default_rng(5))
  sim = make_sim(m, n)
  put(sim, st)
  sim.step() if integrate else sim.forward()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=integrate, follow=got)
  assert_parity(got, ref, n, tag=f" mocap integrate={integrate}", recheck=dict(m=m, state=st, integrate=integrate))
  b = int(np.nonzero(m.body_mocapid >= 0)[0][0])
  np.testing.assert_allclose(got["xpos"].reshape(n, -1, 3)[:, b], st["mocap_pos"][:, :3], atol=1e-6)
  g = [i for i in range(m.ngeom) if m.geom_bodyid[i] == b][0]
  hits = (got["contact_geom"].reshape(n, -1) == g).any(1).mean()
  assert hits > 0.05, hits  # the ball touches the robot in a fair share of worlds


def test_rows_in_global_scratch_are_bit_identical():
  """Worlds whose constraint rows exceed the LDS-resident capacity run the rest
  of their step with the row arrays in global scratch (mjh_step.hip, BIG): the
  same arithmetic on other addresses. With the LDS capacity capped at 8 rows
  (most worlds take that path) every output is bitwise equal to a run capped one
  row below the LDS budget's capacity (few worlds do; both caps change the
  launch plan, so both runs use the generic kernel instance), and both match
  the oracle."""
  from mjlab_amd.sim import native

  n = 256
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(21), drop=0.03)
  outs = []
  lcap = make_sim(m, 8).lds_row_capacity()  # the LDS budget's rows (uncapped)
  try:
    # both caps change the launch plan (generic instance in both runs)
    for cap in (8, lcap - 1):
      native.lib().mjh_set_lds_row_cap(cap)
      sim = make_sim(m, n)
      assert sim.lds_row_capacity() == cap
      put(sim, st)
      sim.step()
      outs.append(get(sim, n))
  finally:
    native.lib().mjh_set_lds_row_cap(0)
  a, b = outs
  assert (a["nefc"] > 8).mean() > 0.5  # most worlds took the global-scratch path
  diffs = {}
  for k in ("qpos", "qvel", "qacc", "qfrc_constraint", "efc_force", "efc_D", "efc_aref", "sensordata", "nefc", "solver_niter",
            "solver_lstrace"):
    d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64)).max(axis=1)
    if (d > 0).any():
      diffs[k] = (int((d > 0).sum()), float(d.max()), [int(w) for w in np.nonzero(d)[0][:6]])
  print("[rows in global scratch] differing fields (worlds, max |d|, first worlds):", diffs)
  assert not diffs, diffs
  ref = Oracle(m).run(n, st, integrate=True, follow=a)
  assert_parity(a, ref, n)


@pytest.mark.parametrize("iterations", [1, 3])
@pytest.mark.parametrize("ls_parallel", [True, False])
def test_cg_solver_parity(ls_parallel, iterations):
  """opt.solver = CG (the reference's own test pipes solver="cg",
  test_sim.py:43-82; MuJoCo Warp implements it): Polak-Ribiere directions from
  M's factor, the same line searches and stop test as Newton, against the
  oracle running CG (follow mode for the parallel search). A few iterations
  (1: the first direction -M^-1 grad; 3: two Polak-Ribiere updates): CG's
  recurrence amplifies round-off, so an unconverged float32 CG and a float64
  one drift apart within tens of iterations even on the same choices (the
  float32 and float64 oracle CG differ by up to 5e-2 relative in qacc after
  50; Newton by 1e-5). That CG reaches the minimiser is the float64 oracle's
  known answer (tests/test_oracle_known_answers.py)."""
  n = 256
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(41))
  cfg = dict(CFG, mujoco=MujocoCfg(timestep=0.005, iterations=iterations, ls_iterations=20, solver="cg"))
  sim = Simulation(n, SimulationCfg(**cfg, ls_parallel=ls_parallel), m, DEV)
  assert m.solver == 1 and m.ls_parallel == int(ls_parallel)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, follow=got if ls_parallel else None)
  # capped by construction (a few iterations), and held to every hard bound: over
  # 1-3 iterations float32 and float64 CG stay together along the same choices
  rep = compare_step(got, ref, cap_exempt=False)
  print(f"[cg iterations={iterations}]", {k: f"{v:.2e}" for k, v in rep["maxerr"].items() if "/" in k})
  assert not rep["failures"], rep["failures"]


BOX_SCENE = """<mujoco><compiler angle="radian"/><option timestep="0.002"/><worldbody>
<geom name="table" type="box" size="0.5 0.5 0.1"/>
<body name="cube" pos="0 0 0.3"><freejoint/><geom type="box" size="0.1 0.08 0.06" mass="1.5"/></body>
<body name="ball" pos="0.2 0 0.3"><freejoint/><geom type="sphere" size="0.07" mass="0.5"/></body>
<body name="pill" pos="-0.2 0 0.3"><freejoint/><geom type="capsule" size="0.04 0.12" mass="0.7"/></body>
</worldbody></mujoco>"""


def _box_states(m, n, rng):
  q = np.zeros((n, m.nq))
  for b in range(3):
    q[:, 7 * b : 7 * b + 3] = rng.uniform([-0.45, -0.45, 0.1], [0.45, 0.45, 0.3], (n, 3))
    quat = rng.normal(size=(n, 4))
    q[:, 7 * b + 3 : 7 * b + 7] = quat / np.linalg.norm(quat, axis=1, keepdims=True)
  return {"qpos": q, "qvel": rng.normal(scale=0.3, size=(n, m.nv)), "qacc_warmstart": np.zeros((n, m.nv))}


def test_box_pairs_parity():
  """sphere-box, capsule-box and box-box (and box-on-box stacks) on the HIP
  step against the oracle's algorithms: random poses of a cube, a ball and a
  capsule over a static table box, one step, tests/scenes.py tolerances."""
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string

  n = 512
  m = compile_spec(read_mjcf_string(BOX_SCENE), 50, 300)
  assert m.nboxpair > 0
  st = _box_states(m, n, np.random.default_rng(51))
  sim = Simulation(n, SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.002, iterations=20,
                                                                               ls_iterations=20)), m, DEV)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, follow=got)
  rep = assert_parity(got, ref, n, min_int_rate=0.95, tag=" box pairs")
  g = got["contact_geom"].reshape(n, -1, 2)
  types = np.asarray(m.geom_type)
  kinds = {(int(types[a]), int(types[b])) for w in range(n) for a, b in g[w, : int(got["ncon"][w, 0])]}
  assert {(2, 6), (3, 6), (6, 6)} <= kinds, kinds  # every box pair was exercised
  print("[box pairs] contact kinds", sorted(kinds), "int rate", rep["int_match_rate"])


def test_box_on_box_carries_its_weight_on_gpu():
  """A 2 kg cube dropped onto a static box settles; the vertical constraint
  force on its free joint carries m g (HIP step, 400 steps of 2 ms)."""
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string

  xml = """<mujoco><option timestep="0.002"/><worldbody><geom type="box" size="0.5 0.5 0.1"/>
  <body name="b" pos="0 0 0"><freejoint/><geom type="box" size="0.1 0.1 0.1" mass="2"/></body></worldbody></mujoco>"""
  m = compile_spec(read_mjcf_string(xml), 8, 64)
  sim = Simulation(4, SimulationCfg(nconmax=8, njmax=64, mujoco=MujocoCfg(timestep=0.002, iterations=20)), m, DEV)
  put(sim, {"qpos": np.tile([0.05, -0.1, 0.205, 1, 0, 0, 0], (4, 1))})
  fz = []
  for _ in range(400):
    sim.step()
    fz.append(sim.data.qfrc_constraint[:, 2].clone())
  fz = torch.stack(fz).cpu().numpy()
  assert np.allclose(fz[-100:].mean(axis=0), 2.0 * 9.81, rtol=0.01)
  q = sim.data.qpos.cpu().numpy()
  assert np.abs(q[:, 2] - 0.2).max() < 2e-3


@pytest.mark.parametrize("ls_parallel", [True, False])
def test_elliptic_cone_parity(ls_parallel):
  """MujocoCfg(cone="elliptic") (reference sim.py:25-28,51 maps it to
  mjCONE_ELLIPTIC; MuJoCo Warp solves it): one row per contact dimension, the
  cone cost per contact, its Hessian block as virtual rows (csrc/mjh_step.hip
  cone_eval / newton_direction), against the oracle's elliptic restatement
  (oracle.c cone_eval: the block formed directly), both line searches, the
  capped iteration count (follow mode for the parallel search)."""
  n = 256
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(61))
  cfg = dict(CFG, mujoco=MujocoCfg(timestep=0.005, iterations=10, ls_iterations=20, cone="elliptic"))
  sim = Simulation(n, SimulationCfg(**cfg, ls_parallel=ls_parallel), m, DEV)
  assert m.cone == 1
  put(sim, st)
  sim.step()
  got = get(sim, n)
  types = {int(t) for w in range(n) for t in got["efc_type"][w, : int(got["nefc"][w, 0])]}
  assert 7 in types and 6 not in types, types
  ref = Oracle(m).run(n, st, integrate=True, follow=got if ls_parallel else None)
  assert_parity(got, ref, n, tag=f" elliptic ls_parallel={ls_parallel}",
                recheck=dict(m=m, state=st, ls_parallel=ls_parallel, cfg=cfg))


def test_elliptic_cone_converged_parity():
  """Elliptic cones with the iteration cap lifted (exact line search,
  iterations 100, tolerance 1e-10): the HIP solve and the float64 oracle reach
  the same qacc in every world (the cone Hessian only shapes the path)."""
  n = 256
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(63))
  cfg = dict(CFG, mujoco=MujocoCfg(timestep=0.005, iterations=100, ls_iterations=50, tolerance=1e-10, cone="elliptic"))
  sim = Simulation(n, SimulationCfg(**cfg, ls_parallel=False), m, DEV)
  put(sim, st)
  sim.forward()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=False)
  rep = compare_step(got, ref, solve_rel=1e-4, solve_frac=1.0, solve_max=1e-4)
  print("[elliptic converged]", rep["int_match_rate"], {k: f"{v:.2e}" for k, v in rep["maxerr"].items() if "/" in k},
        "niter", got["solver_niter"].mean(), ref["solver_niter"].mean())
  assert not rep["failures"], rep["failures"]


@pytest.mark.parametrize("cone,factor", [("elliptic", 1.0), ("pyramidal", 2 ** -0.5)])
def test_diagonal_sliding_by_cone_on_gpu(cone, factor):
  """tests/test_oracle_known_answers.py::test_diagonal_sliding_by_cone on the
  HIP step: a block on an incline (tan 0.8 > mu 0.65) tilted along the
  frame's tangent diagonal slides with a = g (sin - factor mu cos), factor 1
  for the elliptic cone and 1/sqrt(2) for the pyramidal one."""
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string

  mu, g = 0.65, 9.81
  th = np.arctan(0.8)
  gt = g * np.sin(th) / np.sqrt(2)
  xml = f"""<mujoco><option timestep="0.002" gravity="{gt} {gt} {-g * np.cos(th)}"/><worldbody>
  <geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>
  <body name="blk" pos="0 0 0.05"><freejoint/><geom type="box" size="0.1 0.1 0.05" mass="1" friction="{mu} 0.005 0.0001"/></body>
  </worldbody></mujoco>"""
  m = compile_spec(read_mjcf_string(xml), 8, 64)
  # MujocoCfg.apply sets the gravity (as the reference's does), so the tilt goes there
  sim = Simulation(2, SimulationCfg(nconmax=8, njmax=64, mujoco=MujocoCfg(timestep=0.002, iterations=20, cone=cone,
                                                                           gravity=(gt, gt, -g * np.cos(th)))), m, DEV)
  sp = []
  for _ in range(500):
    sim.step()
    v = sim.data.qvel[0, :2].cpu().numpy()
    sp.append(float(np.hypot(v[0], v[1])))
  a = (sp[-1] - sp[249]) / (250 * 0.002)
  assert a == pytest.approx(g * (np.sin(th) - factor * mu * np.cos(th)), rel=0.05)


CYL_SCENE = """<mujoco><compiler angle="radian"/><option timestep="0.002"/><worldbody>
<geom name="floor" type="plane" size="5 5 0.1" contype="1" conaffinity="1"/>
<geom name="post" type="cylinder" size="0.08 0.25" pos="0.3 0 0.25" contype="0" conaffinity="2"/>
<body name="can" pos="0 0 0.3"><freejoint/><geom type="cylinder" size="0.1 0.15" mass="1.2" contype="1" conaffinity="2"/></body>
<body name="egg" pos="-0.3 0 0.3"><freejoint/><geom type="ellipsoid" size="0.15 0.1 0.07" mass="0.8" contype="1" conaffinity="4"/></body>
<body name="ball" pos="0.2 0.2 0.3"><freejoint/><geom type="sphere" size="0.07" mass="0.5" contype="2" conaffinity="0"/></body>
</worldbody></mujoco>"""


def test_cylinder_ellipsoid_pairs_parity():
  """plane-cylinder, plane-ellipsoid and sphere-cylinder (against a moving
  and a static cylinder) on the HIP step against the oracle: random poses,
  one step, tests/scenes.py tolerances."""
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string

  n = 512
  m = compile_spec(read_mjcf_string(CYL_SCENE), 50, 300)
  assert m.nboxpair > 0 and not m.unsupported_pair_types
  rng = np.random.default_rng(53)
  q = np.zeros((n, m.nq))
  for b, (lo, hi) in enumerate([([-0.3, -0.3, -0.05], [0.3, 0.3, 0.2]), ([-0.4, -0.3, -0.05], [0.0, 0.3, 0.15]),
                                ([0.05, -0.3, -0.1], [0.55, 0.3, 0.6])]):
    q[:, 7 * b : 7 * b + 3] = rng.uniform(lo, hi, (n, 3))
    quat = rng.normal(size=(n, 4))
    q[:, 7 * b + 3 : 7 * b + 7] = quat / np.linalg.norm(quat, axis=1, keepdims=True)
  st = {"qpos": q, "qvel": rng.normal(scale=0.3, size=(n, m.nv)), "qacc_warmstart": np.zeros((n, m.nv))}
  sim = Simulation(n, SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.002, iterations=20,
                                                                               ls_iterations=20)), m, DEV)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, follow=got)
  rep = assert_parity(got, ref, n, min_int_rate=0.95, tag=" cylinder/ellipsoid pairs")
  g = got["contact_geom"].reshape(n, -1, 2)
  types = np.asarray(m.geom_type)
  kinds = {(int(types[a]), int(types[b])) for w in range(n) for a, b in g[w, : int(got["ncon"][w, 0])]}
  assert {(0, 4), (0, 5), (2, 5)} <= kinds, kinds
  print("[cylinder/ellipsoid pairs] contact kinds", sorted(kinds), "int rate", rep["int_match_rate"])


CONVEX_SCENE = """<mujoco><option timestep="0.002"/><worldbody>
<geom name="floor" type="plane" size="5 5 0.1"/>
<geom name="table" type="box" size="0.3 0.3 0.05" pos="0 0 0.05"/>
<geom name="post" type="cylinder" size="0.06 0.2" pos="0.3 0 0.2"/>
<body name="egg" pos="0 0 0.3"><freejoint/><geom type="ellipsoid" size="0.1 0.07 0.05" mass="0.8"/></body>
<body name="can" pos="0.1 0 0.3"><freejoint/><geom type="cylinder" size="0.06 0.1" mass="1.0"/></body>
<body name="pill" pos="-0.1 0 0.3"><freejoint/><geom type="capsule" size="0.04 0.08" mass="0.5"/></body>
<body name="ball" pos="0 0.1 0.3"><freejoint/><geom type="sphere" size="0.05" mass="0.4"/></body>
<body name="egg2" pos="0 -0.1 0.3"><freejoint/><geom type="ellipsoid" size="0.08 0.06 0.06" mass="0.6"/></body>
<body name="can2" pos="0.1 0.1 0.3"><freejoint/><geom type="cylinder" size="0.05 0.07" mass="0.7"/></body>
</worldbody></mujoco>"""


def _convex_states(m, n, rng):
  """Each world holds one convex pair in shallow contact (the other bodies
  parked apart, off the floor): world w takes pair kind w % 8; body A at a
  random orientation, body B (or the table top) placed so that its extreme
  point along -u lies 0.5-5 mm inside A's extreme point along a random u: the
  pair intersects at a depth of at most that (a generic, simulation-like
  contact; a deep overlap has several near-equal local minima of the depth and
  no well-defined normal)."""
  from mjlab_amd.utils import rot
  from tests.test_convex import _overlap, _support

  types = np.asarray(m.geom_type)
  sizes = np.asarray(m.geom_size)
  body_of = {name: i for i, name in enumerate(["egg", "can", "pill", "ball", "egg2", "can2"])}
  geom_of = {b: 3 + b for b in range(6)}  # floor, table, post, then one geom per body
  pairs = [("ball", "egg2"), ("pill", "egg"), ("egg", "egg2"), ("pill", "can"), ("egg", "can"), ("can", "can2"),
           ("egg", "table"), ("can", "table")]
  q = np.zeros((n, m.nq))
  for w in range(n):
    for b in range(6):  # parked: 0.6 m apart, 1 m up
      q[w, 7 * b : 7 * b + 3] = [2.0 + 0.6 * b, 0.0, 1.0]
      q[w, 7 * b + 3] = 1.0
    a, c = pairs[w % 8]
    ba = body_of[a]
    qa = rng.normal(size=4)
    qa /= np.linalg.norm(qa)
    ga = geom_of[ba]
    A = (int(types[ga]), list(sizes[ga]), rot.quat_to_mat(qa), np.zeros(3))
    pen = rng.uniform(0.0005, 0.005)
    if c == "table":  # the lowest point of A 'pen' below the table top (z = 0.1)
      low = _support(*A, np.array([[0.0, 0.0, -1.0]]))[0, 2]
      pa = np.array([rng.uniform(-0.15, 0.05), rng.uniform(-0.15, 0.15), 0.1 - low - pen])  # clear of the post
      q[w, 7 * ba : 7 * ba + 7] = np.concatenate([pa, qa])
      continue
    bc = body_of[c]
    qc = rng.normal(size=4)
    qc /= np.linalg.norm(qc)
    gc = geom_of[bc]
    u = rng.normal(size=3)
    u /= np.linalg.norm(u)
    C = (int(types[gc]), list(sizes[gc]), rot.quat_to_mat(qc), np.zeros(3))
    # B's support point along -u placed 'pen' inside A's support point along u:
    # the pair intersects, and its overlap along u (a bound on the depth) is pen
    sa = _support(*A, u[None])[0]
    sc = _support(*C, -u[None])[0]
    pa = np.array([0.0, 0.0, 0.8])
    q[w, 7 * ba : 7 * ba + 7] = np.concatenate([pa, qa])
    q[w, 7 * bc : 7 * bc + 7] = np.concatenate([pa + sa - pen * u - sc, qc])
  return q


def test_convex_pairs_parity():
  """The general convex pairs (GJK + EPA + the normal's Newton polish,
  csrc/mjh_convex.h) on the HIP step against the oracle's float64 build of the
  same collider: 512 worlds, each with one pair in shallow contact (64 worlds
  per pair kind, _convex_states), one step, tests/scenes.py tolerances. The
  collider itself is pinned by tests/test_convex.py's known answers."""
  from mjlab_amd.spec.compiler import CONVEX_PAIRS, compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string

  n = 512
  m = compile_spec(read_mjcf_string(CONVEX_SCENE), 60, 360)
  assert m.nboxpair > 0 and not m.unsupported_pair_types
  rng = np.random.default_rng(57)
  q = _convex_states(m, n, rng)
  st = {"qpos": q, "qvel": rng.normal(scale=0.3, size=(n, m.nv)), "qacc_warmstart": np.zeros((n, m.nv))}
  sim = Simulation(n, SimulationCfg(nconmax=60, njmax=360, mujoco=MujocoCfg(timestep=0.002, iterations=20,
                                                                               ls_iterations=20)), m, DEV)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, follow=got)
  rep = assert_parity(got, ref, n, min_int_rate=0.95, tag=" convex pairs")
  g = got["contact_geom"].reshape(n, -1, 2)
  types = np.asarray(m.geom_type)
  kinds = {(int(types[a]), int(types[b])) for w in range(n) for a, b in g[w, : int(got["ncon"][w, 0])]}
  assert CONVEX_PAIRS <= kinds, sorted(CONVEX_PAIRS - kinds)  # every convex pair was exercised
  print("[convex pairs] contact kinds", sorted(kinds), "int rate", rep["int_match_rate"])
  _check_convex_against_support_minimum(m, got, q, n)


def _check_convex_against_support_minimum(m, got, q, n, per_kind=6):
  """The HIP contacts of the convex pairs against an independent statement of
  the answer (not the shared-source oracle): for each pair
  kind, `per_kind` worlds' contact depth must equal -min over unit u of
  h1(u) + h2(-u) (tests/test_convex.py's numpy support functions, Fibonacci sphere
  + Nelder-Mead), the overlap along the HIP normal must attain that minimum, and
  the contact point must lie midway between the two extreme points along it.
  Tolerances are float32-level (5e-5 m on 0.05-0.2 m shapes)."""
  from mjlab_amd.spec.compiler import CONVEX_PAIRS
  from mjlab_amd.utils import rot
  from tests.test_convex import _min_overlap, _overlap, _support

  types, sizes = np.asarray(m.geom_type), np.asarray(m.geom_size)
  gpos, gquat = np.asarray(m.geom_pos), np.asarray(m.geom_quat)
  bid = np.asarray(m.geom_bodyid)

  def shape(w, g):
    b = int(bid[g])
    if b == 0:  # a static geom: its own pose
      R, c = rot.quat_to_mat(gquat[g]), np.asarray(gpos[g], dtype=np.float64)
    else:  # one geom per body, at the body origin: the body's free-joint pose
      j = 7 * (b - 1)
      R, c = rot.quat_to_mat(q[w, j + 3 : j + 7]), q[w, j : j + 3]
    return (int(types[g]), list(sizes[g]), R, np.asarray(c, dtype=np.float64))

  checked = {}
  geoms = got["contact_geom"].reshape(n, -1, 2)
  for w in range(n):
    for k in range(int(got["ncon"][w, 0])):
      g1, g2 = (int(x) for x in geoms[w, k])
      kind = (int(types[g1]), int(types[g2]))
      if kind not in CONVEX_PAIRS or checked.get(kind, 0) >= per_kind:
        continue
      P, Q = shape(w, g1), shape(w, g2)
      fmin, _ = _min_overlap(P, Q)
      d = float(got["contact_dist"].reshape(n, -1)[w, k])
      nrm = got["contact_frame"].reshape(n, -1, 9)[w, k, :3].astype(np.float64)
      pos = got["contact_pos"].reshape(n, -1, 3)[w, k].astype(np.float64)
      assert abs(d + fmin) <= 5e-5, (kind, w, d, -fmin)
      assert _overlap(P, Q, nrm)[0] - fmin <= 5e-5, (kind, w, nrm)
      lo = np.dot(_support(*Q, -nrm[None])[0], nrm)
      hi = np.dot(_support(*P, nrm[None])[0], nrm)
      assert abs(np.dot(pos, nrm) - 0.5 * (lo + hi)) <= 5e-5, (kind, w)
      checked[kind] = checked.get(kind, 0) + 1
  print("[convex pairs] checked against the support-function minimum:", dict(sorted(checked.items())))
  assert set(checked) == set(CONVEX_PAIRS) and min(checked.values()) == per_kind, checked


BALL_SCENE = """<mujoco><compiler angle="radian"/><option timestep="0.002"/><worldbody>
<geom name="floor" type="plane" size="5 5 0.1"/>
<body name="torso" pos="0 0 0.4"><freejoint/><geom type="box" size="0.12 0.08 0.05" mass="3"/>
  <body name="arm" pos="0.12 0 0"><joint name="shoulder" type="ball" range="0 1.0" limited="true" damping="0.05" stiffness="2"/>
    <geom type="capsule" fromto="0 0 0 0.2 0 -0.05" size="0.03" mass="0.5"/>
    <body name="fore" pos="0.2 0 -0.05"><joint name="elbow" type="hinge" axis="0 1 0" range="-1.5 1.5" limited="true"/>
      <geom type="capsule" fromto="0 0 0 0.15 0 0" size="0.025" mass="0.3"/></body></body>
  <body name="leg" pos="-0.12 0 -0.05"><joint name="hip" type="ball" damping="0.1"/>
    <geom type="capsule" fromto="0 0 0 0 0 -0.25" size="0.035" mass="0.8"/></body>
</body></worldbody></mujoco>"""


def test_ball_joint_parity():
  """Ball joints on the HIP step against the oracle: a free torso with a
  limited, damped, sprung ball shoulder (a hinge elbow below it) and a free
  ball hip, random poses touching the floor, one step (kinematics, the
  three-dof cdof, cdof_dot from the parent velocity, the mju_subQuat spring,
  the cone-limit row, mju_quatIntegrate); tests/scenes.py tolerances. The ball
  joint itself is pinned by tests/test_ball_joint.py's closed forms."""
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string
  from mjlab_amd.utils import rot

  n = 512
  m = compile_spec(read_mjcf_string(BALL_SCENE), 50, 300)
  assert list(m.jnt_type) == [0, 1, 3, 1] and m.nq == 7 + 4 + 1 + 4 and m.nv == 6 + 3 + 1 + 3
  rng = np.random.default_rng(59)
  q = np.zeros((n, m.nq))
  q[:, :3] = rng.uniform([-0.2, -0.2, 0.1], [0.2, 0.2, 0.25], (n, 3))
  for a in (3, 7, 12):
    quat = rng.normal(size=(n, 4))
    q[:, a : a + 4] = quat / np.linalg.norm(quat, axis=1, keepdims=True)
  # the shoulder within 1.3 rad of its rest pose (its cone limit is 1.0 rad)
  ax = rng.normal(size=(n, 3))
  ang = rng.uniform(0, 1.3, n)
  q[:, 7:11] = np.stack([rot.axis_angle_to_quat(ax[i] / np.linalg.norm(ax[i]), ang[i]) for i in range(n)])
  q[:, 11] = rng.uniform(-1.6, 1.6, n)
  st = {"qpos": q, "qvel": rng.normal(scale=0.5, size=(n, m.nv)), "qacc_warmstart": np.zeros((n, m.nv))}
  sim = Simulation(n, SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.002, iterations=20,
                                                                               ls_iterations=20)), m, DEV)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, follow=got)
  rep = assert_parity(got, ref, n, min_int_rate=0.95, tag=" ball joints")
  lim = [(w, r) for w in range(n) for r in range(int(got["nefc"][w, 0])) if got["efc_type"][w, r] == 3]
  assert len(lim) > 20  # shoulder / elbow limit rows were exercised
  assert (got["ncon"] > 0).mean() > 0.5
  print("[ball joints] limit rows", len(lim), "int rate", rep["int_match_rate"])


def test_builtin_sensor_parity():
  """Every builtin sensor type outside the benchmark tasks' set on the HIP
  step against the oracle (tests/test_sensors_builtin.py's scene: frame
  sensors on body / xbody / geom / site objects with body / xbody / geom / site
  reference frames, actuator and joint-actuator sensors, ball-joint sensors,
  clock, e_potential, e_kinetic), random poses and velocities, one step; the
  oracle's sensors are pinned by that file's closed forms."""
  from tests import test_sensors_builtin as tsb

  n = 256
  m = tsb._model()
  st = tsb._state(np.random.default_rng(61), n)
  st["qacc_warmstart"] = np.zeros((n, m.nv))
  sim = Simulation(n, SimulationCfg(nconmax=8, njmax=64, mujoco=MujocoCfg(timestep=0.002)), m, DEV)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, follow=got)
  for s, name in enumerate(m.names["sensor"]):  # per sensor, so a mismatch names its sensor
    a, d = int(m.sensor_adr[s]), int(m.sensor_dim[s])
    err = np.abs(got["sensordata"][:, a:a + d] - ref["sensordata"][:, a:a + d])
    print(f"[sensor {name}] max|d|={err.max():.3e} worst world {int(err.max(axis=1).argmax())}")
  assert_parity(got, ref, n, tag=" builtin sensors")
  # the quaternion sensors as rotations too (the sign of mju_mat2Quat's branch
  # is part of the value compared above; this names the sensor on a mismatch)
  for name in ("fq_body_in_base", "fq_site", "fq_geom_in_body", "bq"):
    s = m.names["sensor"].index(name)
    a = int(m.sensor_adr[s])
    np.testing.assert_allclose(got["sensordata"][:, a:a + 4], ref["sensordata"][:, a:a + 4], atol=2e-5, err_msg=name)


def test_force_torque_sensor_contact_parity():
  """force / torque sensors with contacts on the HIP step against the oracle:
  tests/test_sensors_builtin.py's box-and-ball stack in random poses against
  the floor (the contact wrenches enter cfrc_int), one step; the oracle's
  cfrc_int is pinned there by the resting stack's weights."""
  from tests import test_sensors_builtin as tsb
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string
  from mjlab_amd.utils import rot

  n = 256
  m = compile_spec(read_mjcf_string(tsb.STACK_SCENE), 16, 64)
  rng = np.random.default_rng(62)
  q = np.zeros((n, 7))
  q[:, :2] = rng.uniform(-0.3, 0.3, (n, 2))
  q[:, 2] = rng.uniform(0.05, 0.2, n)
  for w in range(n):
    ax = rng.normal(size=3)
    q[w, 3:7] = rot.axis_angle_to_quat(ax / np.linalg.norm(ax), rng.uniform(0, 0.6))
  st = {"qpos": q, "qvel": rng.normal(scale=0.3, size=(n, 6)), "qacc_warmstart": np.zeros((n, 6))}
  sim = Simulation(n, SimulationCfg(nconmax=16, njmax=64, mujoco=MujocoCfg(timestep=0.002)), m, DEV)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True, follow=got)
  assert (got["ncon"] > 0).mean() > 0.5
  assert_parity(got, ref, n, tag=" force/torque sensors")


def test_rangefinder_parity():
  """rangefinder (mj_ray over plane, sphere, box, capsule, cylinder and
  ellipsoid geoms, the site body's and invisible geoms skipped) on the HIP
  forward against the oracle: the probe of tests/test_sensors_builtin.py's ray
  scene at random positions and orientations; distances to 1e-4 m, misses
  (-1) identical. The oracle is pinned there by closed-form distances."""
  from tests import test_sensors_builtin as tsb
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string

  n = 256
  m = compile_spec(read_mjcf_string(tsb.RAY_SCENE), 8, 64)
  rng = np.random.default_rng(63)
  q = np.zeros((n, 7))
  q[:, :3] = rng.uniform([-0.5, -0.5, 0.5], [0.5, 0.5, 1.5], (n, 3))
  quat = rng.normal(size=(n, 4))
  q[:, 3:] = quat / np.linalg.norm(quat, axis=1, keepdims=True)
  st = {"qpos": q, "qvel": np.zeros((n, 6))}
  sim = Simulation(n, SimulationCfg(nconmax=8, njmax=64, mujoco=MujocoCfg(timestep=0.002)), m, DEV)
  put(sim, st)
  sim.forward()
  got = get(sim, n)["sensordata"]
  ref = Oracle(m).run(n, st, integrate=False)["sensordata"]
  ref32 = Oracle(m, precision="f32").run(n, st, integrate=False)["sensordata"]
  # a grazing ray is ill-conditioned (a plane hit at incidence c moves by ~eps/c,
  # a near-tangent sphere or capsule hit can flip to the geom behind it): an
  # entry passes within 1e-4 m + 1e-3 relative of the float64 oracle, or of the
  # float32 build of the same oracle code (the same flip at float32)
  tol = 1e-4 + 1e-3 * np.abs(ref)
  ok = (np.abs(got - ref) <= tol) | (np.abs(got - ref32) <= tol)
  assert ok.all(), [(int(w), int(k), float(got[w, k]), float(ref[w, k]), float(ref32[w, k])) for w, k in np.argwhere(~ok)[:5]]
  assert (np.abs(got - ref) <= tol).mean() > 0.99  # the float32 exemption stays rare
  assert (ref > 0).mean() > 0.3 and (ref < 0).any()


@pytest.mark.parametrize("iterations", [1, 5])
def test_pgs_solver_parity(iterations):
  """opt.solver = PGS (MuJoCo's projected Gauss-Seidel on the dual; the
  reference's MujocoCfg maps solver="pgs" to mjSOL_PGS, sim.py:34-38,55):
  the HIP sweeps against the oracle's (oracle.c solve_pgs) from the same dual
  warm start, a fixed number of sweeps (a PGS solve rarely meets the 1e-8
  tolerance in a few sweeps, so both run to the cap): the soft solve test, as
  for the capped CG solves."""
  n = 256
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(43))
  cfg = dict(CFG, mujoco=MujocoCfg(timestep=0.005, iterations=iterations, solver="pgs"))
  sim = Simulation(n, SimulationCfg(**cfg, ls_parallel=False), m, DEV)
  assert m.solver == 0
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True)
  assert (got["nefc"] > 0).mean() > 0.5
  assert (got["solver_niter"] == ref["solver_niter"]).mean() > 0.95
  rep = compare_step(got, ref)
  print(f"[pgs iterations={iterations}]", {k: f"{v:.2e}" for k, v in rep["maxerr"].items() if "/" in k})
  assert not [f for f in rep["failures"] if "unconverged at the iteration cap" not in f], rep["failures"]
  # the warm-start decision (dual cost of the warm forces > 0 -> zero forces) agrees
  warm_dev, warm_ref = (got["solver_lstrace"][:, 0] >> 30) & 1, (ref["solver_lstrace"][:, 0] >> 30) & 1
  assert (warm_dev == warm_ref).mean() > 0.98


def test_pgs_converged_matches_newton():
  """PGS run long (3000 sweeps) on the HIP step reaches the minimiser the
  float64 oracle's Newton finds (the dual and primal problems share it), to
  the float32 resolution of a linearly converging iteration."""
  n = 128
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(45))
  cfg = dict(CFG, mujoco=MujocoCfg(timestep=0.005, iterations=3000, tolerance=1e-12, solver="pgs"))
  sim = Simulation(n, SimulationCfg(**cfg, ls_parallel=False), m, DEV)
  put(sim, st)
  sim.forward()
  got = get(sim, n)
  m.solver, m.iterations, m.tolerance, m.ls_parallel, m.ls_iterations = 2, 200, 1e-15, 0, 50
  ref = Oracle(m).run(n, st, integrate=False)
  scale = 1 + np.abs(ref["qacc"]).max(axis=1, keepdims=True)
  err = (np.abs(got["qacc"] - ref["qacc"]) / scale).max(axis=1)
  print("[pgs converged] max/median rel err", err.max(), np.median(err), "sweeps", got["solver_niter"].mean())
  assert np.median(err) < 1e-4 and err.max() < 2e-3, (np.median(err), err.max())


def test_pgs_known_answers_on_gpu():
  """The closed-form scenes on the HIP PGS: the condim-1 ball rests at the
  documented r* (tests/test_soft_constraint.py) and carries m g."""
  from tests.test_soft_constraint import G, MASS, PARAMS, RAD, ball_model, rest_penetration

  solref, solimp = PARAMS["default"]
  m = ball_model(solref, solimp)
  n = 8
  sim = Simulation(n, SimulationCfg(nconmax=8, njmax=32, mujoco=MujocoCfg(timestep=m.timestep, iterations=100,
                                                                          tolerance=1e-10, solver="pgs")), m, DEV)
  q = np.tile([0, 0, RAD + 0.002, 1, 0, 0, 0], (n, 1))
  put(sim, {"qpos": q})
  for _ in range(800):
    sim.step()
  z = sim.data.qpos[:, 2].double().cpu().numpy()
  np.testing.assert_allclose(z - RAD, rest_penetration(solref, solimp, m.timestep), rtol=2e-3)
  np.testing.assert_allclose(sim.data.qfrc_constraint[:, 2].double().cpu().numpy(), MASS * G, rtol=1e-4)
