"""Position reuse (mjh_set_position_reuse): a step launch on a world whose
qpos, mocap poses and model are bit-identical to the last forward's position
pass reuses that pass's results instead of recomputing kinematics, collision
and the constraint rows (the fused kernel: the forward saves them; the split
build, MJH_SPLIT=1: its position launch skips the world). Results must be
bit-identical with reuse on and off, and a change of any input the position
stage reads must force the pass."""

import numpy as np
import pytest
import torch

from mjlab_amd.sim import native
from tests.scenes import g1_mocap_scene, g1_scene_model, mocap_states, random_states
from tests.test_gpu_parity import DEV, get, make_sim, put

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _restore_reuse():
  yield
  native.lib().mjh_set_position_reuse(1)


def _run(sim, reuse, fn):
  fn()  # a graph replay: the reuse setting was captured with the graph (_make)
  torch.cuda.synchronize()


def _make(m, n, reuse, expand=()):
  """A Simulation whose captured step/forward graphs launch with position reuse
  on or off (the setting applies to launches issued after it, graph captures
  included)."""
  native.lib().mjh_set_position_reuse(1 if reuse else 0)
  sim = make_sim(m, n, expand)
  native.lib().mjh_set_position_reuse(1)
  return sim


def _same(a, b, tag):
  for k in a:
    assert a[k].tobytes() == b[k].tobytes(), f"{tag}: {k}"


def _twins(m, n, st, expand=()):
  sims = [_make(m, n, True, expand), _make(m, n, False, expand)]
  for s in sims:
    put(s, st)
  return sims


def test_reuse_is_bitwise_identical_g1():
  n = 64
  m = g1_scene_model(n)
  rng = np.random.default_rng(11)
  st = random_states(m, n, rng)
  on, off = _twins(m, n, st, expand=("geom_friction",))
  for reuse, sim in ((True, on), (False, off)):
    _run(sim, reuse, sim.forward)  # the env's reset-forward, then physics steps
    for _ in range(3):
      _run(sim, reuse, sim.step)
  _same(get(on, n), get(off, n), "forward + 3 steps")
  # reset some worlds' poses, then forward + step (those worlds must recompute)
  st2 = random_states(m, n, np.random.default_rng(12))
  idx = torch.arange(0, n, 5, device=DEV)
  for reuse, sim in ((True, on), (False, off)):
    sim.data.qpos[idx] = torch.as_tensor(st2["qpos"], dtype=torch.float32, device=DEV).view(n, -1)[idx]
    _run(sim, reuse, sim.forward)
    _run(sim, reuse, sim.step)
  _same(get(on, n), get(off, n), "partial reset")
  # domain randomisation between forward and step: the per-world field hash
  for reuse, sim in ((True, on), (False, off)):
    _run(sim, reuse, sim.forward)
    sim.model.geom_friction[3, :, 0] = 0.1
    _run(sim, reuse, sim.step)
  _same(get(on, n), get(off, n), "friction change")


def test_reuse_is_bitwise_identical_mocap():
  n = 32
  m = g1_mocap_scene(n).compile(50, 300)
  st = mocap_states(m, n, np.random.default_rng(13))
  on, off = _twins(m, n, st)
  for reuse, sim in ((True, on), (False, off)):
    _run(sim, reuse, sim.forward)
    sim.data.mocap_pos[::2] += 0.01  # moved mocap bodies: the pass must rerun
    _run(sim, reuse, sim.step)
    _run(sim, reuse, sim.forward)
    _run(sim, reuse, sim.step)
  _same(get(on, n), get(off, n), "mocap")


def test_reuse_skips_unchanged_worlds():
  """White-box: geom_xpos is written by the position pass only, so a sentinel
  written after a forward survives the next step exactly in the skipped worlds."""
  n = 16
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(14))
  sim = _make(m, n, True)
  put(sim, st)
  _run(sim, True, sim.forward)
  ref = sim.data.geom_xpos.clone()
  sim.data.geom_xpos.fill_(123.0)
  sim.data.qpos[1, 2] += 0.001  # world 1 changed
  _run(sim, True, sim.step)
  g = sim.data.geom_xpos
  skipped = torch.ones(n, dtype=torch.bool, device=DEV)
  skipped[1] = False
  assert bool((g[skipped] == 123.0).all())
  assert not bool((g[1] == 123.0).any())
  # the same with reuse off: every world recomputes
  sim2 = _make(m, n, False)
  put(sim2, st)
  _run(sim2, False, sim2.forward)
  sim2.data.geom_xpos.fill_(123.0)
  _run(sim2, False, sim2.step)
  assert torch.equal(sim2.data.geom_xpos, ref)


def test_env_steps_bitwise_with_and_without_reuse():
  """The G1 velocity env (resets, DR, pushes, the gated forward every step):
  observations, rewards and dones identical with position reuse on and off."""
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  n = 64

  def make(reuse):
    native.lib().mjh_set_position_reuse(1 if reuse else 0)
    cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
    cfg.scene.num_envs = n
    cfg.seed = 7
    env = ManagerBasedRlEnv(cfg, device=DEV)
    env.reset()
    env.episode_length_buf.copy_(torch.arange(n, device=DEV) * 15 % int(env.max_episode_length))
    g = torch.Generator(device=DEV).manual_seed(3)
    for _ in range(3):  # the env-step graph is captured here, with this reuse setting
      env.step(2 * torch.rand(n, env.action_manager.total_action_dim, device=DEV, generator=g) - 1)
    native.lib().mjh_set_position_reuse(1)
    return env, g

  (a, ga), (b, _) = make(True), make(False)
  for k in range(20):
    act = 2 * torch.rand(n, a.action_manager.total_action_dim, device=DEV, generator=ga) - 1
    oa, ra, ta, tra, _ = a.step(act)
    ob, rb, tb, trb, _ = b.step(act.clone())
    torch.cuda.synchronize()
    for grp in oa:
      assert torch.equal(oa[grp], ob[grp]), (k, grp)
    assert torch.equal(ra, rb) and torch.equal(ta, tb) and torch.equal(tra, trb), k
  assert torch.equal(a.sim.data.qpos, b.sim.data.qpos)


def test_keep_image_repacks_after_a_model_write():
  """mjh_step_keep_image reuses the packed model image only while no model
  field has changed since the launch that packed it (Simulation tracks the
  model buffers' torch version counters at launch/capture time). A captured
  sequence step -> in-place model write -> step(keep_image=True) must equal
  the eager sequence bitwise (a stale image would keep the old masses)."""
  from mjlab_amd.utils.capture import no_gc

  n = 32
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(13))
  eager, graphed = make_sim(m, n, ("body_mass",)), make_sim(m, n, ("body_mass",))
  for s in (eager, graphed):
    put(s, st)
  eager.step()
  eager.model.body_mass.mul_(1.5)
  eager.step()
  g = torch.cuda.CUDAGraph()
  torch.cuda.synchronize()
  with no_gc(), torch.cuda.graph(g):
    graphed.step()
    graphed.model.body_mass.mul_(1.5)
    graphed.step(keep_image=True)
  g.replay()
  _same(get(eager, n), get(graphed, n), "keep_image after a model write")
  # and without a write in between the image is reused (same results as packing)
  v = graphed.model_version()
  graphed.step()
  assert graphed.model_version() == v
