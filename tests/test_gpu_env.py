"""The full env step on the GPU: graph capture, replay, resets, finiteness."""

import pytest
import torch

from mjlab_amd.envs import mdp as gmdp
from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.managers.manager_term_config import RewardTermCfg
from mjlab_amd.sim import native
from mjlab_amd.tasks import load_env_cfg

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("task,adim", [("Mjlab-Velocity-Flat-Unitree-G1", 29), ("Mjlab-Velocity-Flat-Unitree-Go1", 12)])
def test_env_graph_rollout(task, adim):
  cfg = load_env_cfg(task)
  cfg.scene.num_envs = 256
  cfg.seed = 0
  env = ManagerBasedRlEnv(cfg, device="cuda:0")
  assert env.use_graph
  env.reset()
  g = torch.Generator(device="cuda:0").manual_seed(1)
  dones = 0
  for i in range(60):
    a = 2 * torch.rand(256, adim, device="cuda:0", generator=g) - 1
    obs, rew, term, trunc, extras = env.step(a)
    dones += int((term | trunc).sum())
  assert env._graph is not None
  assert torch.isfinite(obs["policy"]).all() and torch.isfinite(obs["critic"]).all() and torch.isfinite(rew).all()
  assert ((env.sim.data.flags & 4) == 0).all()
  log = extras["log"]
  for k in ("Sim/contact_overflow_worlds", "Sim/efc_overflow_worlds", "Sim/nonfinite_worlds"):
    assert k in log and int(log[k]) >= 0
  assert int(log["Sim/nonfinite_worlds"]) == 0
  assert (env.episode_length_buf <= 60).all()
  assert native.LIB_PATH.name.startswith("libmjh")


def _gpu_motion(tmp_path, frames=120):
  from mjlab_amd.motion import KEYS, save_motion, synthetic_motion

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = frames
  env = ManagerBasedRlEnv(cfg, device="cuda:0")
  mot = synthetic_motion(env.sim, env.scene["robot"], num_frames=frames, fps=50.0)
  path = tmp_path / "clip.npz"
  save_motion(path, 50.0, **{k: mot[k] for k in KEYS})
  return str(path)


def test_tracking_graph_rollout(tmp_path):
  """Config 4 (G1 flat tracking) captured and replayed; the relative body
  targets (fused quaternion kernels) match the reference's torch formulas."""
  from mjlab_amd.utils import math as M

  cfg = load_env_cfg("Mjlab-Tracking-Flat-Unitree-G1")
  cfg.scene.num_envs = 256
  cfg.seed = 0
  cfg.commands["motion"].motion_file = _gpu_motion(tmp_path)
  env = ManagerBasedRlEnv(cfg, device="cuda:0")
  env.reset()
  g = torch.Generator(device="cuda:0").manual_seed(1)
  for _ in range(40):
    obs, rew, term, trunc, extras = env.step(0.2 * (2 * torch.rand(256, 29, device="cuda:0", generator=g) - 1))
  assert env._graph is not None
  assert torch.isfinite(obs["policy"]).all() and torch.isfinite(obs["critic"]).all() and torch.isfinite(rew).all()
  assert obs["policy"].shape == (256, 160) and obs["critic"].shape == (256, 286)
  c = env.command_manager.get_term("motion")
  ts = c.time_steps
  assert ((ts >= 0) & (ts < c.motion.time_step_total)).all()
  torch.testing.assert_close(c.joint_pos, c.motion.joint_pos[ts], rtol=0, atol=0)
  nb = len(c.cfg.body_names)
  a_pos = c.anchor_pos_w[:, None].repeat(1, nb, 1)
  r_pos = c.robot_anchor_pos_w[:, None].repeat(1, nb, 1)
  delta_pos = r_pos.clone()
  delta_pos[..., 2] = a_pos[..., 2]
  delta_ori = M.yaw_quat(M.quat_mul(c.robot_anchor_quat_w[:, None].repeat(1, nb, 1), M.quat_inv(c.anchor_quat_w[:, None].repeat(1, nb, 1))))
  torch.testing.assert_close(c.body_pos_relative_w, delta_pos + M.quat_apply(delta_ori, c.body_pos_w - a_pos), rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(c.body_quat_relative_w, M.quat_mul(delta_ori, c.body_quat_w), rtol=1e-5, atol=1e-5)


def test_vecenv_obs_survive_the_next_graph_replay():
  """RSL-RL stores a step's observations only after the NEXT env.step:
  the wrapper must hand out tensors that the graph replay does not overwrite."""
  from mjlab_amd.rl import RslRlVecEnvWrapper

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 64
  cfg.seed = 0
  env = ManagerBasedRlEnv(cfg, device="cuda:0")
  w = RslRlVecEnvWrapper(env, clip_actions=1.0)
  w.get_observations()
  g = torch.Generator(device="cuda:0").manual_seed(3)
  o1, r1, _, _ = w.step(2 * torch.rand(64, 29, device="cuda:0", generator=g) - 1)
  o1c, r1c = o1["policy"].clone(), r1.clone()
  o2, r2, _, _ = w.step(2 * torch.rand(64, 29, device="cuda:0", generator=g) - 1)
  assert env._graph is not None  # the second step replays the captured graph
  assert torch.equal(o1["policy"], o1c) and torch.equal(r1, r1c)
  assert not torch.equal(o2["policy"], o1c)


def _twin_envs(task: str, n: int, tmp_path=None):
  envs = []
  for use_graph in (True, False):
    cfg = load_env_cfg(task.split("+")[0])
    cfg.scene.num_envs = n
    cfg.seed = 7
    if "Tracking" in task:
      cfg.commands["motion"].motion_file = _gpu_motion(tmp_path)
    if task.endswith("+delay_history"):
      # observation delay and history inside the captured step (constant lags: the
      # draws are deterministic, so graph and eager agree bitwise; no corruption noise)
      pol = cfg.observations["policy"]
      pol.enable_corruption = False
      pol.terms["base_ang_vel"].delay_min_lag = pol.terms["base_ang_vel"].delay_max_lag = 2
      pol.terms["projected_gravity"].history_length = 3
      pol.terms["joint_vel"].delay_min_lag = pol.terms["joint_vel"].delay_max_lag = 1
      pol.terms["joint_vel"].history_length = 2
      pol.terms["joint_vel"].flatten_history_dim = True
    envs.append(ManagerBasedRlEnv(cfg, device="cuda:0", use_graph=use_graph))
  return envs


_STATE = ("qpos", "qvel", "qacc_warmstart", "ctrl", "time", "xpos", "xquat", "cvel", "subtree_com", "sensordata",
          "qfrc_applied", "xfrc_applied", "actuator_force", "nefc", "ncon", "solver_niter")


@pytest.mark.parametrize("task", ["Mjlab-Velocity-Flat-Unitree-G1", "Mjlab-Tracking-Flat-Unitree-G1",
                                  "Mjlab-Velocity-Flat-Unitree-G1+delay_history"])
def test_graph_replay_equals_eager_step(task, tmp_path):
  """The benchmarked object — the captured env step — against the same step run
  eagerly, call by call: from identical state, counters and seeds, every
  returned tensor, every log value and the simulation state must agree
  bitwise over K steps, with resets forced on a subset (episode_length_buf at
  the limit) so the masked reset kernels, the gated forward and the command
  resampling all run inside the graph."""
  n, K = 64, 10
  ge, ee = _twin_envs(task, n, tmp_path)
  adim = ge.action_manager.total_action_dim
  for e in (ge, ee):
    e.reset()
    e.episode_length_buf[:12] = e.max_episode_length - 1 - torch.arange(12, device="cuda:0") % 4
  g = torch.Generator(device="cuda:0").manual_seed(11)
  resets = 0
  for k in range(K):
    a = 2 * torch.rand(n, adim, device="cuda:0", generator=g) - 1
    og, rg, tg, trg, xg = ge.step(a)
    oe, re_, te, tre, xe = ee.step(a)
    if k >= 1:
      assert ge._graph is not None, "graph env must replay from step 2 on"
    assert ee._graph is None
    resets += int((tg | trg).sum())
    for name in ("policy", "critic"):
      assert torch.equal(og[name], oe[name]), f"step {k}: obs {name}"
    assert torch.equal(rg, re_), f"step {k}: reward"
    assert torch.equal(tg, te) and torch.equal(trg, tre), f"step {k}: dones"
    assert set(xg["log"]) == set(xe["log"])
    for key, v in xg["log"].items():
      assert torch.equal(torch.as_tensor(v), torch.as_tensor(xe["log"][key])), f"step {k}: log {key}"
    for f in _STATE:
      assert torch.equal(getattr(ge.sim.data, f), getattr(ee.sim.data, f)), f"step {k}: sim.data.{f}"
    assert torch.equal(ge.episode_length_buf, ee.episode_length_buf)
  assert resets >= 12
  if task.endswith("+delay_history"):
    # the device ring pointer advanced on every replay: the history holds distinct frames
    hb = ge.observation_manager._group_obs_term_history_buffer["policy"]["projected_gravity"]
    assert int(hb._pointer) == K % 3  # 1 + K appends (reset, then one per env step)
    assert not torch.equal(hb.buffer[:, 0], hb.buffer[:, -1])


def test_reset_with_seed_reproduces_device_draws():
  """reset(seed=s) restarts the fused kernels' random stream, so two
  resets with the same seed draw the same reset states and commands."""
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 64
  env = ManagerBasedRlEnv(cfg, device="cuda:0")
  snaps = []
  for _ in range(2):
    env.reset(seed=5)
    cmd = env.command_manager.get_term("twist")
    snaps.append([env.sim.data.qpos.clone(), env.sim.data.qvel.clone(), cmd.vel_command_b.clone(), cmd.time_left.clone()])
    for _ in range(3):
      env.step(torch.rand(64, 29, device="cuda:0"))
  for a, b in zip(*snaps):
    assert torch.equal(a, b)
  env.reset(seed=6)
  assert not torch.equal(env.sim.data.qpos, snaps[0][0])


def test_config1_single_env_zero_agent_against_oracle():
  """BASELINE.json config 1 (G1 flat velocity, num_envs=1, zero agent,
  scripts/play.py:212-215) on the HIP path: the eager env step with every
  physics pass shadowed by the float64 oracle (tests/refsim.Shadow tolerances)."""
  from tests.refsim import Shadow

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 1
  cfg.seed = 42
  env = ManagerBasedRlEnv(cfg, device="cuda:0", use_graph=False)
  sh = Shadow(env.sim)
  env.reset()
  zero = torch.zeros(1, 29, device="cuda:0")
  for _ in range(30):
    obs, rew, term, trunc, _ = env.step(zero)
  assert sh.nsteps >= 30 * 4
  assert torch.isfinite(obs["policy"]).all() and torch.isfinite(rew).all()
  # the zero agent holds the default pose: still standing after 30 env steps
  assert not bool(term.any())


@pytest.mark.parametrize("no_fell_over", [False, True])
def test_batched_reward_pass_equals_separate_launches(no_fell_over):
  """The job batches (mjh_batch_begin / mjh_batch_end: the reward terms as one
  dispatch per source file; the termination pass and the commands + interval
  events as sequential per-env chains) against the same kernels launched one
  by one: over K captured env steps from identical seeds,
  rewards, episode sums, logs, observations and the simulation state agree
  bitwise (the jobs run the same arithmetic; the batch only merges dispatches).
  Without the fell_over termination nothing fills the root-frame cache before
  the reward pass, so the reward terms' root-frame reads (the velocity-tracking
  jobs and a flat_orientation_l2 term's torch sum) depend on the root frame
  launching ahead of the independent batch (mjh_batch kProducer)."""
  from mjlab_amd import envops
  from mjlab_amd.sim import native

  class _NoBatch:
    def __init__(self, like, sequential=False):
      pass

    def __enter__(self):
      return self

    def __exit__(self, *exc):
      return False

  n, K = 64, 6
  envs = []
  for _ in range(2):
    cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
    cfg.scene.num_envs = n
    cfg.seed = 5
    if no_fell_over:
      del cfg.terminations["fell_over"]
      cfg.rewards["flat_orientation_l2"] = RewardTermCfg(func=gmdp.flat_orientation_l2, weight=-0.5)
    envs.append(ManagerBasedRlEnv(cfg, device="cuda:0"))  # captured steps: the sequential batches run too
  eb, es = envs
  assert eb._seq_term and eb._seq_post and eb._seq_reset
  for e in envs:
    e.reset()
    e.episode_length_buf[:8] = e.max_episode_length - 1
  g = torch.Generator(device="cuda:0").manual_seed(3)
  orig = envops.JobBatch
  for k in range(K):
    a = 2 * torch.rand(n, eb.action_manager.total_action_dim, device="cuda:0", generator=g) - 1
    before = native.CALLS["mjh_batch_end"]
    ob, rb, tb, trb, xb = eb.step(a)
    if k < 2:  # eager step, then the capture (later steps replay the graph: no host calls)
      assert native.CALLS["mjh_batch_end"] > before  # the batched passes ran
    envops.JobBatch = _NoBatch
    try:
      os_, rs, ts, trs, xs = es.step(a)
    finally:
      envops.JobBatch = orig
    assert torch.equal(rb, rs), f"step {k}: reward"
    assert torch.equal(eb.reward_manager._sums, es.reward_manager._sums), f"step {k}: episode sums"
    assert torch.equal(eb.reward_manager._step_reward, es.reward_manager._step_reward), f"step {k}: step reward"
    for name in ("policy", "critic"):
      assert torch.equal(ob[name], os_[name]), f"step {k}: obs {name}"
    for key, v in xb["log"].items():
      assert torch.equal(torch.as_tensor(v), torch.as_tensor(xs["log"][key])), f"step {k}: log {key}"
    for f in _STATE:
      assert torch.equal(getattr(eb.sim.data, f), getattr(es.sim.data, f)), f"step {k}: sim.data.{f}"


def test_env_origin_sites_static_and_robot_sites_at_reference_ids():
  """The reference's env-origin sites (terrain_importer.py:95-120) occupy site
  ids 0..num_envs-1 of every world and never move; the robot's sites sit at
  num_envs + k and are the ones the kernel writes (mjh_data.site_wstride /
  site_off): after captured env steps the origin block still equals
  scene.env_origins and the robot's feet sites lie at the feet."""
  n = 16
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = n
  env = ManagerBasedRlEnv(cfg, device="cuda:0")
  env.reset()
  for _ in range(3):
    env.step(torch.zeros(n, env.action_manager.total_action_dim, device="cuda:0"))
  torch.cuda.synchronize()
  sx = env.sim.data.site_xpos
  origins = env.scene.env_origins
  assert tuple(sx.shape) == (n, n + 6, 3)
  assert torch.equal(sx[:, :n], origins.unsqueeze(0).expand(n, n, 3))
  robot = env.scene["robot"]
  ids = robot.indexing.site_ids
  assert ids.tolist() == list(range(n, n + 6))
  torch.testing.assert_close(robot.data.site_pose_w[..., :3], sx[:, ids])
  feet = [env.sim.mj_model.names["site"].index(f"robot/{s}") for s in ("left_foot", "right_foot")]
  assert (sx[:, feet, 2] < 0.2).all() and (sx[:, feet, 2] > -0.05).all()  # on the ground, not at the origin block
