"""The full env step on the GPU: graph capture, replay, resets, finiteness."""

import pytest
import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
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
