"""Tracking task (config 4 of BASELINE.json) on CPU, with the oracle standing in
for the physics (tests/oracle_sim.py): motion npz format, MotionCommand
semantics against direct restatements of the reference formulas
(tasks/tracking/mdp/commands.py), adaptive sampling, dims, capture safety."""

import math

import numpy as np
import pytest
import torch

from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.motion import KEYS, load_motion, save_motion, synthetic_motion
from mjlab_amd.tasks import list_tasks, load_env_cfg
from mjlab_amd.utils import math as M
from tests import oracle_sim
from tests.capture_guard import CaptureGuard

TRK = "Mjlab-Tracking-Flat-Unitree-G1"
FRAMES = 60


@pytest.fixture(scope="module")
def motion_file(tmp_path_factory):
  """Synthetic G1 clip: FRAMES worlds of a velocity-task env, one forward pass."""
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = FRAMES
  env = ManagerBasedRlEnv(cfg, device="cpu")
  oracle_sim.attach(env.sim)
  mot = synthetic_motion(env.sim, env.scene["robot"], num_frames=FRAMES, fps=50.0)
  path = tmp_path_factory.mktemp("motion") / "clip.npz"
  save_motion(path, 50.0, **{k: mot[k] for k in KEYS})
  return str(path)


def make(motion_file, n=6, sampling="adaptive", kernel_size=1):
  cfg = load_env_cfg(TRK)
  cfg.scene.num_envs = n
  cfg.seed = 7
  cfg.commands["motion"].motion_file = motion_file
  cfg.commands["motion"].sampling_mode = sampling
  cfg.commands["motion"].adaptive_kernel_size = kernel_size
  env = ManagerBasedRlEnv(cfg, device="cpu")
  oracle_sim.attach(env.sim, env.event_manager.domain_randomization_fields)
  return env


def test_registry():
  assert {TRK, TRK + "-No-State-Estimation"} <= set(list_tasks())


def test_empty_motion_file_rejected():
  cfg = load_env_cfg(TRK)
  cfg.scene.num_envs = 2
  with pytest.raises(ValueError, match="motion_file"):
    ManagerBasedRlEnv(cfg, device="cpu")


def test_motion_npz_roundtrip(motion_file, tmp_path):
  m = load_motion(motion_file)
  assert m["joint_pos"].shape == (FRAMES, 29) and m["body_quat_w"].shape[1:] == (m["body_pos_w"].shape[1], 4)
  np.testing.assert_allclose(np.linalg.norm(m["body_quat_w"], axis=-1), 1.0, atol=1e-5)
  # joint velocities are the derivative of the joint trajectory
  fd = (m["joint_pos"][2:] - m["joint_pos"][:-2]) * 50.0 / 2
  inside = np.abs(m["joint_vel"][1:-1]) > 0  # clamped joints excluded by tolerance below
  assert np.median(np.abs(fd - m["joint_vel"][1:-1])[inside]) < 0.05
  with pytest.raises(ValueError):
    save_motion(tmp_path / "bad.npz", 50.0, joint_pos=m["joint_pos"])


def test_dims_terms_and_steps(motion_file):
  env = make(motion_file)
  assert env.observation_manager.group_obs_dim == {"policy": (160,), "critic": (286,)}
  assert env.action_manager.total_action_dim == 29
  assert len(env.reward_manager.active_terms) == 9
  assert env.max_episode_length == math.ceil(10.0 / 0.02)
  assert set(env.event_manager.domain_randomization_fields) == {"body_ipos", "qpos0", "geom_friction"}
  env.reset()
  for _ in range(3):
    obs, rew, term, trunc, extras = env.step(0.3 * (2 * torch.rand(env.num_envs, 29) - 1))
  assert torch.isfinite(obs["policy"]).all() and torch.isfinite(obs["critic"]).all() and torch.isfinite(rew).all()


def test_no_state_estimation_variant(motion_file):
  cfg = load_env_cfg(TRK + "-No-State-Estimation")
  cfg.scene.num_envs = 2
  cfg.commands["motion"].motion_file = motion_file
  env = ManagerBasedRlEnv(cfg, device="cpu")
  assert env.observation_manager.group_obs_dim["policy"] == (160 - 6,)


def _ref_relative(c):
  """commands.py:383-405 with .repeat, as the reference writes it."""
  nb = len(c.cfg.body_names)
  a_pos = c.anchor_pos_w[:, None, :].repeat(1, nb, 1)
  a_quat = c.anchor_quat_w[:, None, :].repeat(1, nb, 1)
  r_pos = c.robot_anchor_pos_w[:, None, :].repeat(1, nb, 1)
  r_quat = c.robot_anchor_quat_w[:, None, :].repeat(1, nb, 1)
  delta_pos = r_pos.clone()
  delta_pos[..., 2] = a_pos[..., 2]
  delta_ori = M.yaw_quat(M.quat_mul(r_quat, M.quat_inv(a_quat)))
  return delta_pos + M.quat_apply(delta_ori, c.body_pos_w - a_pos), M.quat_mul(delta_ori, c.body_quat_w)


def test_command_frame_and_relative_bodies(motion_file):
  env = make(motion_file)
  env.reset()
  env.step(torch.zeros(env.num_envs, 29))
  c = env.command_manager.get_term("motion")
  mo = c.motion
  ts = c.time_steps
  assert ((ts >= 0) & (ts < mo.time_step_total)).all()
  torch.testing.assert_close(c.joint_pos, mo.joint_pos[ts], rtol=0, atol=0)
  torch.testing.assert_close(c.command, torch.cat([mo.joint_pos[ts], mo.joint_vel[ts]], 1), rtol=0, atol=0)
  torch.testing.assert_close(c.body_pos_w, mo.body_pos_w[ts] + env.scene.env_origins[:, None, :], rtol=0, atol=0)
  torch.testing.assert_close(c.body_quat_w, mo.body_quat_w[ts], rtol=0, atol=0)
  torch.testing.assert_close(c.anchor_ang_vel_w, mo.body_ang_vel_w[ts, c.motion_anchor_body_index], rtol=0, atol=0)
  pos, quat = _ref_relative(c)
  torch.testing.assert_close(c.body_pos_relative_w, pos, rtol=1e-6, atol=1e-6)
  torch.testing.assert_close(c.body_quat_relative_w, quat, rtol=1e-6, atol=1e-6)
  # robot-side reads == direct gathers
  d = env.scene["robot"].data
  torch.testing.assert_close(c.robot_body_pos_w, d.body_link_pos_w[:, c.body_indexes], rtol=0, atol=0)
  # reward formulas (rewards.py:27-40)
  r = env.reward_manager
  err = torch.sum(torch.square(c.anchor_pos_w - c.robot_anchor_pos_w), dim=-1)
  from mjlab_amd.tasks.tracking import mdp
  torch.testing.assert_close(mdp.motion_global_anchor_position_error_exp(env, "motion", 0.3), torch.exp(-err / 0.09))
  assert r is not None


def test_motion_end_resamples(motion_file):
  env = make(motion_file, sampling="start")
  env.reset()
  c = env.command_manager.get_term("motion")
  assert (c.time_steps == 0).all()
  env.step(torch.zeros(env.num_envs, 29))
  assert (c.time_steps == 1).all() | env.reset_buf.any()
  c.time_steps[:2] = c.motion.time_step_total - 1
  c._update_command()
  assert (c.time_steps[:2] == 0).all()  # "start" mode: wrapped to frame 0
  assert (c.time_steps[2:] >= 1).all()


def test_sampling_probabilities_match_conv1d(motion_file):
  env = make(motion_file, kernel_size=3)
  c = env.command_manager.get_term("motion")
  c.bin_count = 7
  c.bin_failed_count = torch.rand(7)
  ar = torch.arange(7)
  c._smooth_idx = torch.clamp(ar[:, None] + torch.arange(3)[None], max=6)
  got = c.sampling_probabilities()
  p = c.bin_failed_count + c.cfg.adaptive_uniform_ratio / 7.0
  p = torch.nn.functional.pad(p[None, None], (0, 2), mode="replicate")
  ref = torch.nn.functional.conv1d(p, c.kernel.view(1, 1, -1)).view(-1)
  torch.testing.assert_close(got, ref / ref.sum(), rtol=1e-6, atol=1e-7)


def test_adaptive_sampling_follows_failures(motion_file):
  torch.manual_seed(0)
  env = make(motion_file, n=2000)
  c = env.command_manager.get_term("motion")
  assert c.bin_count == int(FRAMES // 50) + 1
  c.bin_failed_count = torch.tensor([0.0, 100.0])
  mask = torch.ones(env.num_envs, dtype=torch.bool)
  c._adaptive_sampling(mask)
  p = c.sampling_probabilities()
  hi_bin = (c.time_steps * c.bin_count // c.motion.time_step_total) == 1
  # frames map to bins by floor(ts * B / T); the second bin holds most of the mass
  assert abs(hi_bin.float().mean().item() - float(p[1])) < 0.05
  assert c.metrics["sampling_top1_bin"][0].item() == pytest.approx(0.5)


def test_failed_bin_histogram(motion_file):
  env = make(motion_file, n=8)
  c = env.command_manager.get_term("motion")
  c.time_steps[:] = torch.tensor([0, 0, 55, 55, 55, 10, 10, 10])
  term = torch.tensor([1, 0, 1, 1, 0, 0, 0, 0], dtype=torch.bool)
  env.termination_manager.terminated.copy_(term)
  mask = torch.tensor([1, 1, 1, 1, 1, 0, 0, 0], dtype=torch.bool)
  c._adaptive_sampling(mask)
  bins = torch.clamp(torch.tensor([0, 0, 55, 55, 55]) * c.bin_count // FRAMES, 0, c.bin_count - 1)
  ref = torch.bincount(bins[term[:5]], minlength=c.bin_count).float()
  torch.testing.assert_close(c._current_bin_failed, ref)


def test_step_body_is_capture_safe(motion_file):
  env = make(motion_file)
  env.sim.step = env.sim.epoch.bump  # physics is the HIP kernel on the GPU: not under test here
  env.sim.forward_gated = lambda g: env.sim.epoch.bump()
  env.reset()
  env.step(torch.zeros(6, 29))
  env.episode_length_buf[:3] = 10_000  # force resets inside the guarded body
  c = env.command_manager.get_term("motion")
  c.time_steps[3:] = c.motion.time_step_total - 1  # force motion-end resampling
  with CaptureGuard():
    env._step_body()
