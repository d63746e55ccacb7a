"""Reset / event / command kernels against the reference's own functions.

``tests/golden/events_g1.npz`` (tools/make_golden_events.py) holds the outputs
of the reference's ``reset_root_state_uniform``, ``reset_joints_by_offset``,
``push_by_setting_velocity``, ``randomize_field``, ``CommandTerm._resample`` +
``UniformVelocityCommand._resample_command`` and ``MotionCommand._resample_command``
(adaptive sampling) on fixed inputs, with the random draws injected as exactly
the elements the fused HIP kernels draw from the env's device stream. Here the
mjlab_amd G1 envs are built on cuda:0, loaded with the fixture's inputs and
stream state (seed, step counter, call counter), and the same terms are called
through the product path, which launches the mjh_fuse.hip kernels.

Tolerances: positions/quaternions 2e-6, velocities 1e-5 (float32, the kernel
fuses some multiply-adds the reference rounds twice); integers and time steps
exact; sampling metrics 1e-6.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from mjlab_amd import envops
from mjlab_amd.envs.mdp import events
from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from mjlab_amd.sim import native
from tests import rng_np

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
AXES = ("x", "y", "z", "roll", "pitch", "yaw")
GOLDEN = __import__("pathlib").Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def fx():
  return dict(np.load(GOLDEN / "events_g1.npz"))


def D(a, dtype=None):
  return torch.as_tensor(np.asarray(a), device=DEV, dtype=dtype).contiguous()


def _ranges(arr) -> dict:
  return {k: (float(a), float(b)) for k, (a, b) in zip(AXES, np.asarray(arr))}


def _stream(env, fx) -> None:
  env._rng_seed = int(fx["seed"])
  env._rng_ctr.fill_(int(fx["step"]))
  env.__dict__["_rng_calls"] = 0


@pytest.fixture(scope="module")
def g1_env():
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 16
  return ManagerBasedRlEnv(cfg, device=DEV)


def _load_state(env, fx, prefix: str = "in_") -> None:
  d = env.scene["robot"].data
  env.sim.data.qpos.copy_(D(fx[prefix + "qpos"]))
  env.sim.data.qvel.copy_(D(fx[prefix + "qvel"]))
  env.scene.env_origins.copy_(D(fx[prefix + "env_origins"]))
  d.soft_joint_pos_limits.copy_(D(fx[prefix + "soft_joint_pos_limits"]))
  if prefix == "in_":
    d.default_root_state.copy_(D(fx["in_default_root_state"]))
    d.default_joint_pos.copy_(D(fx["in_default_joint_pos"]))
    d.default_joint_vel.copy_(D(fx["in_default_joint_vel"]))
  env.sim.epoch.bump()


def _check(got, want, name, tol):
  np.testing.assert_allclose(got.detach().cpu().numpy(), want, rtol=0, atol=tol, err_msg=name)


def test_numpy_stream_matches_device_stream(fx):
  """tests/rng_np.py restates csrc/mjh_rng.h bit for bit."""
  key = rng_np.site_key("reset_root_state_uniform.robot", 1)
  ctr = torch.tensor(int(fx["step"]), dtype=torch.long, device=DEV)
  got = envops.uniform_draws(int(fx["seed"]), key, ctr, 4096, DEV).cpu().numpy()
  assert np.array_equal(got, rng_np.u01(int(fx["seed"]), key, int(fx["step"]), np.arange(4096)))


@pytest.mark.parametrize("case", ["root_cfg", "root_all"])
def test_reset_root_state_uniform_matches_reference(g1_env, fx, case):
  env = g1_env
  _load_state(env, fx)
  _stream(env, fx)
  native.CALLS.clear()
  events.reset_root_state_uniform(env, D(fx["in_mask"]), _ranges(fx[f"{case}_pose_range"]),
                                  _ranges(fx[f"{case}_velocity_range"]), SceneEntityCfg("robot"))
  torch.cuda.synchronize()
  assert native.CALLS["mjh_reset_root_uniform"] > 0
  _check(env.sim.data.qpos, fx[f"{case}_qpos"], f"{case} qpos", 2e-6)
  _check(env.sim.data.qvel, fx[f"{case}_qvel"], f"{case} qvel", 1e-5)


@pytest.mark.parametrize("case", ["joints_cfg", "joints_all"])
def test_reset_joints_by_offset_matches_reference(g1_env, fx, case):
  env = g1_env
  _load_state(env, fx)
  _stream(env, fx)
  native.CALLS.clear()
  (plo, phi), (vlo, vhi) = fx[f"{case}_ranges"]
  events.reset_joints_by_offset(env, D(fx["in_mask"]), (float(plo), float(phi)), (float(vlo), float(vhi)),
                                SceneEntityCfg("robot"))
  torch.cuda.synchronize()
  assert native.CALLS["mjh_reset_joints_offset"] > 0
  _check(env.sim.data.qpos, fx[f"{case}_qpos"], f"{case} qpos", 2e-6)
  _check(env.sim.data.qvel, fx[f"{case}_qvel"], f"{case} qvel", 2e-6)


@pytest.mark.parametrize("case", ["push_cfg", "push_all"])
def test_push_by_setting_velocity_matches_reference(g1_env, fx, case):
  env = g1_env
  _load_state(env, fx)
  robot = env.scene["robot"]
  rb = int(robot.indexing.root_body_id)
  v = D(fx["in_root_link_vel_w"])
  # make the env's root_link_vel_w read the fixture's input: with the root's
  # position at the subtree com, vel = (cvel[3:6], cvel[0:3]) (entity/data.py:20-31)
  env.sim.data.subtree_com[:, rb] = env.sim.data.xpos[:, rb]
  env.sim.data.cvel[:, rb, 0:3] = v[:, 3:6]
  env.sim.data.cvel[:, rb, 3:6] = v[:, 0:3]
  env.sim.epoch.bump()
  _check(robot.data.root_link_vel_w, fx["in_root_link_vel_w"], "root_link_vel_w input", 1e-6)
  _stream(env, fx)
  native.CALLS.clear()
  events.push_by_setting_velocity(env, D(fx["in_mask"]), _ranges(fx[f"{case}_velocity_range"]), SceneEntityCfg("robot"))
  torch.cuda.synchronize()
  assert native.CALLS["mjh_push_velocity"] > 0
  _check(env.sim.data.qvel, fx[f"{case}_qvel"], f"{case} qvel", 1e-5)


def test_velocity_command_resample_matches_reference(g1_env, fx):
  env = g1_env
  cmd = env.command_manager.get_term("twist")
  c = cmd.cfg
  want_cfg = np.array([*c.resampling_time_range, c.rel_heading_envs, c.rel_standing_envs, *c.ranges.lin_vel_x,
                       *c.ranges.lin_vel_y, *c.ranges.ang_vel_z, *c.ranges.heading])
  np.testing.assert_allclose(want_cfg, fx["vc_cfg"], rtol=0, atol=1e-12, err_msg="G1 twist command cfg")
  for k in ("vel_command_b", "heading_target", "is_heading_env", "is_standing_env", "time_left", "command_counter"):
    getattr(cmd, k).copy_(D(fx["vc_in_" + k]))
  _stream(env, fx)
  native.CALLS.clear()
  assert cmd._resample_fused(D(fx["vc_mask"]), reset=False)
  torch.cuda.synchronize()
  assert native.CALLS["mjh_velocity_resample"] > 0
  for k, tol in (("vel_command_b", 2e-6), ("heading_target", 2e-6), ("time_left", 2e-6)):
    _check(getattr(cmd, k), fx["vc_out_" + k], k, tol)
  for k in ("is_heading_env", "is_standing_env", "command_counter"):
    assert np.array_equal(getattr(cmd, k).cpu().numpy(), fx["vc_out_" + k]), k


def test_motion_command_adaptive_resample_matches_reference(fx, tmp_path):
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.motion import save_motion
  from mjlab_amd.tasks import load_env_cfg

  clip = tmp_path / "clip.npz"
  save_motion(clip, float(fx["mo_clip_fps"][0]), **{k: fx["mo_clip_" + k] for k in (
    "joint_pos", "joint_vel", "body_pos_w", "body_quat_w", "body_lin_vel_w", "body_ang_vel_w")})
  cfg = load_env_cfg("Mjlab-Tracking-Flat-Unitree-G1")
  cfg.scene.num_envs = 16
  cfg.commands["motion"].motion_file = str(clip)
  env = ManagerBasedRlEnv(cfg, device=DEV)
  cmd = env.command_manager.get_term("motion")
  c = cmd.cfg
  np.testing.assert_allclose([c.adaptive_kernel_size, c.adaptive_lambda, c.adaptive_uniform_ratio, *c.joint_position_range],
                             fx["mo_cfg"], rtol=0, atol=1e-12, err_msg="G1 motion command cfg")
  assert list(env.scene["robot"].body_names) == [str(b) for b in fx["mo_body_names"]]
  assert cmd.bin_count == int(fx["mo_bin_count"])
  _load_state(env, fx, prefix="mo_in_")
  cmd.time_steps.copy_(D(fx["mo_in_time_steps"]))
  cmd.bin_failed_count.copy_(D(fx["mo_in_bin_failed_count"]))
  cmd._current_bin_failed.copy_(D(fx["mo_in_current_bin_failed"]))
  env.termination_manager.terminated.copy_(D(fx["mo_terminated"]))
  _stream(env, fx)
  native.CALLS.clear()
  cmd._resample_command(D(fx["mo_mask"]))
  torch.cuda.synchronize()
  assert native.CALLS["mjh_motion_adaptive"] > 0 and native.CALLS["mjh_motion_reset"] > 0
  assert np.array_equal(cmd.time_steps.cpu().numpy(), fx["mo_out_time_steps"]), "time steps"
  assert np.array_equal(cmd._current_bin_failed.cpu().numpy(), fx["mo_out_current_bin_failed"]), "failed-bin histogram"
  for m in ("sampling_entropy", "sampling_top1_prob", "sampling_top1_bin"):
    _check(cmd.metrics[m], fx["mo_out_" + m], m, 1e-6)
  _check(env.sim.data.qpos, fx["mo_out_qpos"], "motion reset qpos", 2e-6)
  _check(env.sim.data.qvel, fx["mo_out_qvel"], "motion reset qvel", 1e-5)
