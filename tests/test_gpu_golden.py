"""HIP env-layer kernels fed the reference-generated golden vectors directly
(tests/golden/{math,entity_velocity,velocity_rewards}.npz from
tools/make_golden.py). Each test also asserts, via the C-ABI launch tally
(mjlab_amd.sim.native.CALLS), that the HIP entry point actually ran.
Tolerance: float32 against the reference's float32 torch formulas, 1e-5."""

from pathlib import Path

import numpy as np
import pytest
import torch

from mjlab_amd import envops
from mjlab_amd.entity.data import compute_velocity_from_cvel
from mjlab_amd.sim import native
from tests.test_golden import _env

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
G = Path(__file__).resolve().parent / "golden"


def D(a):
  return torch.as_tensor(a, device=DEV).contiguous()


def _close(got, want, name, tol=1e-5):
  np.testing.assert_allclose(got.detach().cpu().numpy(), want, rtol=tol, atol=tol, err_msg=name)


def _ran(*names):
  for n in names:
    assert native.CALLS[n] > 0, f"HIP entry point {n} never ran"


def test_math_kernels_match_reference_vectors():
  native.CALLS.clear()
  z = np.load(G / "math.npz")
  q1, q2, v, e = D(z["q1"]), D(z["q2"]), D(z["v"]), D(z["e"])
  _close(envops.quat_apply(q1, v), z["quat_apply"], "quat_apply")
  _close(envops.quat_apply_inverse(q1, v), z["quat_apply_inverse"], "quat_apply_inverse")
  _close(envops.quat_mul(q1, q2), z["quat_mul"], "quat_mul")
  _close(envops.quat_from_euler_xyz(e), z["quat_from_euler_xyz"], "quat_from_euler_xyz")
  _close(envops.quat_error_magnitude(q1, q2), z["quat_error_magnitude"], "quat_error_magnitude", 2e-5)
  t12, q12 = envops.frame_subtract(v, q1, e, q2)
  _close(t12, z["sft_pos"], "subtract_frame_transforms pos")
  _close(q12, z["sft_quat"], "subtract_frame_transforms quat")
  torch.cuda.synchronize()
  _ran("mjh_quat_rotate", "mjh_quat_mul", "mjh_quat_from_euler", "mjh_quat_error", "mjh_frame_subtract")


def test_entity_velocity_kernel_matches_reference_vectors():
  native.CALLS.clear()
  z = np.load(G / "entity_velocity.npz")
  out = envops.velocity_from_cvel(D(z["pos"]), D(z["com"]), D(z["cvel"]), compute_velocity_from_cvel)
  _close(out, z["out"], "velocity_from_cvel")
  _ran("mjh_velocity_from_cvel")


def test_velocity_reward_kernels_match_reference_vectors():
  from mjlab_amd.tasks.velocity.mdp import rewards as R

  native.CALLS.clear()
  z = {k: v for k, v in np.load(G / "velocity_rewards.npz").items()}
  env, cfg = _env(z)
  # the same stand-in env with every tensor on the GPU

  def to_dev(ns):
    for k, v in vars(ns).items():
      if isinstance(v, torch.Tensor):
        setattr(ns, k, v.to(DEV))

  to_dev(env.scene["robot"].data)
  to_dev(env.scene["feet"].data)
  env.scene["angmom"].data = env.scene["angmom"].data.to(DEV)
  to_dev(env.scene["self"].data)
  cct = env.scene["feet"].data.current_contact_time
  env.scene["feet"].compute_first_contact = lambda dt, abs_tol=1e-8: (cct > 0) & (cct < dt + abs_tol)
  cmd = D(z["in_cmd"])
  env.command_manager.get_command = lambda name: cmd
  env.device = DEV
  cfg.body_idx = cfg.body_idx.to(DEV)
  got = {
    "track_linear_velocity": R.track_linear_velocity(env, std=0.5, command_name="twist"),
    "track_angular_velocity": R.track_angular_velocity(env, std=0.7, command_name="twist"),
    "flat_orientation_body": R.flat_orientation(env, std=0.45, asset_cfg=cfg),
    "body_angular_velocity_penalty": R.body_angular_velocity_penalty(env, asset_cfg=cfg),
    "angular_momentum_penalty": R.angular_momentum_penalty(env, sensor_name="angmom"),
    "self_collision_cost": R.self_collision_cost(env, sensor_name="self"),
    "feet_air_time": R.feet_air_time(env, sensor_name="feet", threshold_min=0.05, threshold_max=0.5, command_name="twist",
                                     command_threshold=0.5),
    "feet_clearance": R.feet_clearance(env, target_height=0.1, command_name="twist", command_threshold=0.05, asset_cfg=cfg),
    "feet_slip": R.feet_slip(env, sensor_name="feet", command_name="twist", command_threshold=0.05, asset_cfg=cfg),
    "soft_landing": R.soft_landing(env, sensor_name="feet", command_name="twist", command_threshold=0.05),
  }
  for k, v in got.items():
    assert v.is_cuda
    _close(v, z["out_" + k], k)
  _ran("mjh_rew_track", "mjh_rew_flat_orientation", "mjh_rew_sqsum", "mjh_rew_feet")
