"""mjlab_amd's torch layers vs golden vectors produced by the reference's own
functions (tools/make_golden.py, run in the build container against
/root/reference; fixtures are inputs + outputs only)."""

from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

from mjlab_amd.entity.data import compute_velocity_from_cvel
from mjlab_amd.tasks.velocity.mdp import rewards as R
from mjlab_amd.utils import math as M

G = Path(__file__).resolve().parent / "golden"


def T(a):
  return torch.as_tensor(a)


def test_math_matches_reference():
  z = np.load(G / "math.npz")
  q1, q2, v, e, ang = (T(z[k]) for k in ("q1", "q2", "v", "e", "ang"))
  mat = T(z["matrix_from_quat"])
  checks = {
    "quat_mul": M.quat_mul(q1, q2),
    "quat_apply": M.quat_apply(q1, v),
    "quat_apply_inverse": M.quat_apply_inverse(q1, v),
    "quat_from_euler_xyz": M.quat_from_euler_xyz(e[:, 0], e[:, 1], e[:, 2]),
    "matrix_from_quat": M.matrix_from_quat(q1),
    "quat_from_matrix": M.quat_from_matrix(mat),
    "yaw_quat": M.yaw_quat(q1),
    "wrap_to_pi": M.wrap_to_pi(ang),
    "quat_inv": M.quat_inv(q1 * 1.3),
    "axis_angle_from_quat": M.axis_angle_from_quat(q1),
    "quat_error_magnitude": M.quat_error_magnitude(q1, q2),
    "sft_pos": M.subtract_frame_transforms(v, q1, e, q2)[0],
    "sft_quat": M.subtract_frame_transforms(v, q1, e, q2)[1],
  }
  for k, got in checks.items():
    np.testing.assert_allclose(got.numpy(), z[k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_entity_velocity_conversion():
  z = np.load(G / "entity_velocity.npz")
  out = compute_velocity_from_cvel(T(z["pos"]), T(z["com"]), T(z["cvel"]))
  np.testing.assert_allclose(out.numpy(), z["out"], rtol=1e-6, atol=1e-6)


def _env(z):
  i = {k[3:]: T(v) for k, v in z.items() if k.startswith("in_")}
  n = i["cmd"].shape[0]
  data = SimpleNamespace(
    root_link_lin_vel_b=i["root_link_lin_vel_b"], root_link_ang_vel_b=i["root_link_ang_vel_b"],
    projected_gravity_b=i["projected_gravity_b"], body_link_quat_w=i["body_link_quat_w"],
    body_link_ang_vel_w=i["body_link_ang_vel_w"], gravity_vec_w=torch.tensor([0.0, 0.0, -1.0]).repeat(n, 1),
    site_pos_w=i["site_pos_w"], site_lin_vel_w=i["site_lin_vel_w"], joint_pos=i["joint_pos"],
    default_joint_pos=i["default_joint_pos"],
  )
  cur_ct = i["current_contact_time"]
  sensor = SimpleNamespace(
    data=SimpleNamespace(found=i["found"], force=i["force"], current_air_time=i["current_air_time"], current_contact_time=cur_ct),
    compute_first_contact=lambda dt, abs_tol=1e-8: (cur_ct > 0) & (cur_ct < dt + abs_tol),
  )
  scene = {
    "robot": SimpleNamespace(data=data),
    "feet": sensor,
    "angmom": SimpleNamespace(data=i["angmom"]),
    "self": SimpleNamespace(data=SimpleNamespace(found=i["self_found"])),
  }
  cmd = i["cmd"]
  cm = SimpleNamespace(get_command=lambda name: cmd)
  env = SimpleNamespace(scene=scene, command_manager=cm, extras={"log": {}}, step_dt=0.02, num_envs=n, device="cpu")
  cfg = SimpleNamespace(
    name="robot", joint_ids=slice(None), joint_idx=slice(None), body_ids=[1], body_idx=torch.tensor([1]),
    site_ids=slice(None), site_idx=slice(None),
  )
  return env, cfg


def test_velocity_rewards_match_reference():
  z = dict(np.load(G / "velocity_rewards.npz"))
  env, cfg = _env(z)
  got = {
    "track_linear_velocity": R.track_linear_velocity(env, std=0.5, command_name="twist"),
    "track_angular_velocity": R.track_angular_velocity(env, std=0.7, command_name="twist"),
    "flat_orientation_body": R.flat_orientation(env, std=0.45, asset_cfg=cfg),
    "body_angular_velocity_penalty": R.body_angular_velocity_penalty(env, asset_cfg=cfg),
    "angular_momentum_penalty": R.angular_momentum_penalty(env, sensor_name="angmom"),
    "self_collision_cost": R.self_collision_cost(env, sensor_name="self"),
    "feet_air_time": R.feet_air_time(env, sensor_name="feet", threshold_min=0.05, threshold_max=0.5, command_name="twist", command_threshold=0.5),
    "feet_clearance": R.feet_clearance(env, target_height=0.1, command_name="twist", command_threshold=0.05, asset_cfg=cfg),
    "feet_slip": R.feet_slip(env, sensor_name="feet", command_name="twist", command_threshold=0.05, asset_cfg=cfg),
    "soft_landing": R.soft_landing(env, sensor_name="feet", command_name="twist", command_threshold=0.05),
  }
  for k, v in got.items():
    np.testing.assert_allclose(v.numpy(), z["out_" + k], rtol=1e-5, atol=1e-6, err_msg=k)
