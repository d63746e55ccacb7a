"""Generate golden vectors from the reference's pure-torch layers (run HERE only).

The reference's physics backend (mujoco / mujoco_warp / warp) is not installed,
so its package is imported with inert stand-ins for those modules (SURVEY.md
§8c recipe); only torch-only functions are executed: isaaclab math utilities,
entity velocity conversion, velocity-task rewards/observations. Inputs are
seeded random tensors; inputs and outputs go to tests/golden/*.npz (data only —
no reference source is copied). Nothing here runs on the GPU box.
"""

from __future__ import annotations

import importlib.abc
import importlib.machinery
import sys
import types
from pathlib import Path
from types import SimpleNamespace
from unittest.mock import MagicMock

import numpy as np
import torch

REF = Path("/root/reference/src")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"
STUBS = ("warp", "mujoco", "mujoco_warp", "prettytable", "trimesh", "viser", "moviepy", "tensordict", "wandb", "tyro",
         "onnx", "onnxscript", "tqdm", "rsl_rl", "gymnasium", "mediapy", "imageio")


class _Stub(importlib.abc.MetaPathFinder, importlib.abc.Loader):
  def find_spec(self, name, path, target=None):
    if name.split(".")[0] in STUBS:
      return importlib.machinery.ModuleSpec(name, self, is_package=True)
    return None

  def create_module(self, spec):
    m = MagicMock(name=spec.name)
    m.__path__ = []
    m.__version__ = "0"
    m.__spec__ = spec
    return m

  def exec_module(self, module):
    pass


def setup() -> None:
  sys.dont_write_bytecode = True
  sys.meta_path.insert(0, _Stub())
  g = types.ModuleType("gymnasium")
  g.Env = type("Env", (), {})
  g.__path__ = []
  g.__getattr__ = lambda name: MagicMock(name=f"gymnasium.{name}")
  sys.modules["gymnasium"] = g
  sys.path.insert(0, str(REF))


def fake_env(n: int, g: torch.Generator):
  r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
  q = r(n, 4)
  q = q / q.norm(dim=-1, keepdim=True)
  body_q = r(n, 3, 4)
  body_q = body_q / body_q.norm(dim=-1, keepdim=True)
  found = (torch.rand(n, 2, generator=g) > 0.5).float()
  data = SimpleNamespace(
    root_link_lin_vel_b=r(n, 3), root_link_ang_vel_b=r(n, 3), projected_gravity_b=r(n, 3) * 0.3,
    body_link_quat_w=body_q, body_link_ang_vel_w=r(n, 3, 3), gravity_vec_w=torch.tensor([0.0, 0.0, -1.0]).repeat(n, 1),
    site_pos_w=r(n, 2, 3) * 0.1, site_lin_vel_w=r(n, 2, 3), joint_pos=r(n, 5) * 0.2, default_joint_pos=r(n, 5) * 0.1,
    root_link_quat_w=q,
  )
  cmd = r(n, 3)
  sensor = SimpleNamespace(data=SimpleNamespace(found=found, force=r(n, 2, 3) * 50, current_air_time=torch.rand(n, 2, generator=g) * 0.6,
                                                 current_contact_time=torch.rand(n, 2, generator=g) * 0.03))
  angmom = SimpleNamespace(data=r(n, 3))
  selfc = SimpleNamespace(data=SimpleNamespace(found=(torch.rand(n, 1, generator=g) * 3).floor()))
  asset = SimpleNamespace(data=data)
  return data, cmd, sensor, angmom, selfc, asset


def main() -> None:
  setup()
  from mjlab.entity.data import compute_velocity_from_cvel
  from mjlab.tasks.velocity.mdp import rewards as R
  from mjlab.third_party.isaaclab.isaaclab.utils import math as M

  OUT.mkdir(parents=True, exist_ok=True)
  g = torch.Generator().manual_seed(7)
  n = 64
  # ---- math ----
  q1 = torch.randn(n, 4, generator=g); q1 /= q1.norm(dim=-1, keepdim=True)
  q2 = torch.randn(n, 4, generator=g); q2 /= q2.norm(dim=-1, keepdim=True)
  v = torch.randn(n, 3, generator=g)
  e = torch.randn(n, 3, generator=g) * 2
  ang = torch.randn(n, generator=g) * 10
  mat = M.matrix_from_quat(q1)
  math_out = {
    "q1": q1, "q2": q2, "v": v, "e": e, "ang": ang,
    "quat_mul": M.quat_mul(q1, q2), "quat_apply": M.quat_apply(q1, v), "quat_apply_inverse": M.quat_apply_inverse(q1, v),
    "quat_from_euler_xyz": M.quat_from_euler_xyz(e[:, 0], e[:, 1], e[:, 2]), "matrix_from_quat": mat,
    "quat_from_matrix": M.quat_from_matrix(mat), "yaw_quat": M.yaw_quat(q1), "wrap_to_pi": M.wrap_to_pi(ang),
    "quat_inv": M.quat_inv(q1 * 1.3), "axis_angle_from_quat": M.axis_angle_from_quat(q1),
    "quat_error_magnitude": M.quat_error_magnitude(q1, q2),
    "sft_pos": M.subtract_frame_transforms(v, q1, e, q2)[0], "sft_quat": M.subtract_frame_transforms(v, q1, e, q2)[1],
  }
  np.savez(OUT / "math.npz", **{k: t.numpy() for k, t in math_out.items()})
  # ---- entity velocity conversion ----
  pos, com, cvel = torch.randn(n, 3, generator=g), torch.randn(n, 3, generator=g), torch.randn(n, 6, generator=g)
  np.savez(OUT / "entity_velocity.npz", pos=pos.numpy(), com=com.numpy(), cvel=cvel.numpy(),
           out=compute_velocity_from_cvel(pos, com, cvel).numpy())
  # ---- velocity-task rewards on a synthetic env snapshot ----
  data, cmd, sensor, angmom, selfc, asset = fake_env(n, g)
  scene = {"robot": asset, "feet": sensor, "angmom": angmom, "self": selfc}

  class CM:
    def get_command(self, name):
      return cmd

  sensor.compute_first_contact = lambda dt, abs_tol=1e-8: (sensor.data.current_contact_time > 0) & (sensor.data.current_contact_time < dt + abs_tol)
  env = SimpleNamespace(scene=scene, command_manager=CM(), extras={"log": {}}, step_dt=0.02, num_envs=n, device="cpu")
  cfg_all = SimpleNamespace(name="robot", joint_ids=slice(None), body_ids=[1], site_ids=slice(None), joint_names=[".*"], site_names=["a", "b"])
  out = {
    "track_linear_velocity": R.track_linear_velocity(env, std=0.5, command_name="twist"),
    "track_angular_velocity": R.track_angular_velocity(env, std=0.7, command_name="twist"),
    "flat_orientation_body": R.flat_orientation(env, std=0.45, asset_cfg=cfg_all),
    "body_angular_velocity_penalty": R.body_angular_velocity_penalty(env, asset_cfg=cfg_all),
    "angular_momentum_penalty": R.angular_momentum_penalty(env, sensor_name="angmom"),
    "self_collision_cost": R.self_collision_cost(env, sensor_name="self"),
    "feet_air_time": R.feet_air_time(env, sensor_name="feet", threshold_min=0.05, threshold_max=0.5, command_name="twist", command_threshold=0.5),
    "feet_clearance": R.feet_clearance(env, target_height=0.1, command_name="twist", command_threshold=0.05, asset_cfg=cfg_all),
    "feet_slip": R.feet_slip(env, sensor_name="feet", command_name="twist", command_threshold=0.05, asset_cfg=cfg_all),
    "soft_landing": R.soft_landing(env, sensor_name="feet", command_name="twist", command_threshold=0.05),
  }
  inputs = {
    "cmd": cmd, "root_link_lin_vel_b": data.root_link_lin_vel_b, "root_link_ang_vel_b": data.root_link_ang_vel_b,
    "projected_gravity_b": data.projected_gravity_b, "body_link_quat_w": data.body_link_quat_w,
    "body_link_ang_vel_w": data.body_link_ang_vel_w, "site_pos_w": data.site_pos_w, "site_lin_vel_w": data.site_lin_vel_w,
    "joint_pos": data.joint_pos, "default_joint_pos": data.default_joint_pos, "found": sensor.data.found,
    "force": sensor.data.force, "current_air_time": sensor.data.current_air_time,
    "current_contact_time": sensor.data.current_contact_time, "angmom": angmom.data, "self_found": selfc.data.found,
  }
  np.savez(OUT / "velocity_rewards.npz", **{"in_" + k: t.numpy() for k, t in inputs.items()}, **{"out_" + k: t.numpy() for k, t in out.items()})
  print("wrote", sorted(p.name for p in OUT.glob("*.npz")))


if __name__ == "__main__":
  main()
