"""Motion clips for the tracking task: the npz format of
``src/mjlab/scripts/csv_to_npz.py:205-308`` and a synthetic clip generator.

Format (float32 unless noted): ``fps`` (1,), ``joint_pos``/``joint_vel``
(T, nj), ``body_pos_w``/``body_lin_vel_w``/``body_ang_vel_w`` (T, nb, 3),
``body_quat_w`` (T, nb, 4), bodies in the robot entity's body order.

``synthetic_motion`` builds a smooth sinusoidal joint trajectory around the
robot's default pose and evaluates every frame in one batched forward pass
(each frame is a world): joint velocities are the analytic derivatives, body
poses/velocities come from the kinematics outputs, as csv_to_npz takes them
from MuJoCo after mj_forward.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

KEYS = ("joint_pos", "joint_vel", "body_pos_w", "body_quat_w", "body_lin_vel_w", "body_ang_vel_w")


def save_motion(path: str | Path, fps: float, **arrays) -> None:
  missing = [k for k in KEYS if k not in arrays]
  if missing:
    raise ValueError(f"motion arrays missing: {missing}")
  np.savez(path, fps=np.array([fps], np.float32), **{k: np.asarray(arrays[k], np.float32) for k in KEYS})


def load_motion(path: str | Path) -> dict[str, np.ndarray]:
  data = np.load(path)  # allow_pickle=False (default): data only
  out = {k: data[k] for k in KEYS}
  out["fps"] = data["fps"] if "fps" in data.files else np.array([50.0], np.float32)
  T = out["joint_pos"].shape[0]
  for k in KEYS:
    if out[k].shape[0] != T:
      raise ValueError(f"{k}: {out[k].shape[0]} frames, expected {T}")
  return out


def synthetic_motion(sim, robot, num_frames: int = 500, fps: float = 50.0, amplitude: float = 0.25, forward=None) -> dict:
  """Evaluate a sinusoidal joint trajectory on ``sim`` (which must have at
  least ``num_frames`` worlds). ``forward`` defaults to ``sim.forward``."""
  n = sim.num_envs
  if n < num_frames:
    raise ValueError(f"sim has {n} worlds, need {num_frames}")
  dev = sim.data.qpos.device
  t = torch.arange(n, device=dev, dtype=torch.float32) / fps
  nj = robot.num_joints
  phase = torch.linspace(0.0, 2 * torch.pi, nj, device=dev)
  freq = 0.5 + 0.5 * (torch.arange(nj, device=dev) % 3).float()  # 0.5..1.5 Hz
  arg = 2 * torch.pi * freq[None] * t[:, None] + phase[None]
  q0 = robot.data.default_joint_pos[:1]
  jp = q0 + amplitude * torch.sin(arg)
  lim = robot.data.soft_joint_pos_limits[0]
  jp = torch.clamp(jp, lim[:, 0], lim[:, 1])
  jv = amplitude * 2 * torch.pi * freq[None] * torch.cos(arg)
  root = robot.data.default_root_state[:1, :7].repeat(n, 1)
  robot.write_root_link_pose_to_sim(root)
  robot.write_root_link_velocity_to_sim(torch.zeros(n, 6, device=dev))
  robot.write_joint_state_to_sim(jp, jv)
  (forward or sim.forward)()
  d = robot.data
  T = num_frames
  return {
    "fps": np.array([fps], np.float32),
    "joint_pos": jp[:T].cpu().numpy(),
    "joint_vel": jv[:T].cpu().numpy(),
    "body_pos_w": d.body_link_pos_w[:T].cpu().numpy(),
    "body_quat_w": d.body_link_quat_w[:T].cpu().numpy(),
    "body_lin_vel_w": d.body_link_lin_vel_w[:T].cpu().numpy(),
    "body_ang_vel_w": d.body_link_ang_vel_w[:T].cpu().numpy(),
  }
