"""Tracking rewards (``src/mjlab/tasks/tracking/mdp/rewards.py``): Gaussian
kernels of anchor/body pose and velocity errors against the motion command."""

from __future__ import annotations

import torch

from mjlab_amd import envops
from mjlab_amd.envops import quat_error_magnitude


def _get_body_indexes(command, body_names: tuple[str, ...] | None):
  """rewards.py:17-24, as a slice when every tracked body is selected (no
  gather), else a device index tensor made once per body set (a Python list
  index would be an H2D copy inside the captured step)."""
  idx = [i for i, name in enumerate(command.cfg.body_names) if (body_names is None) or (name in body_names)]
  if len(idx) == len(command.cfg.body_names):
    return slice(None)
  cache = command.__dict__.setdefault("_body_index_cache", {})
  key = tuple(idx)
  if key not in cache:
    cache[key] = torch.tensor(idx, dtype=torch.long, device=command.device)
  return cache[key]


def _rows(c, body_names):
  """int32 row indices (motion side, robot entity side) of the selected tracked
  bodies for envops.rew_exp_err, made once per body set."""
  cache = c.__dict__.setdefault("_rew_rows_cache", {})
  key = tuple(body_names) if body_names is not None else None
  if key not in cache:
    idx = [i for i, name in enumerate(c.cfg.body_names) if (body_names is None) or (name in body_names)]
    t = torch.tensor(idx, dtype=torch.int32, device=c.device)
    cache[key] = (None if len(idx) == len(c.cfg.body_names) else t, c.body_indexes[t.long()].to(torch.int32).contiguous())
  return cache[key]


def _robot(c, kind: str):
  """The robot entity's per-body reads the robot_body_* properties gather from (views)."""
  d = c.robot.data
  return {"pos": d.body_link_pos_w, "quat": d.body_link_quat_w, "lin": d.body_link_lin_vel_w,
          "ang": d.body_link_ang_vel_w}[kind]


def _fused_body_err(c, motion, kind: str, std: float, body_names, quat: bool = False):
  ra, rb = _rows(c, body_names)
  return envops.rew_exp_err(motion, _robot(c, kind), std, quat, ra, rb)


def motion_global_anchor_position_error_exp(env, command_name: str, std: float) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  fused = envops.rew_exp_err(c.anchor_pos_w, c.robot_anchor_pos_w, std)
  if fused is not None:
    return fused
  error = torch.sum(torch.square(c.anchor_pos_w - c.robot_anchor_pos_w), dim=-1)
  return torch.exp(-error / std**2)


def motion_global_anchor_orientation_error_exp(env, command_name: str, std: float) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  fused = envops.rew_exp_err(c.anchor_quat_w, c.robot_anchor_quat_w, std, quat=True)
  if fused is not None:
    return fused
  error = quat_error_magnitude(c.anchor_quat_w, c.robot_anchor_quat_w) ** 2
  return torch.exp(-error / std**2)


def motion_relative_body_position_error_exp(env, command_name: str, std: float,
                                            body_names: tuple[str, ...] | None = None) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  fused = _fused_body_err(c, c.body_pos_relative_w, "pos", std, body_names)
  if fused is not None:
    return fused
  b = _get_body_indexes(c, body_names)
  error = torch.sum(torch.square(c.body_pos_relative_w[:, b] - c.robot_body_pos_w[:, b]), dim=-1)
  return torch.exp(-error.mean(-1) / std**2)


def motion_relative_body_orientation_error_exp(env, command_name: str, std: float,
                                               body_names: tuple[str, ...] | None = None) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  fused = _fused_body_err(c, c.body_quat_relative_w, "quat", std, body_names, quat=True)
  if fused is not None:
    return fused
  b = _get_body_indexes(c, body_names)
  error = quat_error_magnitude(c.body_quat_relative_w[:, b], c.robot_body_quat_w[:, b]) ** 2
  return torch.exp(-error.mean(-1) / std**2)


def motion_global_body_linear_velocity_error_exp(env, command_name: str, std: float,
                                                 body_names: tuple[str, ...] | None = None) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  fused = _fused_body_err(c, c.body_lin_vel_w, "lin", std, body_names)
  if fused is not None:
    return fused
  b = _get_body_indexes(c, body_names)
  error = torch.sum(torch.square(c.body_lin_vel_w[:, b] - c.robot_body_lin_vel_w[:, b]), dim=-1)
  return torch.exp(-error.mean(-1) / std**2)


def motion_global_body_angular_velocity_error_exp(env, command_name: str, std: float,
                                                  body_names: tuple[str, ...] | None = None) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  fused = _fused_body_err(c, c.body_ang_vel_w, "ang", std, body_names)
  if fused is not None:
    return fused
  b = _get_body_indexes(c, body_names)
  error = torch.sum(torch.square(c.body_ang_vel_w[:, b] - c.robot_body_ang_vel_w[:, b]), dim=-1)
  return torch.exp(-error.mean(-1) / std**2)


def self_collision_cost(env, sensor_name: str) -> torch.Tensor:
  """rewards.py:115-120: number of self-collisions detected by the sensor."""
  return env.scene[sensor_name].data.found.squeeze(-1)
