"""Tracking terminations (``src/mjlab/tasks/tracking/mdp/terminations.py``)."""

from __future__ import annotations

import torch

from mjlab_amd.envops import quat_apply_inverse
from mjlab_amd.tasks.tracking.mdp.rewards import _get_body_indexes


def bad_anchor_pos(env, command_name: str, threshold: float) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  return torch.norm(c.anchor_pos_w - c.robot_anchor_pos_w, dim=1) > threshold


def bad_anchor_pos_z_only(env, command_name: str, threshold: float) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  return torch.abs(c.anchor_pos_w[:, -1] - c.robot_anchor_pos_w[:, -1]) > threshold


def bad_anchor_ori(env, asset_cfg, command_name: str, threshold: float) -> torch.Tensor:
  asset = env.scene[asset_cfg.name]
  c = env.command_manager.get_term(command_name)
  g = asset.data.gravity_vec_w
  motion_g = quat_apply_inverse(c.anchor_quat_w, g)
  robot_g = quat_apply_inverse(c.robot_anchor_quat_w, g)
  return (motion_g[:, 2] - robot_g[:, 2]).abs() > threshold


def bad_motion_body_pos(env, command_name: str, threshold: float, body_names: tuple[str, ...] | None = None) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  b = _get_body_indexes(c, body_names)
  error = torch.norm(c.body_pos_relative_w[:, b] - c.robot_body_pos_w[:, b], dim=-1)
  return torch.any(error > threshold, dim=-1)


def bad_motion_body_pos_z_only(env, command_name: str, threshold: float,
                               body_names: tuple[str, ...] | None = None) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  b = _get_body_indexes(c, body_names)
  error = torch.abs(c.body_pos_relative_w[:, b, -1] - c.robot_body_pos_w[:, b, -1])
  return torch.any(error > threshold, dim=-1)
