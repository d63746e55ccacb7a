"""Tracking observations (``src/mjlab/tasks/tracking/mdp/observations.py``):
the motion anchor and the robot's tracked bodies in the robot anchor frame.
``subtract_frame_transforms`` + ``matrix_from_quat`` run as one fused kernel
(envops.frame_subtract) on the GPU."""

from __future__ import annotations

import torch

from mjlab_amd import envops


def motion_anchor_pos_b(env, command_name: str) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  pos, _ = envops.frame_subtract(c.robot_anchor_pos_w, c.robot_anchor_quat_w, c.anchor_pos_w, c.anchor_quat_w, want_q=False)
  return pos.view(env.num_envs, -1)


def motion_anchor_ori_b(env, command_name: str) -> torch.Tensor:
  """matrix_from_quat(q12)[..., :2] flattened: [m00, m01, m10, m11, m20, m21]."""
  c = env.command_manager.get_term(command_name)
  _, ori = envops.frame_subtract(c.robot_anchor_pos_w, c.robot_anchor_quat_w, c.anchor_pos_w, c.anchor_quat_w,
                                 want_t=False, qcols=2)
  return ori.reshape(env.num_envs, -1)


def robot_body_pos_b(env, command_name: str) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  pos_b, _ = envops.frame_subtract(c.robot_anchor_pos_w, c.robot_anchor_quat_w, c.robot_body_pos_w, c.robot_body_quat_w,
                                   want_q=False)
  return pos_b.reshape(env.num_envs, -1)


def robot_body_ori_b(env, command_name: str) -> torch.Tensor:
  c = env.command_manager.get_term(command_name)
  _, ori_b = envops.frame_subtract(c.robot_anchor_pos_w, c.robot_anchor_quat_w, c.robot_body_pos_w, c.robot_body_quat_w,
                                   want_t=False, qcols=2)
  return ori_b.reshape(env.num_envs, -1)
