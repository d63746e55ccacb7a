"""Generic termination terms (``src/mjlab/envs/mdp/terminations.py``)."""

from __future__ import annotations

import math

import torch

from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from mjlab_amd.sim.sim import detect_nans

_DEFAULT = SceneEntityCfg("robot")


def time_out(env) -> torch.Tensor:
  if env.episode_length_buf.is_cuda:
    from mjlab_amd import envops

    fused = envops.time_out(env.episode_length_buf, int(env.max_episode_length))
    if fused is not None:
      return fused
  return env.episode_length_buf >= env.max_episode_length


def bad_orientation(env, limit_angle: float, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  """acos(-g_z) > limit (reference terminations.py, ``torch.acos(-g[:, 2]).abs() >
  limit_angle``). acos is decreasing with values in [0, pi], so for a limit in
  [0, pi] this is -cos(limit) < g_z <= 1. The reference's acos is NaN (so False)
  for g_z outside [-1, 1] and for NaN; the comparisons are False there too. The
  two forms can differ only for g_z within float32 rounding of -cos(limit)
  (the reference rounds acos's result, this form the threshold)."""
  g = env.scene[asset_cfg.name].data.projected_gravity_b
  if 0.0 <= limit_angle <= math.pi:
    gz = g[:, 2]
    from mjlab_amd import envops

    fused = envops.gz_above(gz, -math.cos(limit_angle))
    return fused if fused is not None else (gz > -math.cos(limit_angle)) & (gz <= 1.0)
  return torch.acos(-g[:, 2]).abs() > limit_angle


def root_height_below_minimum(env, minimum_height: float, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  return env.scene[asset_cfg.name].data.root_link_pos_w[:, 2] < minimum_height


def nan_detection(env) -> torch.Tensor:
  return detect_nans(env.sim.data)
