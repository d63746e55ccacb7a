"""Generic termination terms (``src/mjlab/envs/mdp/terminations.py``)."""

from __future__ import annotations

import torch

from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from mjlab_amd.sim.sim import detect_nans

_DEFAULT = SceneEntityCfg("robot")


def time_out(env) -> torch.Tensor:
  return env.episode_length_buf >= env.max_episode_length


def bad_orientation(env, limit_angle: float, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  g = env.scene[asset_cfg.name].data.projected_gravity_b
  return torch.acos(-g[:, 2]).abs() > limit_angle


def root_height_below_minimum(env, minimum_height: float, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  return env.scene[asset_cfg.name].data.root_link_pos_w[:, 2] < minimum_height


def nan_detection(env) -> torch.Tensor:
  return detect_nans(env.sim.data)
