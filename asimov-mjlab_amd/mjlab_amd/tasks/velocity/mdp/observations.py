"""Velocity-task observations (``src/mjlab/tasks/velocity/mdp/observations.py``)."""

from __future__ import annotations

import torch

from mjlab_amd.managers.scene_entity_config import SceneEntityCfg

_DEFAULT = SceneEntityCfg("robot")


def foot_height(env, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  return env.scene[asset_cfg.name].data.site_pos_w[:, asset_cfg.site_idx, 2]


def foot_air_time(env, sensor_name: str) -> torch.Tensor:
  return env.scene[sensor_name].data.current_air_time


def foot_contact(env, sensor_name: str) -> torch.Tensor:
  return (env.scene[sensor_name].data.found > 0).float()


def foot_contact_forces(env, sensor_name: str) -> torch.Tensor:
  f = env.scene[sensor_name].data.force.flatten(start_dim=1)
  return torch.sign(f) * torch.log1p(torch.abs(f))
