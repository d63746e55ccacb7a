"""Generic observation terms (``src/mjlab/envs/mdp/observations.py``)."""

from __future__ import annotations

import torch

from mjlab_amd import envops
from mjlab_amd.managers.scene_entity_config import SceneEntityCfg

_DEFAULT = SceneEntityCfg("robot")


def base_lin_vel(env, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  return env.scene[asset_cfg.name].data.root_link_lin_vel_b


def base_ang_vel(env, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  return env.scene[asset_cfg.name].data.root_link_ang_vel_b


def projected_gravity(env, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  return env.scene[asset_cfg.name].data.projected_gravity_b


def joint_pos_rel(env, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  a = env.scene[asset_cfg.name]
  j = asset_cfg.joint_idx
  return a.data.joint_pos[:, j] - a.data.default_joint_pos[:, j]


def joint_vel_rel(env, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  a = env.scene[asset_cfg.name]
  j = asset_cfg.joint_idx
  return a.data.joint_vel[:, j] - a.data.default_joint_vel[:, j]


def _joint_rel_src(env, key: str, state: str, default: str, asset_cfg: SceneEntityCfg = _DEFAULT):
  """joint_{pos,vel}_rel as an in-kernel subtraction of strided views (no
  gather, no subtraction launch) when the entity's joint columns are contiguous."""
  a = env.scene[asset_cfg.name]
  j = asset_cfg.joint_idx
  cols = a.data._cols[key]
  if not isinstance(j, slice) or not isinstance(cols, slice):
    return None
  x = getattr(a.data.data, state)[:, cols][:, j]
  return envops.ObsSrc(x, envops.OBS_SUB, getattr(a.data, default)[:, j])


joint_pos_rel.obs_src = lambda env, asset_cfg=_DEFAULT: _joint_rel_src(env, "joint_q_adr", "qpos", "default_joint_pos", asset_cfg)
joint_vel_rel.obs_src = lambda env, asset_cfg=_DEFAULT: _joint_rel_src(env, "joint_v_adr", "qvel", "default_joint_vel", asset_cfg)


def last_action(env, action_name: str | None = None) -> torch.Tensor:
  if action_name is None:
    return env.action_manager.action
  return env.action_manager.get_term(action_name).raw_action


def generated_commands(env, command_name: str) -> torch.Tensor:
  return env.command_manager.get_command(command_name)


def builtin_sensor(env, sensor_name: str) -> torch.Tensor:
  return env.scene[sensor_name].data
