"""Velocity-task curricula (``src/mjlab/tasks/velocity/mdp/curriculums.py:62-107``).

Host-side schedules on ``env.common_step_counter``; the env runs them before
each step's graph replay. ``terrain_levels_vel`` needs the terrain generator,
which is out of scope (flat terrain only).
"""

from __future__ import annotations

import torch


def commands_vel(env, env_ids, command_name: str, velocity_stages: list[dict]) -> dict[str, torch.Tensor]:
  del env_ids
  cfg = env.command_manager.get_term(command_name).cfg
  for stage in velocity_stages:
    if env.common_step_counter > stage["step"]:
      if stage.get("lin_vel_x") is not None:
        cfg.ranges.lin_vel_x = stage["lin_vel_x"]
      if stage.get("lin_vel_y") is not None:
        cfg.ranges.lin_vel_y = stage["lin_vel_y"]
      if stage.get("ang_vel_z") is not None:
        cfg.ranges.ang_vel_z = stage["ang_vel_z"]
  return {
    "lin_vel_x_min": torch.tensor(cfg.ranges.lin_vel_x[0]),
    "lin_vel_x_max": torch.tensor(cfg.ranges.lin_vel_x[1]),
    "lin_vel_y_min": torch.tensor(cfg.ranges.lin_vel_y[0]),
    "lin_vel_y_max": torch.tensor(cfg.ranges.lin_vel_y[1]),
    "ang_vel_z_min": torch.tensor(cfg.ranges.ang_vel_z[0]),
    "ang_vel_z_max": torch.tensor(cfg.ranges.ang_vel_z[1]),
  }


def reward_weight(env, env_ids, reward_name: str, weight_stages: list[dict]) -> torch.Tensor:
  del env_ids
  tcfg = env.reward_manager.get_term_cfg(reward_name)
  for stage in weight_stages:
    if env.common_step_counter > stage["step"]:
      tcfg.weight = stage["weight"]
  return torch.tensor([tcfg.weight])
