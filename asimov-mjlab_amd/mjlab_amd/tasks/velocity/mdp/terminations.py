"""Velocity-task terminations (``src/mjlab/tasks/velocity/mdp/terminations.py``)."""

from __future__ import annotations

import torch


def illegal_contact(env, sensor_name: str) -> torch.Tensor:
  return torch.any(env.scene[sensor_name].data.found > 0, dim=-1)
