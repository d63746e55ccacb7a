"""Task registry (replaces the ``gym.register`` calls of ``src/mjlab/tasks/*/config/*/__init__.py``)."""

from __future__ import annotations

from copy import deepcopy
from typing import Callable

_REGISTRY: dict[str, Callable] = {}


def register(task_id: str, env_cfg_entry_point: Callable) -> None:
  _REGISTRY[task_id] = env_cfg_entry_point


def list_tasks() -> list[str]:
  _load_all()
  return sorted(_REGISTRY)


def load_env_cfg(task_id: str):
  """Fresh env cfg for ``task_id`` (a deep copy: cfgs are mutated by envs)."""
  _load_all()
  if task_id not in _REGISTRY:
    raise KeyError(f"Unknown task '{task_id}'. Known: {sorted(_REGISTRY)}")
  return deepcopy(_REGISTRY[task_id]())


def _load_all() -> None:
  from mjlab_amd.tasks.velocity import config  # noqa: F401
  from mjlab_amd.tasks.tracking import config as _tracking  # noqa: F401
