"""Shared manager helpers: env-id normalisation to boolean masks.

The reference indexes subsets with ``env_ids`` tensors produced by
``nonzero()`` (a host sync per env step). Here every reset/interval path
works on a boolean mask of shape (num_envs,), so an entire env step can be
captured in one hipGraph. Index tensors and ``None`` are still accepted.
"""

from __future__ import annotations

import torch


def as_mask(env_ids, num_envs: int, device) -> torch.Tensor:
  if env_ids is None or (isinstance(env_ids, slice) and env_ids == slice(None)):
    return torch.ones(num_envs, dtype=torch.bool, device=device)
  if isinstance(env_ids, torch.Tensor) and env_ids.dtype == torch.bool:
    return env_ids
  m = torch.zeros(num_envs, dtype=torch.bool, device=device)
  m[env_ids] = True
  return m


def masked_mean(x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
  w = mask.float()
  return (x * w).sum() / w.sum().clamp(min=1.0)


def resolve_params(env, term_cfg) -> None:
  """Resolve SceneEntityCfg params against the scene (manager_base.py:86-93)."""
  from mjlab_amd.managers.scene_entity_config import SceneEntityCfg

  for value in getattr(term_cfg, "params", {}).values():
    if isinstance(value, SceneEntityCfg):
      value.resolve(env.scene)


class ManagerTermBase:
  def __init__(self, env) -> None:
    self._env = env

  @property
  def num_envs(self) -> int:
    return self._env.num_envs

  @property
  def device(self):
    return self._env.device

  def reset(self, env_ids=None) -> None:
    del env_ids
