"""Observation noise configs (``src/mjlab/utils/noise/noise_cfg.py:22-105``)."""

from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class NoiseCfg:
  operation: str = "add"

  def apply(self, data: torch.Tensor) -> torch.Tensor:
    raise NotImplementedError

  def _t(self, v, like: torch.Tensor):
    return v if not isinstance(v, torch.Tensor) else v.to(like.device)

  def _op(self, data: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
    if self.operation == "add":
      return data + noise
    if self.operation == "scale":
      return data * noise
    if self.operation == "abs":
      return noise
    raise ValueError(f"Unsupported noise operation: {self.operation}")


@dataclass
class ConstantNoiseCfg(NoiseCfg):
  bias: float = 0.0

  def apply(self, data):
    return self._op(data, torch.zeros_like(data) + self._t(self.bias, data))


@dataclass
class UniformNoiseCfg(NoiseCfg):
  n_min: float = -1.0
  n_max: float = 1.0

  def __post_init__(self):
    if isinstance(self.n_min, (int, float)) and isinstance(self.n_max, (int, float)) and self.n_min >= self.n_max:
      raise ValueError(f"n_min ({self.n_min}) must be less than n_max ({self.n_max})")

  def apply(self, data):
    lo, hi = self._t(self.n_min, data), self._t(self.n_max, data)
    return self._op(data, torch.rand_like(data) * (hi - lo) + lo)


@dataclass
class GaussianNoiseCfg(NoiseCfg):
  mean: float = 0.0
  std: float = 1.0

  def apply(self, data):
    return self._op(data, self._t(self.mean, data) + self._t(self.std, data) * torch.randn_like(data))
