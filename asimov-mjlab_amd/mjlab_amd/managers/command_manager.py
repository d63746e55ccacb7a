"""Command manager and CommandTerm base (``src/mjlab/managers/command_manager.py``)."""

from __future__ import annotations

import torch

from mjlab_amd.managers.manager_base import ManagerTermBase, as_mask, masked_mean


class CommandTerm(ManagerTermBase):
  def __init__(self, cfg, env) -> None:
    super().__init__(env)
    self.cfg = cfg
    self.metrics: dict[str, torch.Tensor] = {}
    self.time_left = torch.zeros(self.num_envs, device=self.device)
    self.command_counter = torch.zeros(self.num_envs, device=self.device, dtype=torch.long)
    self._reset_means = torch.zeros(8, device=self.device)

  @property
  def command(self) -> torch.Tensor:
    raise NotImplementedError

  def reset(self, env_ids=None) -> dict:
    m = as_mask(env_ids, self.num_envs, self.device)
    extras = {}
    if self.metrics:
      from mjlab_amd import envops

      if len(self.metrics) > self._reset_means.numel():
        self._reset_means = torch.zeros(len(self.metrics), device=self.device)
      if envops.masked_means(list(self.metrics.values()), m, 1.0, True, self._reset_means):
        for i, k in enumerate(self.metrics):  # one launch: masked means, then the metrics cleared
          extras[k] = self._reset_means[i]
      else:
        w = m.float()
        vals = torch.stack(list(self.metrics.values()), dim=1)
        means = (vals * w[:, None]).sum(0) / w.sum().clamp(min=1.0)
        # no env masked: the log keeps the last reset's values (as the kernel)
        means = torch.where(w.sum() > 0, means, self._reset_means[: len(self.metrics)])
        self._reset_means[: len(self.metrics)] = means
        for i, (k, v) in enumerate(self.metrics.items()):
          extras[k] = means[i]
          v.masked_fill_(m, 0.0)
    if not self._reset_resample(m):
      self.command_counter.masked_fill_(m, 0)
      self._resample(m)
    return extras

  def _reset_resample(self, mask: torch.Tensor) -> bool:
    """Fused counter restart + resampling of the masked envs (terms override);
    False: run the generic masked_fill + _resample."""
    del mask
    return False

  def compute(self, dt: float) -> None:
    self._update_metrics()
    self.time_left -= dt
    self._resample(self.time_left <= 0.0)
    self._update_command()

  def _resample(self, mask: torch.Tensor) -> None:
    lo, hi = self.cfg.resampling_time_range
    torch.where(mask, torch.rand_like(self.time_left) * (hi - lo) + lo, self.time_left, out=self.time_left)
    self._resample_command(mask)
    self.command_counter += mask.long()

  def _update_metrics(self) -> None:
    raise NotImplementedError

  def _resample_command(self, mask: torch.Tensor) -> None:
    raise NotImplementedError

  def _update_command(self) -> None:
    raise NotImplementedError


class CommandManager:
  def __init__(self, cfg: dict, env) -> None:
    self._env = env
    self.cfg = cfg
    self._terms: dict[str, CommandTerm] = {}
    for name, tcfg in cfg.items():
      if tcfg is None:
        continue
      self._terms[name] = tcfg.class_type(tcfg, env)

  @property
  def active_terms(self) -> list[str]:
    return list(self._terms)

  def reset(self, env_ids=None) -> dict:
    extras = {}
    for name, t in self._terms.items():
      for k, v in t.reset(env_ids=env_ids).items():
        extras[f"Metrics/{name}/{k}"] = v
    return extras

  def compute(self, dt: float) -> None:
    for t in self._terms.values():
      t.compute(dt)

  def get_command(self, name: str) -> torch.Tensor:
    return self._terms[name].command

  def get_term(self, name: str) -> CommandTerm:
    return self._terms[name]

  def get_term_cfg(self, name: str):
    return self.cfg[name]


class NullCommandManager:
  active_terms: list[str] = []

  def reset(self, env_ids=None) -> dict:
    return {}

  def compute(self, dt: float) -> None:
    pass

  def get_command(self, name: str):
    return None
