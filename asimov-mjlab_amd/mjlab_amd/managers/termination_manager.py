"""Termination manager (``src/mjlab/managers/termination_manager.py:25-100``)."""

from __future__ import annotations

import torch

from mjlab_amd.managers.manager_base import as_mask, resolve_params


class TerminationManager:
  def __init__(self, cfg: dict, env) -> None:
    self._env = env
    self.cfg = cfg
    self._term_names, self._term_cfgs, self._class_term_cfgs = [], [], []
    for name, tcfg in cfg.items():
      if tcfg is None:
        continue
      resolve_params(env, tcfg)
      if isinstance(tcfg.func, type):
        tcfg.func = tcfg.func(tcfg, env)
        self._class_term_cfgs.append(tcfg)
      self._term_names.append(name)
      self._term_cfgs.append(tcfg)
    n = env.num_envs
    self._term_dones = {k: torch.zeros(n, dtype=torch.bool, device=env.device) for k in self._term_names}
    self._truncated_buf = torch.zeros(n, dtype=torch.bool, device=env.device)
    self._terminated_buf = torch.zeros_like(self._truncated_buf)
    self._dones_buf = torch.zeros_like(self._truncated_buf)
    self._reset_counts = torch.zeros(max(len(self._term_names), 1), dtype=torch.long, device=env.device)

  @property
  def active_terms(self) -> list[str]:
    return list(self._term_names)

  @property
  def dones(self) -> torch.Tensor:
    return self._dones_buf

  @property
  def time_outs(self) -> torch.Tensor:
    return self._truncated_buf

  @property
  def terminated(self) -> torch.Tensor:
    return self._terminated_buf

  def reset(self, env_ids=None) -> dict:
    m = as_mask(env_ids, self._env.num_envs, self._env.device)
    from mjlab_amd import envops

    if not self._term_dones:  # no terms (the reference accepts an empty config)
      extras = {}
    elif envops.masked_counts(list(self._term_dones.values()), m, self._reset_counts):
      extras = {"Episode_Termination/" + k: self._reset_counts[i] for i, k in enumerate(self._term_dones)}
    else:
      counts = torch.stack([(v & m).sum() for v in self._term_dones.values()])
      # no env masked: the log keeps the last reset's counts (as the kernel)
      self._reset_counts[: len(counts)] = torch.where(m.any(), counts, self._reset_counts[: len(counts)])
      extras = {"Episode_Termination/" + k: self._reset_counts[i] for i, k in enumerate(self._term_dones)}
    for tcfg in self._class_term_cfgs:
      if hasattr(tcfg.func, "reset"):
        tcfg.func.reset(env_ids=env_ids)
    return extras

  def compute(self) -> torch.Tensor:
    from mjlab_amd import envops

    values = [tcfg.func(self._env, **tcfg.params) for tcfg in self._term_cfgs]
    if envops.term_combine(values, list(self._term_dones.values()), [c.time_out for c in self._term_cfgs],
                           self._truncated_buf, self._terminated_buf, self._dones_buf):
      return self._dones_buf  # one launch: copies, ORs and dones
    self._truncated_buf.zero_()
    self._terminated_buf.zero_()
    for name, tcfg, value in zip(self._term_names, self._term_cfgs, values):
      if tcfg.time_out:
        self._truncated_buf |= value
      else:
        self._terminated_buf |= value
      self._term_dones[name].copy_(value)
    torch.bitwise_or(self._truncated_buf, self._terminated_buf, out=self._dones_buf)
    return self._dones_buf

  def get_term(self, name: str) -> torch.Tensor:
    return self._term_dones[name]
