"""Reward manager (``src/mjlab/managers/reward_manager.py:25-100``): sum(term * weight * dt)."""

from __future__ import annotations

import torch

from mjlab_amd.managers.manager_base import as_mask, masked_mean, resolve_params


class RewardManager:
  def __init__(self, cfg: dict, env) -> None:
    self._env = env
    self.cfg = cfg
    self._term_names: list[str] = []
    self._term_cfgs = []
    self._class_term_cfgs = []
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
    self._episode_sums = {k: torch.zeros(n, device=env.device) for k in self._term_names}
    self._reward_buf = torch.zeros(n, device=env.device)
    self._step_reward = torch.zeros(n, len(self._term_names), device=env.device)

  @property
  def active_terms(self) -> list[str]:
    return list(self._term_names)

  def reset(self, env_ids=None) -> dict:
    m = as_mask(env_ids, self._env.num_envs, self._env.device)
    extras = {}
    for k, s in self._episode_sums.items():
      extras["Episode_Reward/" + k] = masked_mean(s, m) / self._env.max_episode_length_s
      s.masked_fill_(m, 0.0)
    for tcfg in self._class_term_cfgs:
      if hasattr(tcfg.func, "reset"):
        tcfg.func.reset(env_ids=env_ids)
    return extras

  def compute(self, dt: float) -> torch.Tensor:
    self._reward_buf.zero_()
    for i, (name, tcfg) in enumerate(zip(self._term_names, self._term_cfgs)):
      if tcfg.weight == 0.0:
        self._step_reward[:, i] = 0.0
        continue
      value = tcfg.func(self._env, **tcfg.params) * tcfg.weight * dt
      self._reward_buf += value
      self._episode_sums[name] += value
      self._step_reward[:, i] = value / dt
    return self._reward_buf

  def get_term_cfg(self, name: str):
    if name not in self._term_names:
      raise ValueError(f"Term '{name}' not found in active terms.")
    return self._term_cfgs[self._term_names.index(name)]
