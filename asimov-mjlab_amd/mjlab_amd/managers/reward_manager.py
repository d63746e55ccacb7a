"""Reward manager (``src/mjlab/managers/reward_manager.py:25-100``): sum(term * weight * dt)."""

from __future__ import annotations

import torch

from mjlab_amd.managers.manager_base import as_mask, resolve_params


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
    n, t = env.num_envs, len(self._term_names)
    # one (N, T) accumulator; the per-term dict holds column views (API parity)
    self._sums = torch.zeros(n, t, device=env.device)
    self._episode_sums = {k: self._sums[:, i] for i, k in enumerate(self._term_names)}
    self._reward_buf = torch.zeros(n, device=env.device)
    self._step_reward = torch.zeros(n, t, device=env.device)
    # weights live on the device, refreshed on the host before each (graph) step
    self._w = torch.zeros(t, device=env.device)
    self._reset_means = torch.zeros(max(t, 1), device=env.device)
    self._log_buf = torch.zeros(8, device=env.device)
    self._w_host: tuple | None = None
    self.sync_weights()

  def sync_weights(self) -> None:
    w = tuple(float(c.weight) for c in self._term_cfgs)
    if w != self._w_host:
      self._w.copy_(torch.tensor(w, dtype=torch.float32))
      self._w_host = w

  @property
  def active_pattern(self) -> tuple[bool, ...]:
    """Which terms are evaluated (weight != 0); changing it changes the op sequence."""
    return tuple(float(c.weight) != 0.0 for c in self._term_cfgs)

  @property
  def active_terms(self) -> list[str]:
    return list(self._term_names)

  def reset(self, env_ids=None) -> dict:
    m = as_mask(env_ids, self._env.num_envs, self._env.device)
    from mjlab_amd import envops

    cols = [self._sums[:, i] for i in range(len(self._term_names))]
    if envops.masked_means(cols, m, 1.0 / self._env.max_episode_length_s, True, self._reset_means):
      means = self._reset_means  # one launch: masked means of the episode sums, then cleared
    else:
      w = m.float()
      means = (self._sums * w[:, None]).sum(0) / (w.sum().clamp(min=1.0) * self._env.max_episode_length_s)
      # no env masked: the log keeps the last reset's values (as the kernel)
      means = torch.where(w.sum() > 0, means, self._reset_means[: len(self._term_names)])
      self._reset_means[: len(self._term_names)] = means
      self._sums.masked_fill_(m[:, None], 0.0)
    extras = {"Episode_Reward/" + k: means[i] for i, k in enumerate(self._term_names)}
    for tcfg in self._class_term_cfgs:
      if hasattr(tcfg.func, "reset"):
        tcfg.func.reset(env_ids=env_ids)
    return extras

  def compute(self, dt: float) -> torch.Tensor:
    """sum_i term_i * weight_i * dt (reward_manager.py:76-88); zero-weight terms
    are skipped and report 0, as in the reference."""
    self._env.__dict__["_command_active_cache"] = {}  # shared command-activity masks, this pass only
    self._env.__dict__["_reward_log_ratios"] = []  # the terms' metric logs, evaluated together below
    from mjlab_amd import envops

    # the fused terms are independent per-env jobs: recorded and launched as one
    # batch (mjh_batch_begin / mjh_batch_end); their outputs are read only below
    batch = envops.JobBatch(self._reward_buf)
    try:
      with batch:
        vals = [
          tcfg.func(self._env, **tcfg.params).float() if tcfg.weight != 0.0 else None
          for tcfg in self._term_cfgs
        ]
    finally:
      self._env.__dict__.pop("_command_active_cache", None)
      pending = self._env.__dict__.pop("_reward_log_ratios", [])

    if pending:
      if self._log_buf.numel() < len(pending):
        self._log_buf = torch.zeros(len(pending), device=self._env.device)
      log = self._env.extras.setdefault("log", {})
      if envops.sum_ratios([(a, b) for _, a, b in pending], self._log_buf):
        for i, (key, _, _) in enumerate(pending):
          log[key] = self._log_buf[i]
      else:
        for key, a, b in pending:
          log[key] = envops.ratio_value(a, b)

    if envops.reward_combine(vals, self._w, dt, self._reward_buf, self._step_reward, self._sums):
      return self._reward_buf
    zero = None
    for i, v in enumerate(vals):
      if v is None:
        zero = zero if zero is not None else torch.zeros_like(self._reward_buf)
        vals[i] = zero
    raw = torch.stack(vals, dim=1)  # (N, T) unweighted term values
    weighted = raw * (self._w * dt)
    self._step_reward.copy_(raw * self._w)  # value / dt = term * weight
    self._sums += weighted
    torch.sum(weighted, dim=1, out=self._reward_buf)
    return self._reward_buf

  def get_term_cfg(self, name: str):
    if name not in self._term_names:
      raise ValueError(f"Term '{name}' not found in active terms.")
    return self._term_cfgs[self._term_names.index(name)]
