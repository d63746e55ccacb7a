"""Observation manager (``src/mjlab/managers/observation_manager.py:147-278``).

Pipeline per term: compute -> noise (only if the group enables corruption) ->
clip -> scale -> delay (DelayBuffer) -> history (CircularBuffer, first frame
back-filled after a reset); groups concatenated along ``concatenate_dim``.
Groups without delay or history on the GPU run as one fused launch
(``_compute_fused``); the buffers are device-resident and capturable
(``utils/buffers``), so delayed / history terms run inside the captured env step.
"""

from __future__ import annotations

import numpy as np
import torch

from mjlab_amd.managers.manager_base import resolve_params
from mjlab_amd.utils.buffers import CircularBuffer, DelayBuffer


class ObservationManager:
  def __init__(self, cfg: dict, env) -> None:
    self._env = env
    self.cfg = cfg
    self._group_terms: dict[str, list[tuple[str, object]]] = {}
    self._group_concat: dict[str, bool] = {}
    self._group_concat_dim: dict[str, int] = {}
    # per group: term name -> DelayBuffer / CircularBuffer (the reference's attribute names)
    self._group_obs_term_delay_buffer: dict[str, dict[str, DelayBuffer]] = {}
    self._group_obs_term_history_buffer: dict[str, dict[str, CircularBuffer]] = {}
    self._class_terms = []
    for gname, gcfg in cfg.items():
      if gcfg is None:
        continue
      terms = []
      for tname, tcfg in gcfg.terms.items():
        if tcfg is None:
          continue
        if not gcfg.enable_corruption:
          tcfg.noise = None
        if gcfg.history_length is not None:
          tcfg.history_length = gcfg.history_length
          tcfg.flatten_history_dim = gcfg.flatten_history_dim
        resolve_params(env, tcfg)
        if isinstance(tcfg.func, type):
          tcfg.func = tcfg.func(tcfg, env)
          self._class_terms.append(tcfg.func)
        terms.append((tname, tcfg))
      self._group_terms[gname] = terms
      self._group_concat[gname] = gcfg.concatenate_terms
      self._group_concat_dim[gname] = gcfg.concatenate_dim
    # resolve scales, buffers and dims by evaluating every term once (observation_manager.py:246-278)
    self.group_obs_term_dim: dict[str, list[tuple[int, ...]]] = {}
    for gname, terms in self._group_terms.items():
      dims, delays, hists = [], {}, {}
      for tname, tcfg in terms:
        out = tcfg.func(env, **tcfg.params)
        obs_dims = tuple(out.shape)
        if tcfg.scale is not None and not isinstance(tcfg.scale, torch.Tensor):
          tcfg.scale = torch.tensor(tcfg.scale, dtype=torch.float32, device=env.device)
        if tcfg.delay_max_lag > 0:
          delays[tname] = DelayBuffer(min_lag=tcfg.delay_min_lag, max_lag=tcfg.delay_max_lag, batch_size=env.num_envs,
                                      device=env.device, per_env=tcfg.delay_per_env, hold_prob=tcfg.delay_hold_prob,
                                      update_period=tcfg.delay_update_period, per_env_phase=tcfg.delay_per_env_phase)
        if tcfg.history_length > 0:
          hists[tname] = CircularBuffer(max_len=tcfg.history_length, batch_size=env.num_envs, device=env.device)
          obs_dims = (obs_dims[0], tcfg.history_length, *obs_dims[1:])
          if tcfg.flatten_history_dim:
            obs_dims = (obs_dims[0], int(np.prod(obs_dims[1:])))
        dims.append(tuple(obs_dims[1:]))
      self.group_obs_term_dim[gname] = dims
      self._group_obs_term_delay_buffer[gname] = delays
      self._group_obs_term_history_buffer[gname] = hists
    self._obs_buffer = None
    self._fused = {g: self._fused_plan(g) for g in self._group_terms}
    # optional fixed noise draws per group, (N, group width) in U[0,1): replaces
    # the group's uniform draw in the fused path (used to replay golden vectors)
    self.noise_override: dict[str, torch.Tensor] = {}

  def _fused_plan(self, gname: str):
    """Per-term (offset, width, noise lo/hi or None, clip, scale) for groups that
    can be assembled by the fused kernel: concatenated on the last dim, no
    history, additive uniform (or no) noise, scalar scale."""
    from mjlab_amd.utils.noise import UniformNoiseCfg

    if not self._group_concat[gname] or self._group_concat_dim[gname] not in (-1, 1):
      return None
    plan, off = [], 0
    for (tname, tcfg), dims in zip(self._group_terms[gname], self.group_obs_term_dim[gname]):
      if tcfg.history_length > 0 or tcfg.delay_max_lag > 0 or len(dims) > 1:
        return None
      w = dims[0] if dims else 1
      noise = None
      if tcfg.noise is not None:
        nz = tcfg.noise
        if not (isinstance(nz, UniformNoiseCfg) and nz.operation == "add"):
          return None
        if isinstance(nz.n_min, torch.Tensor) or isinstance(nz.n_max, torch.Tensor):
          return None
        noise = (float(nz.n_min), float(nz.n_max))
      scale = 1.0
      if tcfg.scale is not None:
        if tcfg.scale.numel() != 1:
          return None
        scale = float(tcfg.scale.reshape(-1)[0])
      plan.append((tcfg, off, w, noise, tcfg.clip, scale))
      off += w
    return plan, off

  @property
  def active_terms(self) -> dict[str, list[str]]:
    return {g: [n for n, _ in t] for g, t in self._group_terms.items()}

  @property
  def group_obs_dim(self) -> dict:
    """Concatenated groups: the term dims summed along the concatenation dim
    (observation_manager.py:19-40); other groups: the per-term dims."""
    out = {}
    for g, dims in self.group_obs_term_dim.items():
      if not self._group_concat[g]:
        out[g] = dims
        continue
      if all(len(d) == 1 for d in dims):
        out[g] = (sum(int(d[0]) for d in dims),)
        continue
      if len({len(d) for d in dims}) != 1:
        raise RuntimeError(f"Unable to concatenate observation terms in group {g}.")
      cd = self._group_concat_dim[g]
      axis = cd - 1 if cd > 0 else cd  # the term dims exclude the env dim
      first = list(dims[0])
      first[axis] = sum(int(d[axis]) for d in dims)
      out[g] = tuple(first)
    return out

  @property
  def group_obs_concatenate(self) -> dict[str, bool]:
    return dict(self._group_concat)

  def reset(self, env_ids=None) -> dict:
    ids = None if env_ids is None or isinstance(env_ids, slice) else env_ids
    for gname in self._group_terms:
      for buf in self._group_obs_term_delay_buffer[gname].values():
        buf.reset(batch_ids=ids)
      for buf in self._group_obs_term_history_buffer[gname].values():
        buf.reset(batch_ids=ids)
    for c in self._class_terms:
      if hasattr(c, "reset"):
        c.reset(env_ids=env_ids)
    return {}

  def compute(self, update_history: bool = False) -> dict[str, torch.Tensor]:
    out = {g: self.compute_group(g, update_history) for g in self._group_terms}
    self._obs_buffer = out
    return out

  def compute_group(self, group_name: str, update_history: bool = False):
    fp = self._fused.get(group_name)
    if fp is not None and str(self._env.device).startswith("cuda"):
      out = self._compute_fused(fp, self.noise_override.get(group_name))
      if out is not None:
        return out
    obs_terms = {}
    for tname, tcfg in self._group_terms[group_name]:
      obs = tcfg.func(self._env, **tcfg.params).clone()  # noise/clip/scale act in place below
      if tcfg.noise is not None:
        obs = tcfg.noise.apply(obs)
      if tcfg.clip:
        obs = obs.clip_(min=tcfg.clip[0], max=tcfg.clip[1])
      if tcfg.scale is not None:
        obs = obs.mul_(tcfg.scale)
      if tcfg.delay_max_lag > 0:
        delay = self._group_obs_term_delay_buffer[group_name][tname]
        delay.append(obs)
        obs = delay.compute()
      if tcfg.history_length > 0:
        hist = self._group_obs_term_history_buffer[group_name][tname]
        if update_history or not hist.is_initialized:
          hist.append(obs)
        obs = hist.buffer.reshape(self._env.num_envs, -1) if tcfg.flatten_history_dim else hist.buffer
      obs_terms[tname] = obs
    if self._group_concat[group_name]:
      return torch.cat(list(obs_terms.values()), dim=self._group_concat_dim[group_name])
    return obs_terms

  def _term_input(self, tcfg):
    """The term's value, or an envops.ObsSrc (an elementwise op on strided
    inputs the group kernel evaluates) when the term function offers one."""
    src = getattr(tcfg.func, "obs_src", None)
    if src is not None:
      s = src(self._env, **tcfg.params)
      if s is not None:
        return s
    return tcfg.func(self._env, **tcfg.params).float()

  def _compute_fused(self, fp, u_fixed=None):
    """One fused launch per term writing straight into the group buffer (no
    per-term clone/noise/scale chain, no final cat); one U[0,1) draw per group."""
    from mjlab_amd import envops

    plan, width = fp
    n = self._env.num_envs
    out = torch.empty((n, width), device=self._env.device)
    u, rng = None, None
    if any(p[3] is not None for p in plan):
      if u_fixed is not None:
        u = u_fixed
      else:  # noise drawn inside the group kernel from the env's device stream
        rng = envops.rng_args(self._env, "observation_noise")
    xs = [self._term_input(tcfg) for tcfg, *_ in plan]
    if envops.obs_group(xs, plan, u, out, rng):  # the whole group in one launch
      return out
    if u is None and rng is not None:
      u = torch.rand((n, width), device=self._env.device)
    xs = [x.evaluate() if isinstance(x, envops.ObsSrc) else x for x in xs]
    for x, (tcfg, off, w, noise, clip, scale) in zip(xs, plan):
      lo, hi = noise if noise is not None else (0.0, 0.0)
      uu = u[:, off : off + w] if noise is not None else None
      if not envops.obs_term(x, out[:, off : off + w], uu, lo, hi, clip, scale):
        return None
    return out
