"""Observation manager (``src/mjlab/managers/observation_manager.py:147-260``).

Pipeline per term: compute -> noise (only if the group enables corruption) ->
clip -> scale -> history; groups concatenated along the last dim.
"""

from __future__ import annotations

import torch

from mjlab_amd.managers.manager_base import as_mask, resolve_params


class ObservationManager:
  def __init__(self, cfg: dict, env) -> None:
    self._env = env
    self.cfg = cfg
    self._group_terms: dict[str, list[tuple[str, object]]] = {}
    self._group_concat: dict[str, bool] = {}
    self._group_concat_dim: dict[str, int] = {}
    self._history: dict[tuple[str, str], torch.Tensor] = {}
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
    # resolve scales and dims by evaluating every term once (observation_manager.py:246)
    self.group_obs_term_dim: dict[str, list[tuple[int, ...]]] = {}
    for gname, terms in self._group_terms.items():
      dims = []
      for tname, tcfg in terms:
        out = tcfg.func(env, **tcfg.params)
        if tcfg.scale is not None and not isinstance(tcfg.scale, torch.Tensor):
          tcfg.scale = torch.tensor(tcfg.scale, dtype=torch.float32, device=env.device)
        if tcfg.history_length > 0:
          h = torch.zeros(env.num_envs, tcfg.history_length, *out.shape[1:], device=env.device)
          self._history[(gname, tname)] = h
        dims.append(tuple(out.shape[1:]))
      self.group_obs_term_dim[gname] = dims
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
      if tcfg.history_length > 0 or len(dims) > 1:
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
    out = {}
    for g, dims in self.group_obs_term_dim.items():
      if self._group_concat[g]:
        out[g] = (sum(int(torch.tensor(d).prod()) for d in dims),)
      else:
        out[g] = dims
    return out

  @property
  def group_obs_concatenate(self) -> dict[str, bool]:
    return dict(self._group_concat)

  def reset(self, env_ids=None) -> dict:
    m = as_mask(env_ids, self._env.num_envs, self._env.device)
    for h in self._history.values():
      h.masked_fill_(m.view(-1, *([1] * (h.dim() - 1))), 0.0)
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
      if tcfg.history_length > 0:
        h = self._history[(group_name, tname)]
        if update_history:
          h.copy_(torch.cat([h[:, 1:], obs.unsqueeze(1)], dim=1))
        obs = h.reshape(self._env.num_envs, -1) if tcfg.flatten_history_dim else h
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
