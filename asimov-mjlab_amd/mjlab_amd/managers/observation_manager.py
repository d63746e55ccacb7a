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
    obs_terms = {}
    for tname, tcfg in self._group_terms[group_name]:
      obs = tcfg.func(self._env, **tcfg.params).clone()
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
