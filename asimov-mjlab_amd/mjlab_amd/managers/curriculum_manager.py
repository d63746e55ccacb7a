"""Curriculum manager (``src/mjlab/managers/curriculum_manager.py:20-85``).

Curriculum terms act on host-side schedules (``common_step_counter``); the env
runs them outside the captured device graph, before each step's replay.
"""

from __future__ import annotations

import torch

from mjlab_amd.managers.manager_base import resolve_params


class CurriculumManager:
  def __init__(self, cfg: dict, env) -> None:
    self._env = env
    self.cfg = cfg
    self._term_names, self._term_cfgs = [], []
    for name, tcfg in cfg.items():
      if tcfg is None:
        continue
      resolve_params(env, tcfg)
      if isinstance(tcfg.func, type):
        tcfg.func = tcfg.func(tcfg, env)
      self._term_names.append(name)
      self._term_cfgs.append(tcfg)
    self._curriculum_state: dict[str, object] = {n: None for n in self._term_names}

  @property
  def active_terms(self) -> list[str]:
    return list(self._term_names)

  def reset(self, env_ids=None) -> dict:
    extras = {}
    for name, state in self._curriculum_state.items():
      if state is None:
        continue
      if isinstance(state, dict):
        for k, v in state.items():
          extras[f"Curriculum/{name}/{k}"] = v
      else:
        extras[f"Curriculum/{name}"] = state
    return extras

  def compute(self, env_ids=None) -> None:
    for name, tcfg in zip(self._term_names, self._term_cfgs):
      self._curriculum_state[name] = tcfg.func(self._env, env_ids, **tcfg.params)


class NullCurriculumManager:
  active_terms: list[str] = []

  def reset(self, env_ids=None) -> dict:
    return {}

  def compute(self, env_ids=None) -> None:
    pass
