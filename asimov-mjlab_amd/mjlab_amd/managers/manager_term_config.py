"""Manager term configurations (``src/mjlab/managers/manager_term_config.py``)."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Literal

EventMode = Literal["startup", "reset", "interval"]


@dataclass
class ManagerTermBaseCfg:
  func: Any
  params: dict[str, Any] = field(default_factory=dict)


@dataclass(kw_only=True)
class ActionTermCfg:
  class_type: type
  asset_name: str
  clip: dict[str, tuple] | None = None


@dataclass(kw_only=True)
class CommandTermCfg:
  class_type: type
  resampling_time_range: tuple[float, float]
  debug_vis: bool = False


@dataclass(kw_only=True)
class CurriculumTermCfg(ManagerTermBaseCfg):
  pass


@dataclass(kw_only=True)
class EventTermCfg(ManagerTermBaseCfg):
  mode: EventMode
  interval_range_s: tuple[float, float] | None = None
  is_global_time: bool = False
  min_step_count_between_reset: int = 0
  domain_randomization: bool = False


@dataclass
class ObservationTermCfg(ManagerTermBaseCfg):
  """Pipeline: compute -> noise -> clip -> scale -> delay -> history
  (observation_manager.py:163-188)."""

  noise: Any = None
  clip: tuple[float, float] | None = None
  scale: Any = None
  delay_min_lag: int = 0
  delay_max_lag: int = 0
  delay_per_env: bool = True
  delay_hold_prob: float = 0.0
  delay_update_period: int = 0
  delay_per_env_phase: bool = True
  history_length: int = 0
  flatten_history_dim: bool = True


@dataclass
class ObservationGroupCfg:
  terms: dict[str, ObservationTermCfg]
  concatenate_terms: bool = True
  concatenate_dim: int = -1
  enable_corruption: bool = False
  history_length: int | None = None
  flatten_history_dim: bool = True


@dataclass(kw_only=True)
class RewardTermCfg(ManagerTermBaseCfg):
  func: Any
  weight: float


@dataclass
class TerminationTermCfg(ManagerTermBaseCfg):
  time_out: bool = False
