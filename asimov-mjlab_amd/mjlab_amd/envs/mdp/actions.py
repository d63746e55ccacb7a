"""Joint actions (``src/mjlab/envs/mdp/actions/joint_actions.py:18-108``)."""

from __future__ import annotations

from dataclasses import dataclass

import torch

from mjlab_amd.managers.action_manager import ActionTerm
from mjlab_amd.managers.manager_base import as_mask
from mjlab_amd.managers.manager_term_config import ActionTermCfg
from mjlab_amd.utils.string import resolve_matching_names_values


class JointAction(ActionTerm):
  def __init__(self, cfg, env) -> None:
    super().__init__(cfg, env)
    act_ids, self._actuator_names = self._asset.find_actuators(cfg.actuator_names, preserve_order=cfg.preserve_order)
    joint_ids, _ = self._asset.find_joints(self._actuator_names, preserve_order=cfg.preserve_order)
    self._actuator_ids = torch.tensor(act_ids, device=self.device, dtype=torch.long)
    self._joint_ids = torch.tensor(joint_ids, device=self.device, dtype=torch.long)
    self._action_dim = len(act_ids)
    self._raw_actions = torch.zeros(self.num_envs, self._action_dim, device=self.device)
    self._processed_actions = torch.zeros_like(self._raw_actions)
    if isinstance(cfg.scale, (float, int)):
      self._scale = float(cfg.scale)
    else:
      self._scale = torch.ones(self.num_envs, self._action_dim, device=self.device)
      idx, _, vals = resolve_matching_names_values(cfg.scale, self._actuator_names)
      self._scale[:, idx] = torch.tensor(vals, device=self.device)
    if isinstance(cfg.offset, (float, int)):
      self._offset = float(cfg.offset)
    else:
      self._offset = torch.zeros_like(self._raw_actions)
      idx, _, vals = resolve_matching_names_values(cfg.offset, self._actuator_names)
      self._offset[:, idx] = torch.tensor(vals, device=self.device)

  @property
  def action_dim(self) -> int:
    return self._action_dim

  @property
  def raw_action(self) -> torch.Tensor:
    return self._raw_actions

  @property
  def scale(self):
    return self._scale

  @property
  def offset(self):
    return self._offset

  def process_actions(self, actions: torch.Tensor) -> None:
    self._raw_actions.copy_(actions)
    # processed = raw * scale + offset (joint_actions.py:62-64), one fused launch
    if isinstance(self._scale, torch.Tensor):
      off = self._offset if isinstance(self._offset, torch.Tensor) else torch.full_like(self._raw_actions, self._offset)
      torch.addcmul(off, self._raw_actions, self._scale, out=self._processed_actions)
    elif isinstance(self._offset, torch.Tensor):
      torch.add(self._offset, self._raw_actions, alpha=self._scale, out=self._processed_actions)
    else:
      torch.mul(self._raw_actions, self._scale, out=self._processed_actions).add_(self._offset)

  def reset(self, env_ids=None) -> None:
    self._raw_actions.masked_fill_(as_mask(env_ids, self.num_envs, self.device)[:, None], 0.0)


class JointPositionAction(JointAction):
  # apply_actions writes the same processed targets at every physics substep of an
  # env step and nothing else writes ctrl between substeps, so the env applies it
  # once per env step (the later writes would store identical values)
  apply_is_idempotent = True

  def __init__(self, cfg, env) -> None:
    super().__init__(cfg, env)
    if cfg.use_default_offset:
      self._offset = self._asset.data.default_joint_pos[:, self._joint_ids].clone()

  def apply_actions(self) -> None:
    self._asset.write_joint_position_target_to_sim(self._processed_actions, self._actuator_ids)


@dataclass(kw_only=True)
class JointActionCfg(ActionTermCfg):
  actuator_names: tuple[str, ...]
  scale: float | dict[str, float] = 1.0
  offset: float | dict[str, float] = 0.0
  preserve_order: bool = False


@dataclass(kw_only=True)
class JointPositionActionCfg(JointActionCfg):
  class_type: type = JointPositionAction
  use_default_offset: bool = True
