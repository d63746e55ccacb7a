"""Velocity-task rewards (``src/mjlab/tasks/velocity/mdp/rewards.py``).

Same formulas as the reference; stateful terms update their state in place
(``copy_``) so the captured env-step graph carries it across replays.
"""

from __future__ import annotations

import torch

from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from mjlab_amd import envops
from mjlab_amd.envops import quat_apply_inverse
from mjlab_amd.utils.string import resolve_matching_names_values

_DEFAULT = SceneEntityCfg("robot")


def _command_active(env, command_name, threshold) -> torch.Tensor | None:
  """(|cmd_xy| + |cmd_yaw| > threshold) as float. The command does not change
  while rewards are computed, so terms sharing (command, threshold) share one
  evaluation per reward pass (the reward manager clears the cache)."""
  if command_name is None:
    return None
  command = env.command_manager.get_command(command_name)
  if command is None:
    return None
  cache = env.__dict__.get("_command_active_cache")  # present only during a reward pass
  key = (command_name, float(threshold))
  v = cache.get(key) if cache is not None else None
  if v is None:
    total = torch.norm(command[:, :2], dim=1) + torch.abs(command[:, 2])
    v = (total > threshold).float()
    if cache is not None:
      cache[key] = v
  return v


def track_linear_velocity(env, std: float, command_name: str, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  command = env.command_manager.get_command(command_name)
  actual = env.scene[asset_cfg.name].data.root_link_lin_vel_b
  fused = envops.rew_track(command, actual, std, angular=False)
  if fused is not None:
    return fused
  err = torch.sum(torch.square(command[:, :2] - actual[:, :2]), dim=1) + torch.square(actual[:, 2])
  return torch.exp(-err / std**2)


def track_angular_velocity(env, std: float, command_name: str, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  command = env.command_manager.get_command(command_name)
  actual = env.scene[asset_cfg.name].data.root_link_ang_vel_b
  fused = envops.rew_track(command, actual, std, angular=True)
  if fused is not None:
    return fused
  err = torch.square(command[:, 2] - actual[:, 2]) + torch.sum(torch.square(actual[:, :2]), dim=1)
  return torch.exp(-err / std**2)


def flat_orientation(env, std: float, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  a = env.scene[asset_cfg.name]
  if asset_cfg.body_ids and not isinstance(asset_cfg.body_ids, slice):
    q = a.data.body_link_quat_w[:, asset_cfg.body_idx, :].squeeze(1)
    fused = envops.rew_flat_orientation(q, a.data.gravity_vec_w, std)
    if fused is not None:
      return fused
    g = quat_apply_inverse(q, a.data.gravity_vec_w)
    xy = torch.sum(torch.square(g[:, :2]), dim=1)
  else:
    xy = torch.sum(torch.square(a.data.projected_gravity_b[:, :2]), dim=1)
  return torch.exp(-xy / std**2)


def self_collision_cost(env, sensor_name: str) -> torch.Tensor:
  return env.scene[sensor_name].data.found.squeeze(-1)


def body_angular_velocity_penalty(env, asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  w = env.scene[asset_cfg.name].data.body_link_ang_vel_w[:, asset_cfg.body_idx, :].squeeze(1)
  fused = envops.rew_sqsum(w, 2)
  return fused if fused is not None else torch.sum(torch.square(w[:, :2]), dim=1)


def angular_momentum_penalty(env, sensor_name: str) -> torch.Tensor:
  h = env.scene[sensor_name].data
  sq = envops.rew_sqsum(h, 3) if h.dim() == 2 and h.shape[1] == 3 else None
  sq = sq if sq is not None else torch.sum(torch.square(h), dim=-1)
  envops.log_ratio(env, "Metrics/angular_momentum_mean", sq, None)  # mean(sqrt(sq)), with the pass's other logs
  return sq


def _cmd(env, command_name):
  return env.command_manager.get_command(command_name) if command_name is not None else None


def feet_air_time(env, sensor_name: str, threshold_min: float = 0.05, threshold_max: float = 0.5,
                  command_name: str | None = None, command_threshold: float = 0.5) -> torch.Tensor:
  t = env.scene[sensor_name].data.current_air_time
  fused = envops.rew_air_time(t, _cmd(env, command_name), threshold_min, threshold_max, command_threshold)
  if fused is not None:
    out, num, den = fused
    envops.log_ratio(env, "Metrics/air_time_mean", num, den)
    return out
  reward = torch.sum(((t > threshold_min) & (t < threshold_max)).float(), dim=1)
  in_air = (t > 0).float()
  env.extras["log"]["Metrics/air_time_mean"] = torch.sum(t * in_air) / torch.clamp(torch.sum(in_air), min=1)
  active = _command_active(env, command_name, command_threshold)
  return reward * active if active is not None else reward


def feet_clearance(env, target_height: float, command_name: str | None = None, command_threshold: float = 0.01,
                   asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  a = env.scene[asset_cfg.name]
  if command_name is not None and env.command_manager.get_command(command_name) is not None:
    fused = envops.rew_feet(a.data.site_pos_w[:, asset_cfg.site_idx], a.data.site_lin_vel_w[:, asset_cfg.site_idx], None,
                            env.command_manager.get_command(command_name), target_height, command_threshold, 0.0, "clearance")
    if fused is not None:
      return fused
  z = a.data.site_pos_w[:, asset_cfg.site_idx, 2]
  v = torch.norm(a.data.site_lin_vel_w[:, asset_cfg.site_idx, :2], dim=-1)
  cost = torch.sum(torch.abs(z - target_height) * v, dim=1)
  active = _command_active(env, command_name, command_threshold)
  return cost * active if active is not None else cost


class feet_swing_height:
  def __init__(self, cfg, env) -> None:
    self.sensor_name = cfg.params["sensor_name"]
    self.site_names = cfg.params["asset_cfg"].site_names
    self.peak_heights = torch.zeros((env.num_envs, len(self.site_names)), device=env.device, dtype=torch.float32)
    self.step_dt = env.step_dt

  def __call__(self, env, sensor_name: str, target_height: float, command_name: str, command_threshold: float,
               asset_cfg: SceneEntityCfg) -> torch.Tensor:
    a = env.scene[asset_cfg.name]
    cs = env.scene[sensor_name]
    h = a.data.site_pos_w[:, asset_cfg.site_idx, 2]
    d = cs.data
    fused = envops.rew_swing_height(self.peak_heights, h, d.found, d.current_contact_time, _cmd(env, command_name),
                                    self.step_dt + 1.0e-8, target_height, command_threshold)
    if fused is not None:
      cost, num, den = fused
      envops.log_ratio(env, "Metrics/peak_height_mean", num, den)
      return cost
    in_air = cs.data.found == 0
    torch.where(in_air, torch.maximum(self.peak_heights, h), self.peak_heights, out=self.peak_heights)
    first = cs.compute_first_contact(dt=self.step_dt)
    active = _command_active(env, command_name, command_threshold)
    err = self.peak_heights / target_height - 1.0
    cost = torch.sum(torch.square(err) * first.float(), dim=1) * active
    n = torch.sum(first.float())
    env.extras["log"]["Metrics/peak_height_mean"] = torch.sum(self.peak_heights * first.float()) / torch.clamp(n, min=1)
    self.peak_heights.masked_fill_(first, 0.0)
    return cost


def feet_slip(env, sensor_name: str, command_name: str, command_threshold: float = 0.01,
              asset_cfg: SceneEntityCfg = _DEFAULT) -> torch.Tensor:
  a = env.scene[asset_cfg.name]
  cs = env.scene[sensor_name]
  found = cs.data.found
  fused = envops.rew_feet(a.data.site_pos_w[:, asset_cfg.site_idx], a.data.site_lin_vel_w[:, asset_cfg.site_idx],
                          found, env.command_manager.get_command(command_name), 0.0, 0.0, command_threshold, "slip")
  if fused is not None:
    cost, vsum, cnt = fused
    envops.log_ratio(env, "Metrics/slip_velocity_mean", vsum, cnt)
    return cost
  active = _command_active(env, command_name, command_threshold)
  in_contact = (found > 0).float()
  v = torch.norm(a.data.site_lin_vel_w[:, asset_cfg.site_idx, :2], dim=-1)
  cost = torch.sum(torch.square(v) * in_contact, dim=1) * active
  env.extras["log"]["Metrics/slip_velocity_mean"] = torch.sum(v * in_contact) / torch.clamp(torch.sum(in_contact), min=1)
  return cost


def soft_landing(env, sensor_name: str, command_name: str | None = None, command_threshold: float = 0.05) -> torch.Tensor:
  cs = env.scene[sensor_name]
  d = cs.data
  fused = envops.rew_soft_landing(d.force, d.current_contact_time, _cmd(env, command_name), env.step_dt + 1.0e-8,
                                  command_threshold)
  if fused is not None:
    cost, num, den = fused
    envops.log_ratio(env, "Metrics/landing_force_mean", num, den)
    return cost
  fm = torch.norm(cs.data.force, dim=-1)
  first = cs.compute_first_contact(dt=env.step_dt)
  impact = fm * first.float()
  cost = torch.sum(impact, dim=1)
  env.extras["log"]["Metrics/landing_force_mean"] = torch.sum(impact) / torch.clamp(torch.sum(first.float()), min=1)
  active = _command_active(env, command_name, command_threshold)
  return cost * active if active is not None else cost


class variable_posture:
  def __init__(self, cfg, env) -> None:
    a = env.scene[cfg.params["asset_cfg"].name]
    self.default_joint_pos = a.data.default_joint_pos
    _, names = a.find_joints(cfg.params["asset_cfg"].joint_names)

    def T(key):
      _, _, v = resolve_matching_names_values(data=cfg.params[key], list_of_strings=names)
      return torch.tensor(v, device=env.device, dtype=torch.float32)

    self.std_standing = T("std_standing")
    self.std_walking = T("std_walking")
    self.std_running = T("std_running")

  def __call__(self, env, std_standing, std_walking, std_running, asset_cfg: SceneEntityCfg, command_name: str,
               walking_threshold: float = 0.5, running_threshold: float = 1.5) -> torch.Tensor:
    del std_standing, std_walking, std_running
    a = env.scene[asset_cfg.name]
    command = env.command_manager.get_command(command_name)
    if isinstance(asset_cfg.joint_idx, slice) and asset_cfg.joint_idx == slice(None):
      fused = envops.rew_posture(a.data.joint_pos, self.default_joint_pos, self.std_standing, self.std_walking,
                                 self.std_running, command, walking_threshold, running_threshold)
      if fused is not None:
        return fused
    total = torch.norm(command[:, :2], dim=1) + torch.abs(command[:, 2])
    standing = (total < walking_threshold).float()
    walking = ((total >= walking_threshold) & (total < running_threshold)).float()
    running = (total >= running_threshold).float()
    std = (
      self.std_standing * standing.unsqueeze(1)
      + self.std_walking * walking.unsqueeze(1)
      + self.std_running * running.unsqueeze(1)
    )
    err = torch.square(a.data.joint_pos[:, asset_cfg.joint_idx] - self.default_joint_pos[:, asset_cfg.joint_idx])
    return torch.exp(-torch.mean(err / (std**2), dim=1))
