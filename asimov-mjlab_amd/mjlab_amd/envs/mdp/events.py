"""Event terms (``src/mjlab/envs/mdp/events.py``), mask-based.

``env_ids`` is a boolean mask (or None = all envs). Samples are drawn for all
envs and selected with the mask, so reset/push events never sync the host;
the draws are distributed exactly as the reference's per-subset draws, but the
RNG stream differs ("RNG").
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal

import torch

from mjlab_amd.entity.data import EntityData
from mjlab_amd.managers.manager_base import as_mask
from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from mjlab_amd import envops
from mjlab_amd.envops import quat_mul

_DEFAULT = SceneEntityCfg("robot")
_AXES6 = ["x", "y", "z", "roll", "pitch", "yaw"]


def _ranges6(env, r: dict | None) -> tuple[torch.Tensor, torch.Tensor]:
  key = ("_ranges6", tuple(sorted((r or {}).items())))
  cache = env.__dict__.setdefault("_event_const_cache", {})
  if key not in cache:
    rl = [(r or {}).get(k, (0.0, 0.0)) for k in _AXES6]
    t = torch.tensor(rl, device=env.device, dtype=torch.float32)
    cache[key] = (t[:, 0].clone(), t[:, 1].clone())
  return cache[key]


def _ranges6_host(r: dict | None) -> tuple[list[float], list[float]]:
  rl = [(r or {}).get(k, (0.0, 0.0)) for k in _AXES6]
  return [float(a) for a, _ in rl], [float(b) for _, b in rl]


def _uniform6(env, n, ranges, lo, hi):
  """U(lo, hi) draws for the 6 pose/velocity axes, or None when every range is
  (0, 0): the offsets are then exactly zero and no random kernel is launched."""
  if not ranges or all(tuple(v) == (0.0, 0.0) for v in ranges.values()):
    return None
  return torch.rand(n, 6, device=env.device) * (hi - lo) + lo


def reset_scene_to_default(env, env_ids) -> None:
  m = as_mask(env_ids, env.num_envs, env.device)
  for ent in env.scene.entities.values():
    rs = ent.data.default_root_state.clone()
    rs[:, 0:3] += env.scene.env_origins
    if not ent.is_fixed_base:
      ent.write_root_state_to_sim(rs, env_ids=m)
    if ent.is_articulated:
      ent.write_joint_state_to_sim(ent.data.default_joint_pos.clone(), ent.data.default_joint_vel.clone(), env_ids=m)


def _slice_start(cols):
  """First column of a contiguous column set (EntityData keeps those as slices), else None."""
  return cols.start if isinstance(cols, slice) and cols.step in (None, 1) else None


def _fused_cols(d, prefix: str):
  """(qpos, qvel) start columns of an EntityData's contiguous joint block for the
  fused kernels, else (None, None) (duck-typed entities take the torch path)."""
  if not isinstance(d, EntityData):
    return None, None
  return _slice_start(d._cols[prefix + "_q_adr"]), _slice_start(d._cols[prefix + "_v_adr"])


def _all_range(r) -> bool:
  return bool(r) and not all(tuple(v) == (0.0, 0.0) for v in r.values())


def reset_root_state_uniform(env, env_ids, pose_range: dict, velocity_range: dict | None = None,
                             asset_cfg: SceneEntityCfg = _DEFAULT) -> None:
  m = as_mask(env_ids, env.num_envs, env.device)
  a = env.scene[asset_cfg.name]
  n = env.num_envs
  lo, hi = _ranges6(env, pose_range)
  rs = a.data.default_root_state
  if a.is_fixed_base:
    raise ValueError(f"Cannot reset root state for fixed-base entity '{asset_cfg.name}'.")
  # one launch on the GPU: draws, pose composition and the root pose/velocity
  # writes of EntityData (csrc/mjh_fuse.hip); the torch path below is its reference
  d = a.data
  qa, va = _fused_cols(d, "free_joint")
  if qa is not None and va is not None:
    (plo, phi), (vlo, vhi) = _ranges6_host(pose_range), _ranges6_host(velocity_range)
    if envops.reset_root_uniform(env, f"reset_root_state_uniform.{asset_cfg.name}", d.data.qpos, qa, d.data.qvel, va, m, rs,
                                 env.scene.env_origins, plo, phi, vlo, vhi, _all_range(pose_range), _all_range(velocity_range)):
      return
  pose = _uniform6(env, n, pose_range, lo, hi)
  if pose is None:
    pose = torch.zeros(n, 6, device=env.device)
  pos = rs[:, 0:3] + pose[:, 0:3] + env.scene.env_origins
  quat = quat_mul(rs[:, 3:7], envops.quat_from_euler_xyz(pose[:, 3:6]))
  vlo, vhi = _ranges6(env, velocity_range)
  dv = _uniform6(env, n, velocity_range, vlo, vhi)
  vel = rs[:, 7:13] if dv is None else rs[:, 7:13] + dv
  a.write_root_link_pose_to_sim(torch.cat([pos, quat], dim=-1), env_ids=m)
  a.write_root_link_velocity_to_sim(vel, env_ids=m)


def reset_joints_by_offset(env, env_ids, position_range: tuple[float, float], velocity_range: tuple[float, float],
                           asset_cfg: SceneEntityCfg = _DEFAULT) -> None:
  m = as_mask(env_ids, env.num_envs, env.device)
  a = env.scene[asset_cfg.name]
  j = asset_cfg.joint_idx
  d = a.data
  if isinstance(j, slice) and j == slice(None) and isinstance(d, EntityData):  # all joints: one fused launch
    qa, va = _slice_start(d._cols["joint_q_adr"]), _slice_start(d._cols["joint_v_adr"])
    if qa is not None and va is not None and envops.reset_joints_offset(
        env, f"reset_joints_by_offset.{asset_cfg.name}", d.data.qpos, qa, d.data.qvel, va, m, d.default_joint_pos,
        d.default_joint_vel, d.soft_joint_pos_limits, position_range, velocity_range):
      return
  jp = a.data.default_joint_pos[:, j].clone()
  if tuple(position_range) != (0.0, 0.0):  # (0, 0): exact zero offset, no draw
    jp += torch.rand_like(jp) * (position_range[1] - position_range[0]) + position_range[0]
  lim = a.data.soft_joint_pos_limits[:, j]
  jp = jp.clamp_(lim[..., 0], lim[..., 1])
  jv = a.data.default_joint_vel[:, j].clone()
  if tuple(velocity_range) != (0.0, 0.0):
    jv += torch.rand_like(jv) * (velocity_range[1] - velocity_range[0]) + velocity_range[0]
  a.write_joint_state_to_sim(jp, jv, env_ids=m, joint_ids=None if isinstance(j, slice) else j)


def push_by_setting_velocity(env, env_ids, velocity_range: dict, asset_cfg: SceneEntityCfg = _DEFAULT) -> None:
  m = as_mask(env_ids, env.num_envs, env.device)
  a = env.scene[asset_cfg.name]
  lo, hi = _ranges6(env, velocity_range)
  d = a.data
  qa, va = _fused_cols(d, "free_joint")
  if qa is not None and va is not None and envops.push_velocity(
      env, f"push_by_setting_velocity.{asset_cfg.name}", d.data.qpos, qa, d.data.qvel, va, m, d.root_link_vel_w,
      *_ranges6_host(velocity_range)):
    return
  vel = a.data.root_link_vel_w + torch.rand(env.num_envs, 6, device=env.device) * (hi - lo) + lo
  a.write_root_link_velocity_to_sim(vel, env_ids=m)


def apply_external_force_torque(env, env_ids, force_range, torque_range, asset_cfg: SceneEntityCfg = _DEFAULT) -> None:
  m = as_mask(env_ids, env.num_envs, env.device)
  a = env.scene[asset_cfg.name]
  nb = len(asset_cfg.body_ids) if isinstance(asset_cfg.body_ids, list) else a.num_bodies
  f = torch.rand(env.num_envs, nb, 3, device=env.device) * (force_range[1] - force_range[0]) + force_range[0]
  t = torch.rand(env.num_envs, nb, 3, device=env.device) * (torque_range[1] - torque_range[0]) + torque_range[0]
  a.write_external_wrench_to_sim(f, t, env_ids=m, body_ids=asset_cfg.body_idx)


@dataclass
class FieldSpec:
  entity_type: Literal["dof", "joint", "body", "geom", "site", "actuator"]
  use_address: bool = False
  default_axes: list[int] | None = None
  valid_axes: list[int] | None = None


FIELD_SPECS = {
  "dof_armature": FieldSpec("dof", use_address=True),
  "dof_frictionloss": FieldSpec("dof", use_address=True),
  "dof_damping": FieldSpec("dof", use_address=True),
  "jnt_range": FieldSpec("joint"),
  "jnt_stiffness": FieldSpec("joint"),
  "body_mass": FieldSpec("body"),
  "body_ipos": FieldSpec("body", default_axes=[0, 1, 2]),
  "body_iquat": FieldSpec("body", default_axes=[0, 1, 2, 3]),
  "body_inertia": FieldSpec("body"),
  "body_pos": FieldSpec("body", default_axes=[0, 1, 2]),
  "body_quat": FieldSpec("body", default_axes=[0, 1, 2, 3]),
  "geom_friction": FieldSpec("geom", default_axes=[0], valid_axes=[0, 1, 2]),
  "geom_pos": FieldSpec("geom", default_axes=[0, 1, 2]),
  "geom_quat": FieldSpec("geom", default_axes=[0, 1, 2, 3]),
  "geom_rgba": FieldSpec("geom", default_axes=[0, 1, 2, 3]),
  "site_pos": FieldSpec("site", default_axes=[0, 1, 2]),
  "site_quat": FieldSpec("site", default_axes=[0, 1, 2, 3]),
  "qpos0": FieldSpec("joint", use_address=True),
}


def _entity_indices(ix, asset_cfg, spec: FieldSpec) -> torch.Tensor:
  t = spec.entity_type
  if t == "dof":
    return ix.joint_v_adr[asset_cfg.joint_ids]
  if t == "joint" and spec.use_address:
    return ix.joint_q_adr[asset_cfg.joint_ids]
  if t == "joint":
    return ix.joint_ids[asset_cfg.joint_ids]
  if t == "body":
    return ix.body_ids[asset_cfg.body_ids]
  if t == "geom":
    return ix.geom_ids[asset_cfg.geom_ids]
  if t == "site":
    return ix.site_ids[asset_cfg.site_ids]
  return ix.ctrl_ids


def randomize_field(env, env_ids, field: str, ranges, distribution: str = "uniform", operation: str = "abs",
                    asset_cfg=None, axes: list[int] | None = None) -> None:
  """Per-world model randomisation (events.py:256-395). Runs at startup/reset,
  outside the captured step; ``field`` must have been expanded per world."""
  if field not in FIELD_SPECS:
    raise ValueError(f"Unknown field '{field}'. Supported fields: {list(FIELD_SPECS)}")
  spec = FIELD_SPECS[field]
  asset_cfg = asset_cfg or _DEFAULT
  a = env.scene[asset_cfg.name]
  m = as_mask(env_ids, env.num_envs, env.device)
  env_idx = m.nonzero().flatten()  # startup/reset-time only (never captured)
  model_field = getattr(env.sim.model, field)
  ent = _entity_indices(a.indexing, asset_cfg, spec).long()
  ndim = model_field.dim() - 1
  if axes is not None:
    target = axes
  elif isinstance(ranges, dict):
    target = list(ranges.keys())
  elif spec.default_axes is not None:
    target = spec.default_axes
  else:
    target = list(range(model_field.shape[-1])) if ndim > 1 else [0]
  if spec.valid_axes is not None and set(target) - set(spec.valid_axes):
    raise ValueError(f"Invalid axes {set(target) - set(spec.valid_axes)} for field. Valid axes: {spec.valid_axes}")
  axis_ranges = {ax: ranges for ax in target} if isinstance(ranges, tuple) else {ax: ranges[ax] for ax in target}
  eg, ng = torch.meshgrid(env_idx, ent, indexing="ij")
  data = model_field[eg, ng]
  result = data.clone()
  for ax in target:
    lo, hi = axis_ranges[ax]
    shape = (*data.shape[:-1], 1) if data.dim() > 2 else data.shape
    if distribution == "uniform":
      # bounds as float32 tensors, as the reference (events.py:405-406), so the
      # range is rounded the same way
      lo_t = torch.tensor([lo], device=env.device)
      hi_t = torch.tensor([hi], device=env.device)
      vals = torch.rand(shape, device=env.device) * (hi_t - lo_t) + lo_t
    elif distribution == "log_uniform":
      vals = torch.exp(torch.rand(shape, device=env.device) * (torch.log(torch.tensor(hi)) - torch.log(torch.tensor(lo))) + torch.log(torch.tensor(lo)))
    elif distribution == "gaussian":
      vals = torch.randn(shape, device=env.device) * hi + lo
    else:
      raise ValueError(f"Unknown distribution: {distribution}")
    if data.dim() > 2:
      result[..., ax] = vals.squeeze(-1)
    else:
      result = vals
  if operation == "add":
    model_field[eg, ng] = data + result
  elif operation == "scale":
    model_field[eg, ng] = data * result
  elif operation == "abs":
    model_field[eg, ng] = result
  else:
    raise ValueError(f"Unknown operation: {operation}")
