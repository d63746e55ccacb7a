"""EntityData: state writes and derived reads on the batched sim data.

Restates ``src/mjlab/entity/data.py``. Writes index ``sim.data.<field>`` torch
views in place (``data.py:75-198``); reads derive poses and velocities from the
kinematics outputs of the last forward pass (``data.py:212-528``), including
``compute_velocity_from_cvel`` (``data.py:20-31``) and the convention that body,
geom and site velocities use the *root* subtree com (``data.py:264,282,306,325``).

Writes of a subset of envs use a boolean mask + ``torch.where`` when ``env_ids``
is a bool tensor, so the env loop stays capturable (no ``nonzero`` syncs).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any

import torch

from mjlab_amd import envops
from mjlab_amd.envops import quat_apply, quat_apply_inverse, quat_mul
from mjlab_amd.utils.math import quat_from_matrix


def compute_velocity_from_cvel(pos: torch.Tensor, subtree_com: torch.Tensor, cvel: torch.Tensor) -> torch.Tensor:
  lin_vel_c = cvel[..., 3:6]
  ang_vel_c = cvel[..., 0:3]
  offset = subtree_com - pos
  lin_vel_w = lin_vel_c - torch.cross(ang_vel_c, offset, dim=-1)
  return torch.cat([lin_vel_w, ang_vel_c], dim=-1)


def _cached(fn):
  """Property cached until the sim's forward outputs change (sim.epoch bumps
  on every step/forward). Only quantities derived from forward outputs (poses,
  cvel, subtree_com) are cached — never raw state like qpos/qvel, which
  callers may write directly. Values are identical to recomputing; inside a
  captured env step this removes repeated gathers/quaternion maths."""
  name = fn.__name__

  def get(self):
    ep = self.data.epoch.v
    d = self.__dict__
    if d.get("_cache_ep") != ep:
      d["_cache"] = {}
      d["_cache_ep"] = ep
    c = d["_cache"]
    v = c.get(name)
    if v is None:
      v = fn(self)
      c[name] = v
    return v

  get.__doc__ = fn.__doc__
  return property(get)


def _masked_write(dst: torch.Tensor, cols: torch.Tensor | slice, value: torch.Tensor, env_ids) -> None:
  """dst[env_ids, cols] = value, for env_ids None/slice/index tensor/bool mask."""
  if env_ids is None or isinstance(env_ids, slice):
    rows = env_ids if env_ids is not None else slice(None)
    if isinstance(cols, slice):
      dst[rows, cols] = value
    else:
      dst[rows, cols.long()] = value
    return
  if env_ids.dtype == torch.bool:
    m = env_ids.view(-1, *([1] * (dst.dim() - 1)))
    if isinstance(cols, slice):  # in place on the strided view: where + copy, no gather/scatter
      cur = dst[:, cols]
      torch.where(m, value, cur, out=cur)
      return
    cols_l = cols.long()
    cur = dst[:, cols_l]
    value = value.expand_as(cur) if value.dim() <= cur.dim() else value
    dst[:, cols_l] = torch.where(m, value, cur)
    return
  idx = env_ids.long()[:, None]
  cols_l = torch.arange(dst.shape[1], device=dst.device)[cols] if isinstance(cols, slice) else cols.long()
  dst[idx, cols_l] = value


def _as_slice(idx: torch.Tensor):
  """slice(a, b) if idx == arange(a, b) (checked once, at init), else idx."""
  if idx.numel() == 0:
    return idx
  h = idx.detach().cpu()
  a = int(h[0])
  if torch.equal(h, torch.arange(a, a + h.numel(), dtype=h.dtype)):
    return slice(a, a + h.numel())
  return idx


@dataclass
class EntityData:
  indexing: Any
  data: Any
  model: Any
  device: str
  default_root_state: torch.Tensor
  default_joint_pos: torch.Tensor
  default_joint_vel: torch.Tensor
  default_joint_stiffness: torch.Tensor
  default_joint_damping: torch.Tensor
  default_joint_pos_limits: torch.Tensor
  joint_pos_limits: torch.Tensor
  soft_joint_pos_limits: torch.Tensor
  gravity_vec_w: torch.Tensor
  forward_vec_b: torch.Tensor
  is_fixed_base: bool
  is_articulated: bool
  is_actuated: bool

  def __post_init__(self) -> None:
    # int64 copies of the index tensors, made once: `.long()` on the int32
    # originals would launch a conversion kernel on every access
    ix = self.indexing
    self._ix = {
      k: getattr(ix, k).long()
      for k in ("body_ids", "geom_ids", "site_ids", "ctrl_ids", "joint_ids", "joint_q_adr", "joint_v_adr",
                "free_joint_q_adr", "free_joint_v_adr")
    }
    self._ix["geom_bodyid"] = self.model.geom_bodyid[self._ix["geom_ids"]].long()
    self._ix["site_bodyid"] = self.model.site_bodyid[self._ix["site_ids"]].long()
    self._ix["root_quat_adr"] = self._ix["free_joint_q_adr"][3:7]
    # column sets that are contiguous ranges (the usual case: one entity's
    # joints/dofs/actuators/bodies are consecutive) are written through slices
    self._cols = {k: _as_slice(v) for k, v in self._ix.items()}
    gb = self._ix["body_ids"]
    wcols = (gb[:, None] * 6 + torch.arange(6, device=gb.device)).reshape(-1)
    self._cols["xfrc_all"] = _as_slice(wcols)
    self._cols["xfrc_force"] = _as_slice((gb[:, None] * 6 + torch.arange(3, device=gb.device)).reshape(-1))
    self._cols["xfrc_torque"] = _as_slice((gb[:, None] * 6 + 3 + torch.arange(3, device=gb.device)).reshape(-1))

  ROOT_POSE_DIM = 7
  ROOT_VEL_DIM = 6
  ROOT_STATE_DIM = 13

  # ---- writes ----
  def write_root_state(self, root_state: torch.Tensor, env_ids=None) -> None:
    if self.is_fixed_base:
      raise ValueError("Cannot write root state for fixed-base entity.")
    assert root_state.shape[-1] == self.ROOT_STATE_DIM
    self.write_root_pose(root_state[:, :7], env_ids)
    self.write_root_velocity(root_state[:, 7:], env_ids)

  def write_root_pose(self, pose: torch.Tensor, env_ids=None) -> None:
    if self.is_fixed_base:
      raise ValueError("Cannot write root pose for fixed-base entity.")
    assert pose.shape[-1] == self.ROOT_POSE_DIM
    _masked_write(self.data.qpos, self._cols["free_joint_q_adr"], pose, env_ids)

  def write_root_velocity(self, velocity: torch.Tensor, env_ids=None) -> None:
    if self.is_fixed_base:
      raise ValueError("Cannot write root velocity for fixed-base entity.")
    assert velocity.shape[-1] == self.ROOT_VEL_DIM
    qadr = self._ix["root_quat_adr"]
    if env_ids is None or isinstance(env_ids, slice) or env_ids.dtype == torch.bool:
      quat_w = self.data.qpos[:, qadr] if not isinstance(env_ids, slice) else self.data.qpos[env_ids][:, qadr]
    else:
      quat_w = self.data.qpos[env_ids.long()][:, qadr]
    if velocity.shape[0] != quat_w.shape[0]:
      velocity = velocity.expand(quat_w.shape[0], -1)
    ang_b = quat_apply_inverse(quat_w, velocity[:, 3:])
    qv = torch.cat([velocity[:, :3], ang_b], dim=-1)
    _masked_write(self.data.qvel, self._cols["free_joint_v_adr"], qv, env_ids)

  def write_mocap_pose(self, pose: torch.Tensor, env_ids=None) -> None:
    """Mocap body pose (pos 3, quat 4) of a mocap entity (data.py:178-187)."""
    mid = self.indexing.mocap_id
    if mid is None:
      raise ValueError("Cannot write mocap pose for non-mocap entity.")
    assert pose.shape[-1] == 7
    n = self.data.qpos.shape[0]
    _masked_write(self.data.mocap_pos.view(n, -1), slice(3 * mid, 3 * mid + 3), pose[:, 0:3], env_ids)
    _masked_write(self.data.mocap_quat.view(n, -1), slice(4 * mid, 4 * mid + 4), pose[:, 3:7], env_ids)

  def write_joint_state(self, position, velocity, joint_ids=None, env_ids=None) -> None:
    if not self.is_articulated:
      raise ValueError("Cannot write joint state for non-articulated entity.")
    self.write_joint_position(position, joint_ids, env_ids)
    self.write_joint_velocity(velocity, joint_ids, env_ids)

  def write_joint_position(self, position, joint_ids=None, env_ids=None) -> None:
    if not self.is_articulated:
      raise ValueError("Cannot write joint position for non-articulated entity.")
    cols = self._cols["joint_q_adr"] if joint_ids is None else self._ix["joint_q_adr"][joint_ids]
    _masked_write(self.data.qpos, cols, position, env_ids)

  def write_joint_velocity(self, velocity, joint_ids=None, env_ids=None) -> None:
    if not self.is_articulated:
      raise ValueError("Cannot write joint velocity for non-articulated entity.")
    cols = self._cols["joint_v_adr"] if joint_ids is None else self._ix["joint_v_adr"][joint_ids]
    _masked_write(self.data.qvel, cols, velocity, env_ids)

  def write_external_wrench(self, force, torque, body_ids=None, env_ids=None) -> None:
    xf = self.data.xfrc_applied
    flat = xf.view(xf.shape[0], -1)
    if body_ids is None:
      fcols, tcols = self._cols["xfrc_force"], self._cols["xfrc_torque"]
    else:
      gb = self._ix["body_ids"][body_ids]
      fcols = (gb[:, None] * 6 + torch.arange(3, device=gb.device)).reshape(-1)
      tcols = fcols + 3
    if force is not None:
      _masked_write(flat, fcols, force.reshape(force.shape[0], -1), env_ids)
    if torque is not None:
      _masked_write(flat, tcols, torque.reshape(torque.shape[0], -1), env_ids)

  def write_ctrl(self, ctrl: torch.Tensor, ctrl_ids=None, env_ids=None) -> None:
    if not self.is_actuated:
      raise ValueError("Cannot write control for non-actuated entity.")
    cols = self._cols["ctrl_ids"] if ctrl_ids is None else self._sub_cols("ctrl_ids", ctrl_ids)
    _masked_write(self.data.ctrl, cols, ctrl, env_ids)

  def _sub_cols(self, key: str, ids):
    """Columns self._ix[key][ids], as a slice when contiguous. Resolved once per
    ids object outside graph capture (the action terms pass the same ids every
    step), so a per-step write is one copy instead of a gather + scatter."""
    cache = self.__dict__.setdefault("_sub_cols_cache", {})
    ck = (key, id(ids)) if isinstance(ids, torch.Tensor) else (key, repr(ids))
    hit = cache.get(ck)
    if hit is not None and (hit[0] is ids or not isinstance(ids, torch.Tensor)):
      return hit[1]
    cols = self._ix[key][ids]
    capturing = cols.is_cuda and torch.cuda.is_current_stream_capturing()
    if not capturing and cols.dim() == 1:
      cols = _as_slice(cols)
      cache[ck] = (ids, cols)
    return cols

  def clear_state(self, env_ids=None) -> None:
    """Zero applied generalized forces on the free joint, applied body wrenches
    and controls of this entity (data.py:186-198)."""
    n = self.data.qpos.shape[0]
    if env_ids is not None and not isinstance(env_ids, slice) and env_ids.dtype == torch.bool:
      m = env_ids[:, None]
      xf = self.data.xfrc_applied.view(n, -1)
      views = [self.data.qfrc_applied[:, self._cols["free_joint_v_adr"]], xf[:, self._cols["xfrc_all"]]]
      if self.is_actuated:
        views.append(self.data.ctrl[:, self._cols["ctrl_ids"]])
      if all(isinstance(self._cols[k], slice) for k in ("free_joint_v_adr", "xfrc_all", "ctrl_ids")) and envops.masked_zero(
          [v for v in views if v.shape[1] > 0], env_ids):
        return  # one launch for the applied forces, wrenches and controls
      for dst, key in ((self.data.qfrc_applied, "free_joint_v_adr"), (xf, "xfrc_all"), (self.data.ctrl, "ctrl_ids")):
        cols = self._cols[key]
        if key == "ctrl_ids" and not self.is_actuated:
          continue
        if isinstance(cols, slice):
          dst[:, cols].masked_fill_(m, 0.0)
        elif cols.numel():
          dst[:, cols] = torch.where(m, 0.0, dst[:, cols])
      return
    rows = n if env_ids is None or isinstance(env_ids, slice) else env_ids.numel()
    v = self._ix["free_joint_v_adr"]
    if v.numel():
      _masked_write(self.data.qfrc_applied, v, torch.zeros(rows, v.numel(), device=self.data.qpos.device), env_ids)
    xf = self.data.xfrc_applied.view(n, -1)
    cols = self._ix["body_ids"][:, None] * 6 + torch.arange(6, device=xf.device)
    _masked_write(xf, cols.reshape(-1), torch.zeros(rows, cols.numel(), device=xf.device), env_ids)
    if self.is_actuated:
      c = self._ix["ctrl_ids"]
      _masked_write(self.data.ctrl, c, torch.zeros(rows, c.numel(), device=xf.device), env_ids)

  # ---- reads ----
  @property
  def _root(self) -> int:
    return self.indexing.root_body_id

  @_cached
  def root_link_pose_w(self) -> torch.Tensor:
    return torch.cat([self.data.xpos[:, self._root], self.data.xquat[:, self._root]], dim=-1)

  @_cached
  def _root_frame(self):
    """[root_link_vel_w 6 | lin_vel_b 3 | ang_vel_b 3 | projected_gravity_b 3 |
    heading_w 1] per env from one launch (csrc/mjh_fuse.hip), or None (CPU)."""
    r = self._root
    return envops.root_frame(self.data.xpos[:, r], self.data.xquat[:, r], self.data.subtree_com[:, r], self.data.cvel[:, r],
                             self.gravity_vec_w, self.forward_vec_b)

  @_cached
  def root_link_vel_w(self) -> torch.Tensor:
    f = self._root_frame
    if f is not None:
      return f[:, 0:6]
    r = self._root
    return envops.velocity_from_cvel(self.data.xpos[:, r], self.data.subtree_com[:, r], self.data.cvel[:, r], compute_velocity_from_cvel)

  @_cached
  def root_com_pose_w(self) -> torch.Tensor:
    r = self._root
    q = quat_mul(self.data.xquat[:, r], self.model.body_iquat[:, r].expand(self.data.xquat.shape[0], -1))
    return torch.cat([self.data.xipos[:, r], q], dim=-1)

  @_cached
  def root_com_vel_w(self) -> torch.Tensor:
    r = self._root
    return envops.velocity_from_cvel(self.data.xipos[:, r], self.data.subtree_com[:, r], self.data.cvel[:, r], compute_velocity_from_cvel)

  @_cached
  def body_link_pose_w(self) -> torch.Tensor:
    ids = self._ix["body_ids"]
    return torch.cat([self.data.xpos[:, ids], self.data.xquat[:, ids]], dim=-1)

  def _vel_rows(self, arr, key: str, body_key: str):
    """compute_velocity_from_cvel of this entity's rows of `arr` in one launch
    (strided reads, no gathers), or None when the layout is unsupported."""
    if not arr.is_cuda:
      return None
    b32 = self.__dict__.setdefault("_ix32", {})
    if body_key not in b32:
      b32[body_key] = self._ix[body_key].to(torch.int32).contiguous()
    return envops.velocity_rows(arr[:, self._rows(key)], self.data.subtree_com[:, self._root], self.data.cvel,
                                b32[body_key])

  @_cached
  def body_link_vel_w(self) -> torch.Tensor:
    v = self._vel_rows(self.data.xpos, "body_ids", "body_ids")
    if v is not None:
      return v
    ids = self._ix["body_ids"]
    com = self.data.subtree_com[:, self._root].unsqueeze(1)
    return compute_velocity_from_cvel(self.data.xpos[:, ids], com, self.data.cvel[:, ids])

  @_cached
  def body_com_pose_w(self) -> torch.Tensor:
    ids = self._ix["body_ids"]
    iq = self.model.body_iquat[:, ids].expand(self.data.xquat.shape[0], -1, -1)
    return torch.cat([self.data.xipos[:, ids], quat_mul(self.data.xquat[:, ids], iq)], dim=-1)

  @_cached
  def body_com_vel_w(self) -> torch.Tensor:
    v = self._vel_rows(self.data.xipos, "body_ids", "body_ids")
    if v is not None:
      return v
    ids = self._ix["body_ids"]
    com = self.data.subtree_com[:, self._root].unsqueeze(1)
    return compute_velocity_from_cvel(self.data.xipos[:, ids], com, self.data.cvel[:, ids])

  @property
  def body_external_wrench(self) -> torch.Tensor:
    return self.data.xfrc_applied[:, self._ix["body_ids"]]

  @_cached
  def geom_pose_w(self) -> torch.Tensor:
    ids = self._ix["geom_ids"]
    return torch.cat([self.data.geom_xpos[:, ids], quat_from_matrix(self.data.geom_xmat[:, ids])], dim=-1)

  @_cached
  def geom_vel_w(self) -> torch.Tensor:
    v = self._vel_rows(self.data.geom_xpos, "geom_ids", "geom_bodyid")
    if v is not None:
      return v
    ids = self._ix["geom_ids"]
    bids = self._ix["geom_bodyid"]
    com = self.data.subtree_com[:, self._root].unsqueeze(1)
    return compute_velocity_from_cvel(self.data.geom_xpos[:, ids], com, self.data.cvel[:, bids])

  @_cached
  def site_pose_w(self) -> torch.Tensor:
    ids = self._ix["site_ids"]
    return torch.cat([self.data.site_xpos[:, ids], quat_from_matrix(self.data.site_xmat[:, ids])], dim=-1)

  @_cached
  def site_vel_w(self) -> torch.Tensor:
    v = self._vel_rows(self.data.site_xpos, "site_ids", "site_bodyid")
    if v is not None:
      return v
    ids = self._ix["site_ids"]
    bids = self._ix["site_bodyid"]
    com = self.data.subtree_com[:, self._root].unsqueeze(1)
    return compute_velocity_from_cvel(self.data.site_xpos[:, ids], com, self.data.cvel[:, bids])

  @property
  def joint_pos(self) -> torch.Tensor:
    return self.data.qpos[:, self._ix["joint_q_adr"]]

  @property
  def joint_vel(self) -> torch.Tensor:
    return self.data.qvel[:, self._ix["joint_v_adr"]]

  @property
  def joint_acc(self) -> torch.Tensor:
    return self.data.qacc[:, self._ix["joint_v_adr"]]

  @property
  def actuator_force(self) -> torch.Tensor:
    return self.data.actuator_force[:, self._ix["ctrl_ids"]]

  @property
  def generalized_force(self) -> torch.Tensor:
    return self.data.qfrc_applied[:, self._ix["free_joint_v_adr"]]

  # == root_link_pose_w[:, 0:3] / [:, 3:7], read straight from the kinematics
  # outputs (views: no gather or concatenation launched)
  root_link_pos_w = property(lambda s: s.data.xpos[:, s._root])
  root_link_quat_w = property(lambda s: s.data.xquat[:, s._root])
  root_link_lin_vel_w = property(lambda s: s.root_link_vel_w[:, 0:3])
  root_link_ang_vel_w = property(lambda s: s.root_link_vel_w[:, 3:6])
  root_com_pos_w = property(lambda s: s.root_com_pose_w[:, 0:3])
  root_com_quat_w = property(lambda s: s.root_com_pose_w[:, 3:7])
  root_com_lin_vel_w = property(lambda s: s.root_com_vel_w[:, 0:3])
  root_com_ang_vel_w = property(lambda s: s.root_com_vel_w[:, 3:6])
  body_link_pos_w = property(lambda s: s._body_link_pos_w)
  body_link_quat_w = property(lambda s: s._body_link_quat_w)
  body_link_lin_vel_w = property(lambda s: s.body_link_vel_w[..., 0:3])
  body_link_ang_vel_w = property(lambda s: s.body_link_vel_w[..., 3:6])
  body_com_pos_w = property(lambda s: s.body_com_pose_w[..., 0:3])
  body_com_quat_w = property(lambda s: s.body_com_pose_w[..., 3:7])
  body_com_lin_vel_w = property(lambda s: s.body_com_vel_w[..., 0:3])
  body_com_ang_vel_w = property(lambda s: s.body_com_vel_w[..., 3:6])
  body_external_force = property(lambda s: s.body_external_wrench[..., 0:3])
  body_external_torque = property(lambda s: s.body_external_wrench[..., 3:6])
  geom_pos_w = property(lambda s: s._geom_pos_w)
  geom_quat_w = property(lambda s: s.geom_pose_w[..., 3:7])
  geom_lin_vel_w = property(lambda s: s.geom_vel_w[..., 0:3])
  geom_ang_vel_w = property(lambda s: s.geom_vel_w[..., 3:6])
  site_pos_w = property(lambda s: s._site_pos_w)
  site_quat_w = property(lambda s: s.site_pose_w[..., 3:7])
  site_lin_vel_w = property(lambda s: s.site_vel_w[..., 0:3])
  site_ang_vel_w = property(lambda s: s.site_vel_w[..., 3:6])

  def _rows(self, key: str):
    """Index of this entity's bodies/geoms/sites in the data arrays: a slice
    (reads are views, no gather launch) when they are consecutive, as usual."""
    c = self._cols[key]
    return c if isinstance(c, slice) else self._ix[key]

  @_cached
  def _body_link_pos_w(self) -> torch.Tensor:
    """== body_link_pose_w[..., 0:3]"""
    return self.data.xpos[:, self._rows("body_ids")]

  @_cached
  def _body_link_quat_w(self) -> torch.Tensor:
    """== body_link_pose_w[..., 3:7]"""
    return self.data.xquat[:, self._rows("body_ids")]

  @_cached
  def _geom_pos_w(self) -> torch.Tensor:
    """== geom_pose_w[..., 0:3], without converting the frames to quaternions."""
    return self.data.geom_xpos[:, self._rows("geom_ids")]

  @_cached
  def _site_pos_w(self) -> torch.Tensor:
    """== site_pose_w[..., 0:3], without converting the frames to quaternions."""
    return self.data.site_xpos[:, self._rows("site_ids")]

  @_cached
  def projected_gravity_b(self) -> torch.Tensor:
    rf = self._root_frame
    if rf is not None:
      return rf[:, 12:15]
    return quat_apply_inverse(self.root_link_quat_w, self.gravity_vec_w)

  @_cached
  def heading_w(self) -> torch.Tensor:
    rf = self._root_frame
    if rf is not None:
      return rf[:, 15]
    f = quat_apply(self.root_link_quat_w, self.forward_vec_b)
    return torch.atan2(f[:, 1], f[:, 0])

  @_cached
  def root_link_lin_vel_b(self) -> torch.Tensor:
    rf = self._root_frame
    if rf is not None:
      return rf[:, 6:9]
    return quat_apply_inverse(self.root_link_quat_w, self.root_link_lin_vel_w)

  @_cached
  def root_link_ang_vel_b(self) -> torch.Tensor:
    rf = self._root_frame
    if rf is not None:
      return rf[:, 9:12]
    return quat_apply_inverse(self.root_link_quat_w, self.root_link_ang_vel_w)

  @_cached
  def root_com_lin_vel_b(self) -> torch.Tensor:
    return quat_apply_inverse(self.root_link_quat_w, self.root_com_lin_vel_w)

  @_cached
  def root_com_ang_vel_b(self) -> torch.Tensor:
    return quat_apply_inverse(self.root_link_quat_w, self.root_com_ang_vel_w)
