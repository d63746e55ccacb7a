"""Contact sensors: pattern expansion into ``contact`` sensors + air-time tracking.

Restates ``src/mjlab/sensor/contact_sensor.py``: one device sensor per
(primary, field) with ``intprm = [1 << field, reduce, num_slots]``
(``:472-533``), sensordata views reshaped ``(B, num_slots, dim)`` (``:282-304``),
and the air/contact timers (``:327-367``). The contact matching and reduction
itself runs inside the HIP step kernel (sensor stage), like ``mjSENS_CONTACT``
inside MuJoCo Warp.
"""

from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Literal

import torch

from mjlab_amd import envops

from mjlab_amd.spec.spec import SensorSpec, Spec

_CONTACT_DATA_MAP = {"found": 0, "force": 1, "torque": 2, "dist": 3, "pos": 4, "normal": 5, "tangent": 6}
_CONTACT_DATA_DIMS = {"found": 1, "force": 3, "torque": 3, "dist": 1, "pos": 3, "normal": 3, "tangent": 3}
_CONTACT_REDUCE_MAP = {"none": 0, "mindist": 1, "maxforce": 2, "netforce": 3}
_MODE_TO_OBJTYPE = {"geom": "geom", "body": "body", "subtree": "xbody"}


@dataclass
class ContactMatch:
  mode: Literal["geom", "body", "subtree"]
  pattern: str | tuple[str, ...]
  entity: str | None = None
  exclude: tuple[str, ...] = ()


@dataclass
class SensorCfg:
  name: str


def _regular_slots(cols: list[int], dim: int):
  """(first column, slot spacing, slots) when cols = [a + i*s + c for i < k, c < dim], else None."""
  if not cols or len(cols) % dim:
    return None
  k = len(cols) // dim
  a = cols[0]
  s = cols[dim] - a if k > 1 else dim
  if s < dim:
    return None
  return (a, s, k) if cols == [a + i * s + c for i in range(k) for c in range(dim)] else None


@dataclass
class ContactSensorCfg(SensorCfg):
  primary: ContactMatch = None  # type: ignore[assignment]
  secondary: ContactMatch | None = None
  fields: tuple[str, ...] = ("found", "force")
  reduce: Literal["none", "mindist", "maxforce", "netforce"] = "maxforce"
  num_slots: int = 1
  secondary_policy: Literal["first", "any", "error"] = "first"
  track_air_time: bool = False
  global_frame: bool = False
  debug: bool = False

  def build(self) -> "ContactSensor":
    return ContactSensor(self)


@dataclass
class _ContactSlot:
  primary_name: str
  field_name: str
  sensor_name: str
  data_view: torch.Tensor | None = None


@dataclass
class _AirTimeState:
  current_air_time: torch.Tensor
  last_air_time: torch.Tensor
  current_contact_time: torch.Tensor
  last_contact_time: torch.Tensor
  last_time: torch.Tensor


@dataclass
class ContactData:
  found: torch.Tensor | None = None
  force: torch.Tensor | None = None
  torque: torch.Tensor | None = None
  dist: torch.Tensor | None = None
  pos: torch.Tensor | None = None
  normal: torch.Tensor | None = None
  tangent: torch.Tensor | None = None
  current_air_time: torch.Tensor | None = None
  last_air_time: torch.Tensor | None = None
  current_contact_time: torch.Tensor | None = None
  last_contact_time: torch.Tensor | None = None


class ContactSensor:
  def __init__(self, cfg: ContactSensorCfg) -> None:
    self.cfg = cfg
    if cfg.global_frame and cfg.reduce != "netforce":
      if "normal" not in cfg.fields or "tangent" not in cfg.fields:
        raise ValueError(
          f"Sensor '{cfg.name}': global_frame=True requires 'normal' and 'tangent' in fields"
        )
    self._slots: list[_ContactSlot] = []
    self._data = None
    self._air_time_state: _AirTimeState | None = None

  # ---- spec ----
  def edit_spec(self, scene_spec: Spec, entities: dict) -> None:
    self._slots.clear()
    prims = self._resolve_primary_names(entities, self.cfg.primary)
    if self.cfg.secondary is None or self.cfg.secondary_policy == "any":
      sec = None
    else:
      sec = self._resolve_single_secondary(entities, self.cfg.secondary, self.cfg.secondary_policy)
    for p in prims:
      for f in self.cfg.fields:
        sname = f"{self.cfg.name}_{p}_{f}"
        self._add(scene_spec, sname, p, sec, f)
        self._slots.append(_ContactSlot(p, f, sname))

  def _add(self, spec: Spec, sname: str, prim: str, sec: str | None, field: str) -> None:
    pe = self.cfg.primary.entity
    pname = f"{pe}/{prim}" if pe else prim
    s = SensorSpec(
      name=sname,
      type="contact",
      objtype=_MODE_TO_OBJTYPE[self.cfg.primary.mode],
      objname=pname,
      intprm=[1 << _CONTACT_DATA_MAP[field], _CONTACT_REDUCE_MAP[self.cfg.reduce], self.cfg.num_slots],
    )
    if sec is not None:
      se = self.cfg.secondary.entity
      s.reftype = _MODE_TO_OBJTYPE[self.cfg.secondary.mode]
      s.refname = f"{se}/{sec}" if se else sec
    spec.sensors.append(s)

  def _resolve_primary_names(self, entities: dict, match: ContactMatch) -> list[str]:
    if match.entity in (None, ""):
      return [match.pattern] if isinstance(match.pattern, str) else list(match.pattern)
    if match.entity not in entities:
      raise ValueError(f"Primary entity '{match.entity}' not found. Available: {list(entities)}")
    ent = entities[match.entity]
    pats = [match.pattern] if isinstance(match.pattern, str) else list(match.pattern)
    if match.mode == "geom":
      _, names = ent.find_geoms(pats)
    elif match.mode in ("body", "subtree"):
      _, names = ent.find_bodies(pats)
    else:
      raise ValueError("Primary mode must be one of {'geom','body','subtree'}")
    if match.exclude:
      exact = {e for e in match.exclude if not any(c in e for c in r".*+?[]{}()\|^$")}
      rx = [re.compile(e) for e in match.exclude if e not in exact]
      names = [n for n in names if n not in exact and not any(r.search(n) for r in rx)]
    if not names:
      raise ValueError(f"Primary pattern '{match.pattern}' matched no names in '{match.entity}'")
    return names

  def _resolve_single_secondary(self, entities: dict, match: ContactMatch, policy: str) -> str | None:
    if policy == "any":
      return None
    if isinstance(match.pattern, tuple):
      raise ValueError("Secondary must specify a single name (string).")
    if match.entity in (None, ""):
      return match.pattern
    if match.entity not in entities:
      raise ValueError(f"Secondary entity '{match.entity}' not found.")
    ent = entities[match.entity]
    if match.mode == "subtree":
      return match.pattern
    _, names = ent.find_geoms(match.pattern) if match.mode == "geom" else ent.find_bodies(match.pattern)
    if not names:
      raise ValueError(f"Secondary pattern '{match.pattern}' matched nothing")
    if len(names) == 1 or policy == "first":
      return names[0]
    raise ValueError(f"Secondary pattern '{match.pattern}' matched multiple: {names}.")

  # ---- runtime ----
  def initialize(self, model, sim_model, data, device: str) -> None:
    if not self._slots:
      raise RuntimeError(f"There was an error initializing contact sensor '{self.cfg.name}'")
    for slot in self._slots:
      s = model.sensor(slot.sensor_name)
      a, d = int(s.adr[0]), int(s.dim[0])
      slot.data_view = data.sensordata[:, a : a + d]
    self._data = data
    # sensordata columns of the `found` slots, for the fused timer kernel
    fcols = [int(model.sensor(sl.sensor_name).adr[0]) for sl in self._slots if sl.field_name == "found"]
    self._found_cols = torch.tensor(fcols, dtype=torch.int32, device=device)
    self._found_cols_host = fcols
    if self.cfg.track_air_time:
      n = data.time.shape[0]
      k = len({s.primary_name for s in self._slots})
      z = lambda: torch.zeros((n, k), device=device)  # noqa: E731
      self._air_time_state = _AirTimeState(z(), z(), z(), z(), torch.zeros((n,), device=device))

  def attach_air_time_to(self, sim) -> bool:
    """Fuse this sensor's timer update into the physics step of an env's
    decimation loop (Simulation.attach_air_time): the step updates the timers
    with the arithmetic of _update_air_time_tracking, so Scene.update skips
    this sensor there. False when the sensor has no timers or the layout does
    not fit the fused path."""
    st = self._air_time_state
    if st is None or len(self._found_cols_host) != st.current_air_time.shape[1]:
      return False
    return sim.attach_air_time(self._found_cols_host, st.last_time, st.current_air_time, st.last_air_time,
                               st.current_contact_time, st.last_contact_time)

  @property
  def data(self) -> ContactData:
    out = self._extract_sensor_data()
    st = self._air_time_state
    if st is not None:
      out.current_air_time = st.current_air_time
      out.last_air_time = st.last_air_time
      out.current_contact_time = st.current_contact_time
      out.last_contact_time = st.last_contact_time
    return out

  def reset(self, env_ids=None) -> None:
    st = self._air_time_state
    if st is None:
      return
    if env_ids is not None and isinstance(env_ids, torch.Tensor) and env_ids.dtype == torch.bool:
      m = env_ids[:, None]
      timers = (st.current_air_time, st.last_air_time, st.current_contact_time, st.last_contact_time)
      if not envops.masked_zero(list(timers), env_ids):  # one launch for the four timers
        for t in timers:
          t.masked_fill_(m, 0.0)
      if not envops.masked_copy(st.last_time, self._data.time, env_ids):
        torch.where(env_ids, self._data.time, st.last_time, out=st.last_time)
      return
    ids = slice(None) if env_ids is None else env_ids
    st.current_air_time[ids] = 0.0
    st.last_air_time[ids] = 0.0
    st.current_contact_time[ids] = 0.0
    st.last_contact_time[ids] = 0.0
    st.last_time[ids] = self._data.time[ids]

  def update(self, dt: float) -> None:
    del dt
    if self._air_time_state is not None:
      self._update_air_time_tracking()

  def compute_first_contact(self, dt: float, abs_tol: float = 1.0e-8) -> torch.Tensor:
    st = self._require_air()
    return (st.current_contact_time > 0.0) & (st.current_contact_time < (dt + abs_tol))

  def compute_first_air(self, dt: float, abs_tol: float = 1.0e-8) -> torch.Tensor:
    st = self._require_air()
    return (st.current_air_time > 0.0) & (st.current_air_time < (dt + abs_tol))

  def _require_air(self) -> _AirTimeState:
    if self._air_time_state is None:
      raise RuntimeError(f"Sensor '{self.cfg.name}' must have track_air_time=True")
    return self._air_time_state

  def _extract_sensor_data(self) -> ContactData:
    """Slots of each field gathered in one indexed read of sensordata (instead of
    a concatenation of per-slot views), cached until the next step/forward."""
    ep = self._data.epoch.v
    if getattr(self, "_cache_ep", None) == ep:
      return ContactData(**vars(self._cache))
    if not hasattr(self, "_field_cols"):
      self._field_cols = {}
      for f in self.cfg.fields:
        cols = []
        for slot in self._slots:
          if slot.field_name == f:
            a = slot.data_view.storage_offset() - self._data.sensordata.storage_offset()
            cols += list(range(a, a + slot.data_view.shape[1]))
        self._field_cols[f] = torch.tensor(cols, dtype=torch.long, device=self._data.sensordata.device)
        self._field_stride = getattr(self, "_field_stride", {})
        self._field_stride[f] = _regular_slots(cols, _CONTACT_DATA_DIMS[f])
    out = ContactData()
    sd = self._data.sensordata
    n = sd.shape[0]
    for f in self.cfg.fields:
      dim = _CONTACT_DATA_DIMS[f]
      reg = self._field_stride.get(f)
      if reg is not None and sd.stride(1) == 1:  # slots evenly spaced: a strided view, no gather launch
        a, s, k = reg
        cat = sd.as_strided((n, k, dim), (sd.stride(0), s, 1), sd.storage_offset() + a)
      else:
        cat = sd[:, self._field_cols[f]].view(n, -1, dim)
      if cat.size(-1) == 1:
        cat = cat.squeeze(-1)
      setattr(out, f, cat)
    if self.cfg.global_frame and self.cfg.reduce != "netforce":
      nrm, t = out.normal, out.tangent
      R = torch.stack([t, torch.cross(nrm, t, dim=-1), nrm], dim=-1)
      has = torch.norm(nrm, dim=-1, keepdim=True) > 1e-8
      if out.force is not None:
        out.force = torch.where(has, torch.einsum("...ij,...j->...i", R, out.force), out.force)
      if out.torque is not None:
        out.torque = torch.where(has, torch.einsum("...ij,...j->...i", R, out.torque), out.torque)
    self._cache, self._cache_ep = out, ep
    return ContactData(**vars(out))

  def _update_air_time_tracking(self) -> None:
    st = self._air_time_state
    if self._found_cols.numel() == st.current_air_time.shape[1] and envops.air_time_update(
      self._data.sensordata, self._found_cols, self._data.time, st.last_time, st.current_air_time, st.last_air_time,
      st.current_contact_time, st.last_contact_time,
    ):
      return
    cd = self._extract_sensor_data()
    if cd.found is None:
      return
    now = self._data.time
    el = (now - st.last_time).unsqueeze(-1)
    is_c = cd.found > 0
    first_c = (st.current_air_time > 0) & is_c
    first_d = (st.current_contact_time > 0) & ~is_c
    torch.where(first_c, st.current_air_time + el, st.last_air_time, out=st.last_air_time)
    torch.where(~is_c, st.current_air_time + el, torch.zeros_like(st.current_air_time), out=st.current_air_time)
    torch.where(first_d, st.current_contact_time + el, st.last_contact_time, out=st.last_contact_time)
    torch.where(is_c, st.current_contact_time + el, torch.zeros_like(st.current_contact_time), out=st.current_contact_time)
    st.last_time.copy_(now)
