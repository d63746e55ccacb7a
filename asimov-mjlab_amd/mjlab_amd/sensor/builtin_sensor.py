"""Builtin sensors: views into ``sensordata`` (``src/mjlab/sensor/builtin_sensor.py:171-340``).

``BuiltinSensorCfg`` / ``ObjRef`` keep the reference's validation rules
(``builtin_sensor.py:206-259``: site sensors need a site, frame sensors a
spatial frame, subtree sensors a body, joint sensors a joint; ``ref`` only on
frame sensors; the name is prefixed ``entity/`` when ``obj.entity`` is set).
The step kernel evaluates the sensor types in ``spec.compiler.SENSOR_TYPES``;
any other type raises at ``edit_spec`` instead of reading zeros.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Literal

import torch

from mjlab_amd.sensor.contact_sensor import SensorCfg
from mjlab_amd.spec.compiler import SENSOR_TYPES
from mjlab_amd.spec.spec import SensorSpec

_REQUIRING_SITE = {"accelerometer", "velocimeter", "gyro", "force", "torque", "magnetometer", "rangefinder"}
_REQUIRING_FRAME = {"framepos", "framequat", "framexaxis", "frameyaxis", "framezaxis", "framelinvel", "frameangvel",
                    "framelinacc", "frameangacc"}
_REQUIRING_BODY = {"subtreecom", "subtreelinvel", "subtreeangmom"}
_REQUIRING_OBJ = {"jointpos": "joint", "jointvel": "joint", "jointlimitpos": "joint", "jointlimitvel": "joint",
                  "jointlimitfrc": "joint", "jointactuatorfrc": "joint", "tendonpos": "tendon", "tendonvel": "tendon",
                  "tendonactuatorfrc": "tendon", "actuatorpos": "actuator", "actuatorvel": "actuator",
                  "actuatorfrc": "actuator"}
_SPATIAL = {"body", "xbody", "geom", "site", "camera"}


@dataclass
class ObjRef:
  type: Literal["body", "xbody", "joint", "geom", "site", "actuator", "tendon", "camera"]
  name: str
  entity: str | None = None

  def prefixed_name(self) -> str:
    return f"{self.entity}/{self.name}" if self.entity else self.name


@dataclass
class BuiltinSensorCfg(SensorCfg):
  sensor_type: str
  obj: ObjRef | None = None
  ref: ObjRef | None = None
  cutoff: float = 0.0

  def __post_init__(self) -> None:
    if self.obj is not None and self.obj.entity is not None:
      self.name = f"{self.obj.entity}/{self.name}"
    t = self.sensor_type
    if t in _REQUIRING_SITE:
      if self.obj is None or self.obj.type != "site":
        raise ValueError(f"Sensor type '{t}' requires obj.type='site', got "
                         f"'{None if self.obj is None else self.obj.type}'")
    elif t in _REQUIRING_FRAME:
      if self.obj is None or self.obj.type not in _SPATIAL:
        raise ValueError(f"Sensor type '{t}' requires obj.type in {_SPATIAL}")
    elif t in _REQUIRING_BODY:
      if self.obj is None or self.obj.type != "body":
        raise ValueError(f"Sensor type '{t}' requires obj.type='body'")
    elif t in _REQUIRING_OBJ:
      req = _REQUIRING_OBJ[t]
      if self.obj is None or self.obj.type != req:
        raise ValueError(f"Sensor type '{t}' requires obj.type='{req}'")
    if self.ref is not None and t not in _REQUIRING_FRAME:
      raise ValueError(f"Sensor type '{t}' does not support ref specification")

  def build(self) -> "BuiltinSensor":
    return BuiltinSensor(self)


class BuiltinSensor:
  def __init__(self, cfg: BuiltinSensorCfg | None = None, name: str | None = None) -> None:
    if cfg is None and name is None:
      raise ValueError("Must provide either cfg or name")
    self.cfg = cfg
    self._name = cfg.name if cfg is not None else name
    self._data = None
    self._data_view: torch.Tensor | None = None

  @classmethod
  def from_existing(cls, name: str) -> "BuiltinSensor":
    return cls(cfg=None, name=name)

  def edit_spec(self, scene_spec, entities) -> None:
    """Add the sensor to the scene spec (``builtin_sensor.py:291-325``)."""
    del entities
    c = self.cfg
    if c is None:
      return
    for s in scene_spec.sensors:
      if s.name == c.name:
        if c.obj is not None and c.obj.entity is not None:
          raise ValueError(f"Sensor '{c.name}' is defined in both entity XML and scene config. Remove the sensor "
                           f"definition from the entity XML file, or remove the BuiltinSensorCfg from scene.sensors.")
        raise ValueError(f"Sensor '{c.name}' already exists in the scene. Rename this sensor to avoid conflicts.")
    if c.sensor_type not in SENSOR_TYPES or c.sensor_type == "contact":
      raise NotImplementedError(f"builtin sensor type '{c.sensor_type}' is not evaluated by the HIP step; "
                                f"supported: {sorted(k for k in SENSOR_TYPES if k != 'contact')}")
    spec = SensorSpec(name=c.name, type=c.sensor_type, cutoff=float(c.cutoff))
    if c.obj is not None:
      spec.objtype, spec.objname = c.obj.type, c.obj.prefixed_name()
    if c.ref is not None:
      spec.reftype, spec.refname = c.ref.type, c.ref.prefixed_name()
    scene_spec.sensors.append(spec)

  def initialize(self, model, sim_model, data, device: str) -> None:
    del sim_model, device
    self._data = data
    s = model.sensor(self._name)
    a, d = int(s.adr[0]), int(s.dim[0])
    self._data_view = data.sensordata[:, a : a + d]

  @property
  def data(self) -> torch.Tensor:
    assert self._data_view is not None
    return self._data_view

  def reset(self, env_ids=None) -> None:
    del env_ids

  def update(self, dt: float) -> None:
    del dt
