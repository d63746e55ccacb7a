"""In-memory model specification (the MjSpec analogue).

mjlab edits a ``mujoco.MjSpec`` before compiling it (collision cfg, actuators,
keyframes, contact sensors; ``src/mjlab/utils/spec_config.py:136-428``,
``src/mjlab/entity/entity.py:131-166``, ``src/mjlab/sensor/contact_sensor.py:472-533``).
MuJoCo is not available on MI355X boxes, so this package carries its own spec
tree: plain dataclasses that the MJCF reader fills and the compiler
(``mjlab_amd.spec.compiler``) flattens into per-world device arrays.

Element semantics follow the MJCF schema (MuJoCo 3.x XML reference); only the
subset used by mjlab's robots and tests is modelled, anything else raises.
"""

from __future__ import annotations

import copy
import json
from dataclasses import asdict, dataclass, field
from typing import Any

# MuJoCo enum values (mjtGeom / mjtJoint / mjtSensor / mjtObj) re-declared here
# so that integer codes in the device arrays match what mjlab code compares to.
GEOM_TYPES = {
  "plane": 0,
  "hfield": 1,
  "sphere": 2,
  "capsule": 3,
  "ellipsoid": 4,
  "cylinder": 5,
  "box": 6,
  "mesh": 7,
}
JOINT_TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}
OBJ_TYPES = {"body": 1, "xbody": 2, "joint": 3, "geom": 5, "site": 6}


@dataclass
class JointSpec:
  name: str = ""
  type: str = "hinge"
  pos: list[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])
  axis: list[float] = field(default_factory=lambda: [0.0, 0.0, 1.0])
  range: list[float] = field(default_factory=lambda: [0.0, 0.0])
  limited: str = "auto"  # "auto" | "true" | "false"
  ref: float = 0.0
  springref: float = 0.0
  armature: float = 0.0
  damping: float = 0.0
  stiffness: float = 0.0
  frictionloss: float = 0.0
  margin: float = 0.0
  solref_limit: list[float] = field(default_factory=lambda: [0.02, 1.0])
  solimp_limit: list[float] = field(
    default_factory=lambda: [0.9, 0.95, 0.001, 0.5, 2.0]
  )
  solref_friction: list[float] = field(default_factory=lambda: [0.02, 1.0])
  solimp_friction: list[float] = field(
    default_factory=lambda: [0.9, 0.95, 0.001, 0.5, 2.0]
  )


@dataclass
class GeomSpec:
  name: str = ""
  type: str = "sphere"
  size: list[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])
  pos: list[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])
  quat: list[float] = field(default_factory=lambda: [1.0, 0.0, 0.0, 0.0])
  fromto: list[float] | None = None
  contype: int = 1
  conaffinity: int = 1
  condim: int = 3
  priority: int = 0
  friction: list[float] = field(default_factory=lambda: [1.0, 0.005, 0.0001])
  solmix: float = 1.0
  solref: list[float] = field(default_factory=lambda: [0.02, 1.0])
  solimp: list[float] = field(default_factory=lambda: [0.9, 0.95, 0.001, 0.5, 2.0])
  margin: float = 0.0
  gap: float = 0.0
  group: int = 0
  rgba: list[float] = field(default_factory=lambda: [0.5, 0.5, 0.5, 1.0])
  mesh: str | None = None
  material: str | None = None
  density: float = 1000.0
  mass: float | None = None


@dataclass
class SiteSpec:
  name: str = ""
  type: str = "sphere"
  pos: list[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])
  quat: list[float] = field(default_factory=lambda: [1.0, 0.0, 0.0, 0.0])
  size: list[float] = field(default_factory=lambda: [0.005, 0.005, 0.005])
  group: int = 0
  rgba: list[float] = field(default_factory=lambda: [0.5, 0.5, 0.5, 1.0])


@dataclass
class InertialSpec:
  pos: list[float]
  quat: list[float]
  mass: float
  diaginertia: list[float]


@dataclass
class BodySpec:
  name: str = ""
  pos: list[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])
  quat: list[float] = field(default_factory=lambda: [1.0, 0.0, 0.0, 0.0])
  mocap: bool = False
  inertial: InertialSpec | None = None
  joints: list[JointSpec] = field(default_factory=list)
  geoms: list[GeomSpec] = field(default_factory=list)
  sites: list[SiteSpec] = field(default_factory=list)
  children: list["BodySpec"] = field(default_factory=list)

  # Iteration helpers (depth-first, MuJoCo body order).
  def walk(self):
    yield self
    for c in self.children:
      yield from c.walk()


@dataclass
class ActuatorSpec:
  """Joint-transmission actuator with fixed gain and affine bias.

  Mirrors what ``ActuatorSetCfg.edit_spec`` creates
  (``src/mjlab/utils/spec_config.py:402-414``): ``gaintype=FIXED``,
  ``biastype=AFFINE``, ``inheritrange``, ``forcerange``.
  """

  name: str = ""
  joint: str = ""
  gear: float = 1.0
  gainprm: list[float] = field(default_factory=lambda: [1.0, 0.0, 0.0])
  biasprm: list[float] = field(default_factory=lambda: [0.0, 0.0, 0.0])
  ctrlrange: list[float] = field(default_factory=lambda: [0.0, 0.0])
  ctrllimited: str = "auto"
  forcerange: list[float] = field(default_factory=lambda: [0.0, 0.0])
  forcelimited: str = "auto"
  inheritrange: float = 0.0


@dataclass
class SensorSpec:
  name: str = ""
  type: str = ""  # gyro|velocimeter|accelerometer|subtreeangmom|contact|...
  objtype: str = ""
  objname: str = ""
  reftype: str = ""
  refname: str = ""
  intprm: list[int] = field(default_factory=lambda: [0, 0, 0])
  cutoff: float = 0.0


@dataclass
class KeySpec:
  name: str = ""
  qpos: list[float] | None = None
  ctrl: list[float] | None = None


@dataclass
class OptionSpec:
  timestep: float = 0.002
  gravity: list[float] = field(default_factory=lambda: [0.0, 0.0, -9.81])
  magnetic: list[float] = field(default_factory=lambda: [0.0, -0.5, 0.0])  # mjOption.magnetic (magnetometer)
  impratio: float = 1.0
  tolerance: float = 1e-8
  ls_tolerance: float = 0.01
  iterations: int = 100
  ls_iterations: int = 50
  integrator: str = "euler"
  cone: str = "pyramidal"
  solver: str = "newton"
  jacobian: str = "auto"


@dataclass
class Spec:
  """Root of a model specification (one MJCF file or a composed scene)."""

  model: str = ""
  worldbody: BodySpec = field(default_factory=lambda: BodySpec(name="world"))
  excludes: list[tuple[str, str]] = field(default_factory=list)
  actuators: list[ActuatorSpec] = field(default_factory=list)
  sensors: list[SensorSpec] = field(default_factory=list)
  keys: list[KeySpec] = field(default_factory=list)
  option: OptionSpec = field(default_factory=OptionSpec)
  autolimits: bool = True

  # --- Queries mirroring the MjSpec accessors mjlab uses. ---

  @property
  def bodies(self) -> list[BodySpec]:
    return list(self.worldbody.walk())

  @property
  def joints(self) -> list[JointSpec]:
    return [j for b in self.bodies for j in b.joints]

  @property
  def geoms(self) -> list[GeomSpec]:
    return [g for b in self.bodies for g in b.geoms]

  @property
  def sites(self) -> list[SiteSpec]:
    return [s for b in self.bodies for s in b.sites]

  def body(self, name: str) -> BodySpec:
    for b in self.bodies:
      if b.name == name:
        return b
    raise KeyError(f"body '{name}' not found")

  def joint(self, name: str) -> JointSpec:
    for j in self.joints:
      if j.name == name:
        return j
    raise KeyError(f"joint '{name}' not found")

  def geom(self, name: str) -> GeomSpec:
    for g in self.geoms:
      if g.name == name:
        return g
    raise KeyError(f"geom '{name}' not found")

  def copy(self) -> "Spec":
    return copy.deepcopy(self)

  def attach(self, child: "Spec", prefix: str = "") -> None:
    """Attach ``child``'s world children, excludes, actuators, sensors and keys.

    Same effect as ``MjSpec.attach(child, prefix=..., frame=<identity>)`` used by
    ``Scene._add_entities`` (``src/mjlab/scene/scene.py:149-154``): every named
    element is renamed ``prefix + name``.
    """
    c = child.copy()

    def pre(n: str) -> str:
      return prefix + n if n else n

    for b in c.worldbody.walk():
      if b is not c.worldbody:
        b.name = pre(b.name)
      for j in b.joints:
        j.name = pre(j.name)
      for g in b.geoms:
        g.name = pre(g.name)
      for s in b.sites:
        s.name = pre(s.name)
    # World-level geoms/sites of the child become world-level here.
    self.worldbody.geoms.extend(c.worldbody.geoms)
    self.worldbody.sites.extend(c.worldbody.sites)
    self.worldbody.children.extend(c.worldbody.children)
    self.excludes.extend((pre(a), pre(b)) for a, b in c.excludes)
    for a in c.actuators:
      a.name = pre(a.name)
      a.joint = pre(a.joint)
      self.actuators.append(a)
    for s in c.sensors:
      s.name = pre(s.name)
      if s.objname:
        s.objname = pre(s.objname)
      if s.refname:
        s.refname = pre(s.refname)
      self.sensors.append(s)
    # Keyframes are merged at compile time by the compiler (per entity).
    self.keys.extend(c.keys)

  # --- JSON round trip (robot assets ship as resolved-spec JSON). ---

  def to_json(self) -> str:
    return json.dumps(asdict(self))

  @staticmethod
  def from_json(text: str) -> "Spec":
    return _spec_from_dict(json.loads(text))


def _body_from_dict(d: dict[str, Any]) -> BodySpec:
  inertial = d.get("inertial")
  return BodySpec(
    name=d["name"],
    pos=d["pos"],
    quat=d["quat"],
    mocap=d.get("mocap", False),
    inertial=InertialSpec(**inertial) if inertial else None,
    joints=[JointSpec(**j) for j in d["joints"]],
    geoms=[GeomSpec(**g) for g in d["geoms"]],
    sites=[SiteSpec(**s) for s in d["sites"]],
    children=[_body_from_dict(c) for c in d["children"]],
  )


def _spec_from_dict(d: dict[str, Any]) -> Spec:
  return Spec(
    model=d.get("model", ""),
    worldbody=_body_from_dict(d["worldbody"]),
    excludes=[tuple(e) for e in d.get("excludes", [])],
    actuators=[ActuatorSpec(**a) for a in d.get("actuators", [])],
    sensors=[SensorSpec(**s) for s in d.get("sensors", [])],
    keys=[KeySpec(**k) for k in d.get("keys", [])],
    option=OptionSpec(**d.get("option", {})),
    autolimits=d.get("autolimits", True),
  )
