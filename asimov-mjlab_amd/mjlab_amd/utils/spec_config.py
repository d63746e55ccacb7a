"""Spec editors mirroring mjlab's ``CollisionCfg`` / ``ActuatorCfg`` / ``ActuatorSetCfg``.

Semantics follow ``src/mjlab/utils/spec_config.py:136-237`` (collision: regex
subset, per-pattern condim/contype/conaffinity/priority/friction/solref/solimp,
other geoms disabled) and ``:325-428`` (PD position actuators: fixed gain,
affine bias ``[0, -kp, -kd]``, ``inheritrange=1``, ``forcerange=±effort``,
armature/frictionloss written to the joint), applied to
:class:`mjlab_amd.spec.spec.Spec` instead of ``mujoco.MjSpec``.
"""

from __future__ import annotations

from dataclasses import dataclass

from mjlab_amd.spec.spec import ActuatorSpec, Spec
from mjlab_amd.utils.string import filter_exp, resolve_field

_GEOM_ATTR_DEFAULTS = {
  "condim": 3,
  "contype": 1,
  "conaffinity": 1,
  "priority": 0,
  "friction": None,
  "solref": None,
  "solimp": None,
}


@dataclass
class CollisionCfg:
  geom_names_expr: tuple[str, ...]
  contype: int | dict[str, int] = 1
  conaffinity: int | dict[str, int] = 1
  condim: int | dict[str, int] = 3
  priority: int | dict[str, int] = 0
  friction: tuple[float, ...] | dict[str, tuple[float, ...]] | None = None
  solref: tuple[float, ...] | dict[str, tuple[float, ...]] | None = None
  solimp: tuple[float, ...] | dict[str, tuple[float, ...]] | None = None
  disable_other_geoms: bool = True

  def validate(self) -> None:
    valid = {1, 3, 4, 6}
    vals = self.condim.values() if isinstance(self.condim, dict) else [self.condim]
    for v in vals:
      if v not in valid:
        raise ValueError(f"condim must be one of {valid}, got {v}")
    for name in ("contype", "conaffinity", "priority"):
      f = getattr(self, name)
      for v in f.values() if isinstance(f, dict) else [f]:
        if v < 0:
          raise ValueError(f"{name} must be non-negative")

  def edit_spec(self, spec: Spec) -> None:
    self.validate()
    geoms = spec.geoms
    names = tuple(g.name for g in geoms)
    subset = filter_exp(self.geom_names_expr, names)
    resolved = {
      k: resolve_field(getattr(self, k), subset, d) for k, d in _GEOM_ATTR_DEFAULTS.items()
    }
    for i, gname in enumerate(subset):
      g = spec.geom(gname)
      g.condim = int(resolved["condim"][i])
      g.contype = int(resolved["contype"][i])
      g.conaffinity = int(resolved["conaffinity"][i])
      g.priority = int(resolved["priority"][i])
      for key in ("friction", "solref", "solimp"):
        vals = resolved[key][i]
        if vals is not None:
          arr = list(getattr(g, key))
          for k, v in enumerate(vals):
            arr[k] = float(v)
          setattr(g, key, arr)
    if self.disable_other_geoms:
      for gname in set(names).difference(subset):
        g = spec.geom(gname)
        g.contype = 0
        g.conaffinity = 0


@dataclass
class ActuatorCfg:
  joint_names_expr: tuple[str, ...]
  effort_limit: float
  stiffness: float
  damping: float
  frictionloss: float = 0.0
  armature: float = 0.0


@dataclass
class ActuatorSetCfg:
  cfgs: tuple[ActuatorCfg, ...]

  def validate(self) -> None:
    for c in self.cfgs:
      if c.effort_limit <= 0:
        raise ValueError(f"effort_limit must be positive, got {c.effort_limit}")
      for k in ("stiffness", "damping", "frictionloss", "armature"):
        if getattr(c, k) < 0:
          raise ValueError(f"{k} must be non-negative, got {getattr(c, k)}")

  def edit_spec(self, spec: Spec) -> None:
    self.validate()
    joints = [j for j in spec.joints if j.type != "free"]
    names = tuple(j.name for j in joints)
    pairs: list[tuple[ActuatorCfg, str]] = []
    for c in self.cfgs:
      for n in filter_exp(c.joint_names_expr, names):
        pairs.append((c, n))
    if self.cfgs and not pairs:
      raise ValueError(f"No joints matched actuator patterns. Available joints: {names}")
    pairs.sort(key=lambda p: names.index(p[1]))
    for c, n in pairs:
      j = spec.joint(n)
      limited = j.limited == "true" or (j.limited == "auto" and j.range[0] < j.range[1])
      if not limited:
        raise ValueError(f"Joint {n} must be limited for position control")
      j.armature = c.armature
      j.frictionloss = c.frictionloss
      spec.actuators.append(
        ActuatorSpec(
          name=n,
          joint=n,
          gainprm=[c.stiffness, 0.0, 0.0],
          biasprm=[0.0, -c.stiffness, -c.damping],
          inheritrange=1.0,
          forcerange=[-c.effort_limit, c.effort_limit],
        )
      )
