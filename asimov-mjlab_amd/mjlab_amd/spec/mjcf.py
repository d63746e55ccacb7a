"""MJCF (MuJoCo XML) reader producing a :class:`~mjlab_amd.spec.spec.Spec`.

Handles the MJCF subset mjlab's robots and tests use: ``<compiler>``,
``<option>``, nested ``<default>`` classes with ``childclass`` inheritance,
``<body>``/``<inertial>``/``<joint>``/``<freejoint>``/``<geom>``/``<site>``,
``<contact><exclude>``, ``<actuator><position|motor|general>``, ``<sensor>`` and
``<keyframe>``. Orientation via ``quat``, ``axisangle``, ``euler``, ``xyaxes`` or
``zaxis`` (MuJoCo XML reference, "Frame orientations").

Unsupported elements that carry physics (tendons, equality constraints, meshes
used as collision geometry) raise ``NotImplementedError`` instead of being
silently dropped; purely visual ones (lights, cameras, materials) are skipped.
"""

from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from pathlib import Path

import numpy as np

from mjlab_amd.spec.spec import (
  ActuatorSpec,
  BodySpec,
  GeomSpec,
  InertialSpec,
  JointSpec,
  KeySpec,
  SensorSpec,
  SiteSpec,
  Spec,
)
from mjlab_amd.utils import rot

_VISUAL_ONLY = {"light", "camera", "frame_visual"}


def _floats(s: str | None, n: int | None = None) -> list[float] | None:
  if s is None:
    return None
  v = [float(x) for x in s.split()]
  if n is not None and len(v) < n:
    v = v + [0.0] * (n - len(v))
  return v


def _orientation(attrs: dict[str, str], angle_deg: bool, eulerseq: str) -> list[float] | None:
  """Resolve the alternative orientation specifiers to a unit quaternion."""
  if "quat" in attrs:
    q = np.array(_floats(attrs["quat"]), dtype=np.float64)
    return list(q / np.linalg.norm(q))
  scale = math.pi / 180.0 if angle_deg else 1.0
  if "axisangle" in attrs:
    a = _floats(attrs["axisangle"])
    return list(rot.axis_angle_to_quat(np.array(a[:3]), a[3] * scale))
  if "euler" in attrs:
    e = np.array(_floats(attrs["euler"])) * scale
    q = np.array([1.0, 0.0, 0.0, 0.0])
    for ang, ax in zip(e, eulerseq):
      axis = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ax.lower()]
      qa = rot.axis_angle_to_quat(np.array(axis, float), ang)
      # Lower case: axes rotate with the frame (post-multiply); upper: fixed.
      q = rot.quat_mul(q, qa) if ax.islower() else rot.quat_mul(qa, q)
    return list(q / np.linalg.norm(q))
  if "xyaxes" in attrs:
    v = np.array(_floats(attrs["xyaxes"]))
    x = v[:3] / np.linalg.norm(v[:3])
    y = v[3:] - x * np.dot(x, v[3:])
    y /= np.linalg.norm(y)
    z = np.cross(x, y)
    return list(rot.mat_to_quat(np.stack([x, y, z], axis=1)))
  if "zaxis" in attrs:
    return list(rot.quat_z2vec(np.array(_floats(attrs["zaxis"]))))
  return None


class _Defaults:
  """Flattened default classes: class name -> element tag -> attribute dict."""

  def __init__(self) -> None:
    self.classes: dict[str, dict[str, dict[str, str]]] = {"main": {}}

  def parse(self, node: ET.Element, parent: str | None) -> None:
    name = node.get("class", "main")
    base = {} if parent is None else {k: dict(v) for k, v in self.classes[parent].items()}
    for child in node:
      if child.tag == "default":
        continue
      base.setdefault(child.tag, {}).update(child.attrib)
    self.classes[name] = base
    for child in node:
      if child.tag == "default":
        self.parse(child, name)

  def resolve(self, tag: str, cls: str, attrs: dict[str, str]) -> dict[str, str]:
    out = dict(self.classes.get(cls, {}).get(tag, {}))
    out.update(attrs)
    return out


class MjcfReader:
  def __init__(self, path: str | Path) -> None:
    self.path = Path(path)
    self.root = ET.parse(self.path).getroot()
    comp = self.root.find("compiler")
    comp_attr = comp.attrib if comp is not None else {}
    self.angle_deg = comp_attr.get("angle", "degree") == "degree"
    self.eulerseq = comp_attr.get("eulerseq", "xyz")
    self.autolimits = comp_attr.get("autolimits", "true") == "true"
    self.defaults = _Defaults()
    dnode = self.root.find("default")
    if dnode is not None:
      self.defaults.parse(dnode, None)

  def read(self) -> Spec:
    spec = Spec(model=self.root.get("model", ""), autolimits=self.autolimits)
    opt = self.root.find("option")
    if opt is not None:
      for k, v in opt.attrib.items():
        if k in ("timestep", "impratio", "tolerance", "ls_tolerance"):
          setattr(spec.option, k, float(v))
        elif k in ("iterations", "ls_iterations"):
          setattr(spec.option, k, int(v))
        elif k == "gravity":
          spec.option.gravity = _floats(v)
        elif k == "magnetic":
          spec.option.magnetic = _floats(v)
        elif k in ("integrator", "cone", "solver", "jacobian"):
          setattr(spec.option, k, v.lower())
    for tag in ("tendon", "equality"):
      node = self.root.find(tag)
      if node is not None and len(node):
        raise NotImplementedError(f"MJCF <{tag}> is not supported by mjlab_amd")
    wb = self.root.find("worldbody")
    if wb is not None:
      self._read_body_contents(wb, spec.worldbody, "main")
    contact = self.root.find("contact")
    if contact is not None:
      for ex in contact.findall("exclude"):
        spec.excludes.append((ex.get("body1"), ex.get("body2")))
      if contact.findall("pair"):
        raise NotImplementedError("explicit <contact><pair> is not supported")
    act = self.root.find("actuator")
    if act is not None:
      for a in act:
        spec.actuators.append(self._read_actuator(a))
    sens = self.root.find("sensor")
    if sens is not None:
      for s in sens:
        spec.sensors.append(self._read_sensor(s))
    kf = self.root.find("keyframe")
    if kf is not None:
      for k in kf.findall("key"):
        spec.keys.append(
          KeySpec(name=k.get("name", ""), qpos=_floats(k.get("qpos")), ctrl=_floats(k.get("ctrl")))
        )
    return spec

  # ------------------------------------------------------------------
  def _read_body_contents(self, node: ET.Element, body: BodySpec, childclass: str) -> None:
    for child in node:
      tag = child.tag
      if tag == "body":
        body.children.append(self._read_body(child, childclass))
      elif tag == "geom":
        body.geoms.append(self._read_geom(child, childclass))
      elif tag == "site":
        body.sites.append(self._read_site(child, childclass))
      elif tag in ("joint", "freejoint"):
        body.joints.append(self._read_joint(child, childclass))
      elif tag == "inertial":
        a = child.attrib
        q = _orientation(a, self.angle_deg, self.eulerseq) or [1.0, 0.0, 0.0, 0.0]
        if "fullinertia" in a:
          full = _floats(a["fullinertia"])
          I = np.array(
            [[full[0], full[3], full[4]], [full[3], full[1], full[5]], [full[4], full[5], full[2]]]
          )
          w, V = np.linalg.eigh(I)
          if np.linalg.det(V) < 0:
            V[:, 0] = -V[:, 0]
          q = list(rot.quat_mul(np.array(q), rot.mat_to_quat(V)))
          diag = list(w)
        else:
          diag = _floats(a.get("diaginertia"), 3)
        body.inertial = InertialSpec(
          pos=_floats(a.get("pos", "0 0 0")), quat=q, mass=float(a["mass"]), diaginertia=diag
        )
      elif tag in _VISUAL_ONLY:
        continue
      elif tag == "frame":
        raise NotImplementedError("MJCF <frame> is not supported")
      else:
        raise NotImplementedError(f"unsupported body child <{tag}>")

  def _read_body(self, node: ET.Element, parent_class: str) -> BodySpec:
    a = node.attrib
    childclass = a.get("childclass", parent_class)
    b = BodySpec(name=a.get("name", ""))
    b.pos = _floats(a.get("pos", "0 0 0"))
    b.quat = _orientation(a, self.angle_deg, self.eulerseq) or [1.0, 0.0, 0.0, 0.0]
    b.mocap = a.get("mocap", "false") == "true"
    self._read_body_contents(node, b, childclass)
    return b

  def _attrs(self, node: ET.Element, tag: str, childclass: str) -> dict[str, str]:
    cls = node.get("class", childclass)
    return self.defaults.resolve(tag, cls, node.attrib)

  def _read_joint(self, node: ET.Element, childclass: str) -> JointSpec:
    if node.tag == "freejoint":
      return JointSpec(name=node.get("name", ""), type="free", limited="false")
    a = self._attrs(node, "joint", childclass)
    j = JointSpec(name=a.get("name", ""), type=a.get("type", "hinge"))
    j.pos = _floats(a.get("pos", "0 0 0"))
    ax = np.array(_floats(a.get("axis", "0 0 1")))
    j.axis = list(ax / np.linalg.norm(ax))
    scale = math.pi / 180.0 if (self.angle_deg and j.type in ("hinge", "ball")) else 1.0
    if "range" in a:
      j.range = [x * scale for x in _floats(a["range"])]
    j.limited = a.get("limited", "auto")
    j.ref = float(a.get("ref", 0.0)) * scale
    j.springref = float(a.get("springref", 0.0)) * scale
    for k in ("armature", "damping", "stiffness", "frictionloss", "margin"):
      if k in a:
        setattr(j, k, float(a[k]))
    if "solreflimit" in a:
      j.solref_limit = _floats(a["solreflimit"])
    if "solimplimit" in a:
      j.solimp_limit = _floats(a["solimplimit"], 5)
    if "solreffriction" in a:
      j.solref_friction = _floats(a["solreffriction"])
    if "solimpfriction" in a:
      j.solimp_friction = _floats(a["solimpfriction"], 5)
    return j

  def _read_geom(self, node: ET.Element, childclass: str) -> GeomSpec:
    a = self._attrs(node, "geom", childclass)
    g = GeomSpec(name=a.get("name", ""), type=a.get("type", "sphere"))
    if "size" in a:
      g.size = _floats(a["size"], 3)
    g.pos = _floats(a.get("pos", "0 0 0"))
    g.quat = _orientation(a, self.angle_deg, self.eulerseq) or [1.0, 0.0, 0.0, 0.0]
    if "fromto" in a:
      g.fromto = _floats(a["fromto"])
    for k in ("contype", "conaffinity", "condim", "priority", "group"):
      if k in a:
        setattr(g, k, int(a[k]))
    for k in ("solmix", "margin", "gap", "density"):
      if k in a:
        setattr(g, k, float(a[k]))
    if "mass" in a:
      g.mass = float(a["mass"])
    if "friction" in a:
      f = _floats(a["friction"])
      g.friction = f + [1.0, 0.005, 0.0001][len(f):]
    if "solref" in a:
      g.solref = _floats(a["solref"])
    if "solimp" in a:
      g.solimp = _floats(a["solimp"], 5)
    if "rgba" in a:
      g.rgba = _floats(a["rgba"])
    g.mesh = a.get("mesh")
    g.material = a.get("material")
    if g.type in ("hfield", "sdf"):
      raise NotImplementedError(f"geom type {g.type} is not supported")
    return g

  def _read_site(self, node: ET.Element, childclass: str) -> SiteSpec:
    a = self._attrs(node, "site", childclass)
    s = SiteSpec(name=a.get("name", ""), type=a.get("type", "sphere"))
    s.pos = _floats(a.get("pos", "0 0 0"))
    s.quat = _orientation(a, self.angle_deg, self.eulerseq) or [1.0, 0.0, 0.0, 0.0]
    if "size" in a:
      s.size = _floats(a["size"], 3)
    if "group" in a:
      s.group = int(a["group"])
    return s

  def _read_actuator(self, node: ET.Element) -> ActuatorSpec:
    a = self._attrs(node, node.tag, "main")
    if "joint" not in a:
      raise NotImplementedError("only joint transmissions are supported")
    act = ActuatorSpec(name=a.get("name", ""), joint=a["joint"])
    act.gear = _floats(a.get("gear", "1"))[0]
    if node.tag == "motor":
      act.gainprm = [1.0, 0.0, 0.0]
      act.biasprm = [0.0, 0.0, 0.0]
    elif node.tag == "position":
      kp = float(a.get("kp", 1.0))
      kv = float(a.get("kv", 0.0))
      act.gainprm = [kp, 0.0, 0.0]
      act.biasprm = [0.0, -kp, -kv]
    elif node.tag == "general":
      act.gainprm = _floats(a.get("gainprm", "1 0 0"), 3)[:3]
      act.biasprm = _floats(a.get("biasprm", "0 0 0"), 3)[:3]
    else:
      raise NotImplementedError(f"actuator <{node.tag}> not supported")
    if "ctrlrange" in a:
      act.ctrlrange = _floats(a["ctrlrange"])
    if "forcerange" in a:
      act.forcerange = _floats(a["forcerange"])
    act.ctrllimited = a.get("ctrllimited", "auto")
    act.forcelimited = a.get("forcelimited", "auto")
    act.inheritrange = float(a.get("inheritrange", 0.0))
    return act

  def _read_sensor(self, node: ET.Element) -> SensorSpec:
    a = node.attrib
    s = SensorSpec(name=a.get("name", ""), type=node.tag)
    if node.tag == "contact":
      # MuJoCo >= 3.3 contact sensor: {geom,body,subtree}{1,2}, data, reduce, num
      # (mjlab adds these through MjSpec with the same intprm encoding,
      # contact_sensor.py:472-496)
      fields = ("found", "force", "torque", "dist", "pos", "normal", "tangent")
      kinds = {"geom": "geom", "body": "body", "subtree": "xbody"}
      for side in ("1", "2"):
        for k, ot in kinds.items():
          if k + side in a:
            if side == "1":
              s.objtype, s.objname = ot, a[k + side]
            else:
              s.reftype, s.refname = ot, a[k + side]
      bits = 0
      for f in a.get("data", "found").split():
        bits |= 1 << fields.index(f)
      reduce = {"none": 0, "mindist": 1, "maxforce": 2, "netforce": 3}[a.get("reduce", "none")]
      s.intprm = [bits, reduce, int(a.get("num", 1))]
      return s
    frame = ("framepos", "framequat", "framexaxis", "frameyaxis", "framezaxis", "framelinvel", "frameangvel",
             "framelinacc", "frameangacc")
    if node.tag in frame:
      s.objtype, s.objname = a["objtype"], a["objname"]
      if "reftype" in a or "refname" in a:
        s.reftype, s.refname = a["reftype"], a["refname"]
    elif node.tag in ("gyro", "velocimeter", "accelerometer", "force", "torque", "magnetometer", "rangefinder"):
      s.objtype, s.objname = "site", a["site"]
    elif node.tag in ("subtreeangmom", "subtreecom", "subtreelinvel"):
      s.objtype, s.objname = "body", a["body"]
    elif node.tag in ("jointpos", "jointvel", "jointactuatorfrc", "ballquat", "ballangvel", "jointlimitpos",
                      "jointlimitvel", "jointlimitfrc"):
      s.objtype, s.objname = "joint", a["joint"]
    elif node.tag in ("actuatorpos", "actuatorvel", "actuatorfrc"):
      s.objtype, s.objname = "actuator", a["actuator"]
    elif node.tag in ("clock", "e_potential", "e_kinetic"):
      pass
    else:
      raise NotImplementedError(f"sensor <{node.tag}> not supported")
    s.cutoff = float(a.get("cutoff", 0.0))
    return s


def read_mjcf(path: str | Path) -> Spec:
  return MjcfReader(path).read()


def read_mjcf_string(text: str, name: str = "inline.xml") -> Spec:
  import tempfile

  with tempfile.NamedTemporaryFile("w", suffix=".xml", delete=False) as f:
    f.write(text)
    p = f.name
  try:
    return read_mjcf(p)
  finally:
    Path(p).unlink(missing_ok=True)


# ---- writer: compiled model -> MJCF (for NaN dumps; MuJoCo's mj_saveModel is absent) ----
_GEOM_NAMES = {0: "plane", 2: "sphere", 3: "capsule", 4: "ellipsoid", 5: "cylinder", 6: "box", 7: "mesh"}
_SENSOR_TAGS = {1: "accelerometer", 2: "velocimeter", 3: "gyro", 4: "force", 5: "torque", 6: "magnetometer", 7: "rangefinder", 9: "jointpos", 10: "jointvel", 13: "actuatorpos",
                14: "actuatorvel", 15: "actuatorfrc", 16: "jointactuatorfrc", 18: "ballquat", 19: "ballangvel",
                20: "jointlimitpos", 21: "jointlimitvel", 22: "jointlimitfrc", 30: "framepos", 31: "framequat", 34: "subtreecom", 35: "subtreelinvel", 36: "subtreeangmom",
                41: "framexaxis", 42: "frameyaxis", 43: "framezaxis", 44: "framelinvel", 45: "frameangvel",
                46: "framelinacc", 47: "frameangacc", 48: "e_potential", 49: "e_kinetic", 50: "clock"}
_FRAME_SENSORS = {30, 31, 41, 42, 43, 44, 45, 46, 47}
_OBJ_NAMES = {1: "body", 2: "xbody", 3: "joint", 5: "geom", 6: "site", 19: "actuator"}
_CONTACT_OBJ = {1: "body", 2: "subtree", 5: "geom"}


def _fmt(v) -> str:
  return " ".join(f"{float(x):.9g}" for x in np.asarray(v).reshape(-1))


def model_to_mjcf(m) -> str:
  """MJCF of a compiled model (mjlab_amd.spec.compiler.Model) that MuJoCo's
  ``MjModel.from_xml_string`` compiles to the same bodies, dofs, geoms, sites,
  actuators and sensors, in the same order (so an mjSTATE_PHYSICS vector of
  this build restores with ``mj_setState``). Every body gets its compiled
  inertial explicitly; visual mesh geoms (no mesh data on this path) become
  massless non-colliding spheres so geom indices are kept. Used by the NaN
  guard in place of ``mj_saveModel`` (reference utils/nan_guard.py:156)."""
  names = m.names
  nb = int(m.nbody)
  children: dict[int, list[int]] = {i: [] for i in range(nb)}
  for b in range(1, nb):
    children[int(m.body_parentid[b])].append(b)
  geoms_of: dict[int, list[int]] = {i: [] for i in range(nb)}
  for g in range(int(m.ngeom)):
    geoms_of[int(m.geom_bodyid[g])].append(g)
  sites_of: dict[int, list[int]] = {i: [] for i in range(nb)}
  for s in range(int(m.nsite)):
    sites_of[int(m.site_bodyid[s])].append(s)
  out = ['<mujoco model="mjlab_amd export">', '  <compiler angle="radian" autolimits="false" inertiafromgeom="false"/>',
         f'  <option timestep="{m.timestep:.9g}" gravity="{_fmt(m.gravity)}" magnetic="{_fmt(m.magnetic)}" impratio="{m.impratio:.9g}" '
         f'tolerance="{m.tolerance:.9g}" ls_tolerance="{m.ls_tolerance:.9g}" iterations="{int(m.iterations)}" '
         f'ls_iterations="{int(m.ls_iterations)}" integrator="{ {0: "Euler", 3: "implicitfast"}.get(int(m.integrator), "Euler") }" '
         f'cone="{ {0: "pyramidal", 1: "elliptic"}[int(m.cone)] }" solver="{ {0: "PGS", 1: "CG", 2: "Newton"}[int(m.solver)] }"/>',
         "  <worldbody>"]

  def geom_xml(g: int, ind: str) -> str:
    t = int(m.geom_type[g])
    nm = f' name="{names["geom"][g]}"' if names["geom"][g] else ""
    common = (f' pos="{_fmt(m.geom_pos[g])}" quat="{_fmt(m.geom_quat[g])}" group="{int(m.geom_group[g])}" '
              f'rgba="{_fmt(m.geom_rgba[g])}"')
    if t == 7:  # visual mesh without mesh data: an inert placeholder keeps the index
      return f'{ind}<geom{nm} type="sphere" size="0.001" contype="0" conaffinity="0" mass="0"{common}/>'
    size = np.asarray(m.geom_size[g])
    sz = {0: size[:3], 2: size[:1], 3: size[:2], 4: size[:3], 5: size[:2], 6: size[:3]}[t]
    if t == 0:
      sz = [max(float(size[0]), 0.0), max(float(size[1]), 0.0), max(float(size[2]), 0.01)]
    return (f'{ind}<geom{nm} type="{_GEOM_NAMES[t]}" size="{_fmt(sz)}"{common} contype="{int(m.geom_contype[g])}" '
            f'conaffinity="{int(m.geom_conaffinity[g])}" condim="{int(m.geom_condim[g])}" '
            f'priority="{int(m.geom_priority[g])}" friction="{_fmt(m.geom_friction[g])}" solmix="{float(m.geom_solmix[g]):.9g}" '
            f'solref="{_fmt(m.geom_solref[g])}" solimp="{_fmt(m.geom_solimp[g])}" margin="{float(m.geom_margin[g]):.9g}" '
            f'gap="{float(m.geom_gap[g]):.9g}" mass="0"/>')

  def body_xml(b: int, depth: int) -> None:
    ind = "  " * (depth + 2)
    if b != 0:
      moc = ' mocap="true"' if int(m.body_mocapid[b]) >= 0 else ""
      out.append(f'{ind}<body name="{names["body"][b]}" pos="{_fmt(m.body_pos[b])}" quat="{_fmt(m.body_quat[b])}"{moc}>')
      if float(m.body_mass[b]) > 0:
        out.append(f'{ind}  <inertial pos="{_fmt(m.body_ipos[b])}" quat="{_fmt(m.body_iquat[b])}" '
                   f'mass="{float(m.body_mass[b]):.9g}" diaginertia="{_fmt(np.maximum(m.body_inertia[b], 1e-12))}"/>')
      ja, jn = int(m.body_jntadr[b]), int(m.body_jntnum[b])
      for j in range(ja, ja + jn if ja >= 0 else ja):
        t = int(m.jnt_type[j])
        if t == 0:
          out.append(f'{ind}  <freejoint name="{names["joint"][j]}"/>')
          continue
        d = int(m.jnt_dofadr[j])
        lim = "true" if int(m.jnt_limited[j]) else "false"
        out.append(f'{ind}  <joint name="{names["joint"][j]}" type="{ {1: "ball", 2: "slide", 3: "hinge"}[t] }" pos="{_fmt(m.jnt_pos[j])}" '
                   f'axis="{_fmt(m.jnt_axis[j])}" limited="{lim}" range="{_fmt(m.jnt_range[j])}" '
                   f'ref="{float(m.qpos0[int(m.jnt_qposadr[j])]):.9g}" springref="{float(m.qpos_spring[int(m.jnt_qposadr[j])]):.9g}" '
                   f'stiffness="{float(m.jnt_stiffness[j]):.9g}" armature="{float(m.dof_armature[d]):.9g}" '
                   f'damping="{float(m.dof_damping[d]):.9g}" frictionloss="{float(m.dof_frictionloss[d]):.9g}" '
                   f'margin="{float(m.jnt_margin[j]):.9g}" solreflimit="{_fmt(m.jnt_solref[j])}" '
                   f'solimplimit="{_fmt(m.jnt_solimp[j])}" solreffriction="{_fmt(m.dof_solref[d])}" '
                   f'solimpfriction="{_fmt(m.dof_solimp[d])}"/>')
    for g in geoms_of[b]:
      out.append(geom_xml(g, ind + ("  " if b else "")))
    for s in sites_of[b]:
      nm = f' name="{names["site"][s]}"' if names["site"][s] else ""
      out.append(f'{ind}{"  " if b else ""}<site{nm} pos="{_fmt(m.site_pos[s])}" quat="{_fmt(m.site_quat[s])}"/>')
    for c in children[b]:
      body_xml(c, depth + (1 if b else 0))
    if b != 0:
      out.append(f"{ind}</body>")

  body_xml(0, 0)
  out.append("  </worldbody>")
  # the compiled pair table is the authority: parent/weld/contype filters are
  # recomputed by MuJoCo, the spec's <exclude> pairs are re-emitted
  excl = getattr(m, "excludes", [])
  if excl:
    out.append("  <contact>")
    out += [f'    <exclude body1="{a}" body2="{b}"/>' for a, b in excl]
    out.append("  </contact>")
  if int(m.nu):
    out.append("  <actuator>")
    for i in range(int(m.nu)):
      j = int(m.actuator_trnid[i])
      out.append(f'    <general name="{names["actuator"][i]}" joint="{names["joint"][j]}" gear="{float(m.actuator_gear[i]):.9g}" '
                 f'gaintype="fixed" biastype="affine" gainprm="{_fmt(m.actuator_gainprm[i][:3])}" '
                 f'biasprm="{_fmt(m.actuator_biasprm[i][:3])}" ctrllimited="{"true" if int(m.actuator_ctrllimited[i]) else "false"}" '
                 f'ctrlrange="{_fmt(m.actuator_ctrlrange[i])}" forcelimited="{"true" if int(m.actuator_forcelimited[i]) else "false"}" '
                 f'forcerange="{_fmt(m.actuator_forcerange[i])}"/>')
    out.append("  </actuator>")
  if int(m.nsensor):
    out.append("  <sensor>")
    for s in range(int(m.nsensor)):
      t, ot, oid = int(m.sensor_type[s]), int(m.sensor_objtype[s]), int(m.sensor_objid[s])
      nm = names["sensor"][s]
      cut = float(m.sensor_cutoff[s])
      cut_a = f' cutoff="{cut:.9g}"' if cut > 0 else ""
      if t == 40:  # mjSENS_CONTACT (MuJoCo >= 3.3): intprm = [1 << field bits, reduce, num]
        bits, red, num = (int(x) for x in m.sensor_intprm[s])
        fields = " ".join(f for k, f in enumerate(("found", "force", "torque", "dist", "pos", "normal", "tangent")) if bits & (1 << k))
        o1 = f' {_CONTACT_OBJ[ot]}1="{names["geom" if ot == 5 else "body"][oid]}"'
        rt, rid = int(m.sensor_reftype[s]), int(m.sensor_refid[s])
        o2 = f' {_CONTACT_OBJ[rt]}2="{names["geom" if rt == 5 else "body"][rid]}"' if rid >= 0 and rt in _CONTACT_OBJ else ""
        out.append(f'    <contact name="{nm}"{o1}{o2} data="{fields}" '
                   f'reduce="{ {0: "none", 1: "mindist", 2: "maxforce", 3: "netforce"}[red] }" num="{num}"/>')
        continue
      if ot == 0:  # no object (clock, energies)
        out.append(f'    <{_SENSOR_TAGS[t]} name="{nm}"{cut_a}/>')
        continue
      kind = _OBJ_NAMES[ot]
      attr = {"site": "site", "joint": "joint", "body": "body", "xbody": "body", "actuator": "actuator"}.get(kind, kind)
      obj = names[{"xbody": "body"}.get(kind, kind)][oid]
      if t in _FRAME_SENSORS:
        rt, rid = int(m.sensor_reftype[s]), int(m.sensor_refid[s])
        ref = ""
        if rid >= 0 and rt in _OBJ_NAMES:
          rk = _OBJ_NAMES[rt]
          ref = f' reftype="{rk}" refname="{names[{"xbody": "body"}.get(rk, rk)][rid]}"'
        out.append(f'    <{_SENSOR_TAGS[t]} name="{nm}" objtype="{kind}" objname="{obj}"{ref}{cut_a}/>')
      else:
        out.append(f'    <{_SENSOR_TAGS[t]} name="{nm}" {attr}="{obj}"{cut_a}/>')
    out.append("  </sensor>")
  out.append("</mujoco>")
  return "\n".join(out) + "\n"
