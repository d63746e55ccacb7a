"""Reference-held model values for the L0 compiler check (run HERE only).

Writes tests/golden/model_{g1,go1}.json — data, no reference source — from two
independent reads of the reference:

* the robot constants, imported from the reference package with inert
  stand-ins for its missing physics modules (tools/make_golden.py's setup):
  actuator groups (armature, stiffness, damping, effort, frictionloss), the
  action scale, the init-state keyframe, the collision configs and the soft
  joint-limit factor (src/mjlab/asset_zoo/robots/unitree_g1/g1_constants.py:
  133-297, unitree_go1/go1_constants.py);
* the robot MJCF (g1.xml, go1.xml) parsed with xml.etree.ElementTree here,
  not by mjlab_amd/spec/mjcf.py: default classes resolved by MJCF's rule
  (the element's class, else the nearest enclosing body's childclass; nested
  defaults inherit), per body its inertial (mass, pos, quat, diaginertia) and
  frame, per joint its type/axis/range, per named geom its type and size
  (a capsule/cylinder ``fromto`` gives radius and half-length |to - from| / 2,
  centred at the midpoint).

tests/test_model_pinned.py compares the compiled models against these files.
Nothing here runs on the GPU box.
"""

from __future__ import annotations

import dataclasses
import json
import sys
import xml.etree.ElementTree as ET
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import make_golden  # noqa: E402

ROBOTS = Path("/root/reference/src/mjlab/asset_zoo/robots")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"


def _jsonable(x):
  if dataclasses.is_dataclass(x):
    return {f.name: _jsonable(getattr(x, f.name)) for f in dataclasses.fields(x) if not callable(getattr(x, f.name))}
  if isinstance(x, dict):
    return {str(k): _jsonable(v) for k, v in x.items()}
  if isinstance(x, (list, tuple)):
    return [_jsonable(v) for v in x]
  if isinstance(x, (bool, int, float, str)) or x is None:
    return x
  if isinstance(x, np.generic):
    return x.item()
  return repr(x)


def _floats(s: str | None) -> list[float] | None:
  return None if s is None else [float(v) for v in s.split()]


def parse_mjcf(path: Path) -> dict:
  root = ET.parse(path).getroot()
  # default classes: class -> tag -> attrs (nested defaults inherit from the enclosing one)
  defaults: dict[str, dict[str, dict[str, str]]] = {}

  def walk_default(el, parent: dict[str, dict[str, str]], name: str) -> None:
    mine = {t: dict(a) for t, a in parent.items()}
    for ch in el:
      if ch.tag != "default":
        mine.setdefault(ch.tag, {}).update(ch.attrib)
    defaults[name] = mine
    for ch in el:
      if ch.tag == "default":
        walk_default(ch, mine, ch.get("class", "main"))

  for d in root.findall("default"):
    walk_default(d, {}, d.get("class", "main"))

  def attrs(el, cls: str) -> dict[str, str]:
    a = dict(defaults.get(el.get("class", cls), defaults.get("main", {})).get(el.tag, {}))
    a.update(el.attrib)
    return a

  out = {"bodies": {}, "joints": {}, "geoms": {}}

  def walk_body(b, cls: str) -> None:
    cls = b.get("childclass", cls)
    inert = b.find("inertial")
    rec = {"pos": _floats(b.get("pos", "0 0 0")), "quat": _floats(b.get("quat", "1 0 0 0"))}
    if inert is not None:
      rec.update(mass=float(inert.get("mass")), ipos=_floats(inert.get("pos", "0 0 0")),
                 iquat=_floats(inert.get("quat", "1 0 0 0")), diaginertia=_floats(inert.get("diaginertia")))
    out["bodies"][b.get("name")] = rec
    for ch in b:
      if ch.tag in ("joint", "freejoint"):
        a = attrs(ch, cls)
        typ = "free" if ch.tag == "freejoint" else a.get("type", "hinge")
        out["joints"][a.get("name")] = {"type": typ, "axis": _floats(a.get("axis", "0 0 1")), "range": _floats(a.get("range"))}
      elif ch.tag == "geom" and ch.get("name"):
        a = attrs(ch, cls)
        typ = a.get("type", "sphere")
        size = _floats(a.get("size"))
        rec = {"type": typ, "size": size, "pos": _floats(a.get("pos", "0 0 0"))}
        if "fromto" in a:
          ft = np.array(_floats(a["fromto"]))
          rec["size"] = [size[0], float(np.linalg.norm(ft[3:] - ft[:3]) / 2)]
          rec["pos"] = ((ft[:3] + ft[3:]) / 2).tolist()
          rec["fromto"] = ft.tolist()
        out["geoms"][a["name"]] = rec
      elif ch.tag == "body":
        walk_body(ch, cls)

  for b in root.find("worldbody").findall("body"):
    walk_body(b, "main")
  return out


def main() -> None:
  make_golden.setup()
  from mjlab.asset_zoo.robots.unitree_g1 import g1_constants as g1
  from mjlab.asset_zoo.robots.unitree_go1 import go1_constants as go1

  for name, mod, cfg, scale, xml in (
    ("g1", g1, g1.get_g1_robot_cfg(), g1.G1_ACTION_SCALE, ROBOTS / "unitree_g1/xmls/g1.xml"),
    ("go1", go1, go1.get_go1_robot_cfg(), go1.GO1_ACTION_SCALE, ROBOTS / "unitree_go1/xmls/go1.xml"),
  ):
    art = cfg.articulation
    fx = {
      "robot": name,
      "sources": [str(Path(mod.__file__).relative_to("/root/reference")), str(xml.relative_to("/root/reference"))],
      "actuators": [_jsonable(a) for a in art.actuators],
      "soft_joint_pos_limit_factor": art.soft_joint_pos_limit_factor,
      "action_scale": _jsonable(scale),
      "init_state": _jsonable(cfg.init_state),
      "collisions": [_jsonable(c) for c in cfg.collisions],
      "xml": parse_mjcf(xml),
    }
    path = OUT / f"model_{name}.json"
    path.write_text(json.dumps(fx, indent=1) + "\n")
    print("wrote", path, len(fx["xml"]["bodies"]), "bodies", len(fx["xml"]["joints"]), "joints", len(fx["xml"]["geoms"]), "geoms")


if __name__ == "__main__":
  main()
