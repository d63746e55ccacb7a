"""The L0 model compiler pinned by reference-held values.

tests/golden/model_{g1,go1}.json hold (tools/make_golden_model.py) the
reference's robot constants — imported from the reference package itself —
and an ElementTree parse of the reference MJCF, independent of
mjlab_amd/spec/mjcf.py. The compiled models (the velocity tasks' scenes) are
compared with them here, applying the reference's own edit semantics
(restated, with citations): actuators per joint in spec order
(src/mjlab/utils/spec_config.py:361-414), collision fields by first-matching
pattern (spec_config.py:206-235, utils/string.py:7-23), the init-state
keyframe (entity/entity.py:145-162) and the soft joint limits
(entity/entity.py:366-381). Analytic known answers pin dof/body invweight0
and meaninertia (MuJoCo's mj_setConst definitions).
"""

import json
import re
from pathlib import Path

import numpy as np
import pytest

from tests.scenes import g1_scene_model, go1_scene_model

GOLD = Path(__file__).resolve().parent / "golden"
MODELS = {"g1": g1_scene_model, "go1": go1_scene_model}
GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4, "cylinder": 5, "box": 6, "mesh": 7}
JNT_TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}
GEOM_DEFAULTS = {"condim": 3, "contype": 1, "conaffinity": 1, "priority": 0}  # spec_config.py:25-33


def fixture(name: str) -> dict:
  return json.loads((GOLD / f"model_{name}.json").read_text())


def strip(names) -> list[str]:
  return [n.split("/", 1)[1] if n.startswith("robot/") else None for n in names]


def first_match(pattern_map: dict, names, default):
  """utils/string.py:7-23: the first pattern (re.match) wins, else the default."""
  pats = [(re.compile(p), v) for p, v in pattern_map.items()]
  out = []
  for n in names:
    for p, v in pats:
      if p.match(n):
        out.append(v)
        break
    else:
      out.append(default)
  return out


def resolve_field(v, names, default):
  return first_match(v, names, default) if isinstance(v, dict) else [v] * len(names)


@pytest.fixture(scope="module", params=["g1", "go1"])
def robot(request):
  return request.param, fixture(request.param), MODELS[request.param](1)


def test_actuators_follow_reference_constants(robot):
  name, fx, m = robot
  jn = strip(m.names["joint"])
  nonfree = [(j, n) for j, n in enumerate(jn) if n is not None and m.jnt_type[j] != 0]
  names = [n for _, n in nonfree]
  pairs = []  # spec_config.py:373-388: per cfg its matched joints, then sorted by spec order
  for a in fx["actuators"]:
    pats = [re.compile(e) for e in a["joint_names_expr"]]
    pairs += [(a, n) for n in names if any(p.match(n) for p in pats)]
  pairs.sort(key=lambda p: names.index(p[1]))
  an = strip(m.names["actuator"])
  assert len(pairs) == m.nu == len(names)
  for i, (a, jname) in enumerate(pairs):
    j = jn.index(jname)
    d = m.jnt_dofadr[j]
    assert an[i] == jname and np.asarray(m.actuator_trnid).reshape(m.nu, -1)[i, 0] == j
    assert m.actuator_gainprm[i, 0] == pytest.approx(a["stiffness"], rel=1e-9)
    assert m.actuator_biasprm[i, 1] == pytest.approx(-a["stiffness"], rel=1e-9)
    assert m.actuator_biasprm[i, 2] == pytest.approx(-a["damping"], rel=1e-9)
    np.testing.assert_allclose(m.actuator_forcerange[i], [-a["effort_limit"], a["effort_limit"]], rtol=1e-9)
    np.testing.assert_allclose(m.actuator_ctrlrange[i], m.jnt_range[j], rtol=1e-12)  # inheritrange=1
    assert m.dof_armature[d] == pytest.approx(a["armature"], rel=1e-9)
    assert m.dof_frictionloss[d] == pytest.approx(a["frictionloss"], abs=1e-12)


def test_init_state_keyframe(robot):
  name, fx, m = robot
  st = fx["init_state"]
  jn = strip(m.names["joint"])
  names = [n for j, n in enumerate(jn) if n is not None and m.jnt_type[j] != 0]
  jp = first_match(st["joint_pos"], names, 0.0)
  np.testing.assert_allclose(m.key_qpos, np.hstack([st["pos"], st["rot"], jp]), rtol=0, atol=1e-12)
  by = dict(zip(names, jp))
  np.testing.assert_allclose(m.key_ctrl, [by.get(n, 0.0) for n in strip(m.names["actuator"])], atol=1e-12)


def test_collision_config(robot):
  name, fx, m = robot
  gn = strip(m.names["geom"])
  robot_geoms = [(g, n) for g, n in enumerate(gn) if n is not None]
  xml = fx["xml"]["geoms"]
  for c in fx["collisions"]:
    pats = [re.compile(e) for e in c["geom_names_expr"]]
    subset = [n for _, n in robot_geoms if n and any(p.match(n) for p in pats)]
    assert subset, c["geom_names_expr"]
    res = {k: resolve_field(c[k], subset, dv) for k, dv in GEOM_DEFAULTS.items()}
    for k in ("friction", "solref", "solimp"):
      res[k] = resolve_field(c[k], subset, None)
    for i, n in enumerate(subset):
      g = gn.index(n)
      assert m.geom_condim[g] == res["condim"][i], n
      assert m.geom_contype[g] == res["contype"][i] and m.geom_conaffinity[g] == res["conaffinity"][i], n
      assert m.geom_priority[g] == res["priority"][i], n
      for k, arr in (("friction", m.geom_friction), ("solref", m.geom_solref), ("solimp", m.geom_solimp)):
        v = res[k][i]
        if v is not None:  # set_array_field: the leading entries (spec_config.py:166-171)
          np.testing.assert_allclose(arr[g][: len(v)], v, rtol=1e-12, err_msg=f"{k} {n}")
      assert n in xml, n  # every collision geom is a named MJCF geom
    if c["disable_other_geoms"]:
      for g, n in robot_geoms:
        if n not in subset:
          assert m.geom_contype[g] == 0 and m.geom_conaffinity[g] == 0, n


def _quat_close(a, b, tol=1e-9) -> bool:
  a = np.asarray(a, float) / np.linalg.norm(a)
  b = np.asarray(b, float) / np.linalg.norm(b)
  return min(np.abs(a - b).max(), np.abs(a + b).max()) < tol


def test_bodies_joints_geoms_match_mjcf(robot):
  """Masses, inertias (diaginertia + its frame), body frames, joint
  type/axis/range and primitive geom type/size/position against the
  ElementTree parse of the reference MJCF."""
  name, fx, m = robot
  x = fx["xml"]
  bn = strip(m.names["body"])
  assert sorted(n for n in bn if n) == sorted(x["bodies"])
  for n, b in x["bodies"].items():
    i = bn.index(n)
    assert m.body_mass[i] == pytest.approx(b["mass"], rel=1e-12), n
    np.testing.assert_allclose(m.body_inertia[i], b["diaginertia"], rtol=1e-12, err_msg=n)
    np.testing.assert_allclose(m.body_ipos[i], b["ipos"], atol=1e-12, err_msg=n)
    assert _quat_close(m.body_iquat[i], b["iquat"]), n
    if i != bn.index(next(iter(x["bodies"]))):  # the root's frame is the init state's, not the MJCF's
      np.testing.assert_allclose(m.body_pos[i], b["pos"], atol=1e-12, err_msg=n)
      assert _quat_close(m.body_quat[i], b["quat"]), n
  jn = strip(m.names["joint"])
  assert sorted(n for n in jn if n) == sorted(x["joints"])
  for n, j in x["joints"].items():
    i = jn.index(n)
    assert m.jnt_type[i] == JNT_TYPES[j["type"]], n
    if j["type"] != "free":
      ax = np.asarray(j["axis"], float)
      np.testing.assert_allclose(m.jnt_axis[i], ax / np.linalg.norm(ax), atol=1e-12, err_msg=n)
    if j["range"] is not None:
      np.testing.assert_allclose(m.jnt_range[i], j["range"], rtol=1e-12, err_msg=n)
  gn = strip(m.names["geom"])
  for n, g in x["geoms"].items():
    i = gn.index(n)
    assert m.geom_type[i] == GEOM_TYPES[g["type"]], n
    k = {"sphere": 1, "capsule": 2, "cylinder": 2, "box": 3, "ellipsoid": 3}[g["type"]]
    np.testing.assert_allclose(m.geom_size[i][:k], g["size"][:k], rtol=1e-12, err_msg=n)
    np.testing.assert_allclose(m.geom_pos[i], g["pos"], atol=1e-12, err_msg=n)


def test_mass_totals(robot):
  name, fx, m = robot
  total = sum(b["mass"] for b in fx["xml"]["bodies"].values())
  assert float(np.sum(m.body_mass)) == pytest.approx(total, rel=1e-12)


TASKS = {"g1": "Mjlab-Velocity-Flat-Unitree-G1", "go1": "Mjlab-Velocity-Flat-Unitree-Go1"}


@pytest.mark.parametrize("name", ["g1", "go1"])
def test_task_action_scale_and_soft_limits(name):
  """The velocity task's JointPositionAction scale per actuator equals the
  reference's {G1,GO1}_ACTION_SCALE (0.25 effort / stiffness, the pattern that
  matches the actuator's name), and the entity's soft joint limits are the
  MJCF ranges shrunk about their midpoint by soft_joint_pos_limit_factor
  (entity/entity.py:366-381)."""
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
  from mjlab_amd.tasks import load_env_cfg

  fx = fixture(name)
  cfg = load_env_cfg(TASKS[name])
  cfg.scene.num_envs = 2
  env = ManagerBasedRlEnv(cfg, device="cpu")
  term = env.action_manager._terms["joint_pos"]
  acts = list(term._actuator_names)
  want = []
  for a in acts:
    hits = [v for p, v in fx["action_scale"].items() if re.fullmatch(p, a)]
    assert len(hits) == 1, a
    want.append(hits[0])
  np.testing.assert_allclose(term.scale[0].numpy(), want, rtol=1e-6)
  robot = env.scene["robot"]
  names = list(robot.joint_names)
  rng = np.array([fx["xml"]["joints"][n]["range"] for n in names])
  mid, half = rng.mean(axis=1), 0.5 * (rng[:, 1] - rng[:, 0]) * fx["soft_joint_pos_limit_factor"]
  soft = robot.data.soft_joint_pos_limits[0].numpy()
  np.testing.assert_allclose(soft, np.stack([mid - half, mid + half], axis=1), rtol=1e-6, atol=1e-6)


# ---- analytic known answers: invweight0 and meaninertia (mj_setConst) ----

FREE_BOX = """<mujoco><worldbody>
<body name="box" pos="0 0 1"><freejoint/>
<inertial pos="0 0 0" mass="2.5" diaginertia="0.1 0.2 0.4"/>
<geom type="box" size="0.1 0.2 0.3" contype="0" conaffinity="0" mass="2.5"/></body>
</worldbody></mujoco>"""

CHAIN = """<mujoco><worldbody>
<body name="l1" pos="0 0 1"><joint name="j1" type="hinge" axis="0 1 0" armature="0.01"/>
<inertial pos="0.3 0 0" mass="2" diaginertia="0.05 0.05 0.05"/>
<body name="l2" pos="0.6 0 0"><joint name="j2" type="hinge" axis="0 1 0" armature="0.02"/>
<inertial pos="0.25 0 0" mass="1" diaginertia="0.03 0.03 0.03"/></body></body>
</worldbody></mujoco>"""


def _compile(xml: str):
  from mjlab_amd.spec.compiler import compile_spec
  from mjlab_amd.spec.mjcf import read_mjcf_string

  return compile_spec(read_mjcf_string(xml), 4, 16)


def test_free_box_invweight_meaninertia():
  """A free body with its com at the joint: M = diag(m, m, m, I1, I2, I3);
  dof_invweight0 = 1/m (translation), mean(1/I) (rotation); body_invweight0 =
  (1/m, mean(1/I)); meaninertia = trace(M) / 6."""
  m = _compile(FREE_BOX)
  mass, inertia = 2.5, np.array([0.1, 0.2, 0.4])
  np.testing.assert_allclose(m.dof_invweight0, [1 / mass] * 3 + [np.mean(1 / inertia)] * 3, rtol=1e-12)
  b = m.names["body"].index("box")
  np.testing.assert_allclose(m.body_invweight0[b], [1 / mass, np.mean(1 / inertia)], rtol=1e-12)
  assert m.meaninertia == pytest.approx((3 * mass + inertia.sum()) / 6, rel=1e-12)


def test_two_link_chain_invweight_meaninertia():
  """A planar 2-link chain (hinges about y, stretched along x at qpos0):
  M11 = I1 + m1 c1^2 + I2 + m2 (L + c2)^2 + a1, M12 = I2 + m2 c2 (L + c2),
  M22 = I2 + m2 c2^2 + a2; dof_invweight0 = diag(M^-1); body_invweight0 of a
  link = (tr(Jp M^-1 Jp^T) / 3, tr(Jr M^-1 Jr^T) / 3) with Jp, Jr the com
  Jacobians (the com at x moves along -z by x per unit rotation about y)."""
  m = _compile(CHAIN)
  m1, c1, I1, a1 = 2.0, 0.3, 0.05, 0.01
  m2, c2, I2, a2, L = 1.0, 0.25, 0.03, 0.02, 0.6
  M = np.array([[I1 + m1 * c1**2 + I2 + m2 * (L + c2) ** 2 + a1, I2 + m2 * c2 * (L + c2)],
                [I2 + m2 * c2 * (L + c2), I2 + m2 * c2**2 + a2]])
  Mi = np.linalg.inv(M)
  np.testing.assert_allclose(m.dof_invweight0, np.diag(Mi), rtol=1e-12)
  assert m.meaninertia == pytest.approx(np.trace(M) / 2, rel=1e-12)
  for body, jp, jr in (("l1", [-c1, 0.0], [1.0, 0.0]), ("l2", [-(L + c2), -c2], [1.0, 1.0])):
    jp, jr = np.array(jp), np.array(jr)
    b = m.names["body"].index(body)
    np.testing.assert_allclose(m.body_invweight0[b], [jp @ Mi @ jp / 3, jr @ Mi @ jr / 3], rtol=1e-12, err_msg=body)
