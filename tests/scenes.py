"""Shared test scenes, synthetic states and the GPU-vs-oracle comparison.

Tolerances (float32 HIP step vs float64 oracle, one physics step) are written
here once and cited by the tests:

* integer outputs (ncon, nefc, contact geoms, efc_type/efc_id): identical;
* kinematics (xpos, xquat, xmat, xipos, geom_xpos, site_xpos, subtree_com):
  |d| <= 5e-5 (metres / unit quaternions; fp32 ulp at 1 m is 6e-8, the tree is
  11 levels deep);
* smooth dynamics (cvel, qfrc_bias, qfrc_actuator, qfrc_smooth, qacc_smooth,
  actuator_force): |d| <= 1e-4 * (1 + max|ref|);
* constraint solve (qacc, qfrc_constraint): |d| <= 2e-2 * (1 + max|ref|) — the
  Newton solver stops on a tolerance test, and a float32 run can take one
  more/fewer iteration than the float64 one (MuJoCo Warp has the same property);
* integrated state: qvel |d| <= 1e-2 * (1 + max|ref qvel|), qpos |d| <= 1e-4 + dt * (qvel bound)
  (qpos integrates the new qvel);
* sensordata: |d| <= 2e-2 * (1 + max|ref|) (contact forces come out of the solve).
"""

from __future__ import annotations

import numpy as np

from mjlab_amd.asset_zoo.g1 import get_g1_robot_cfg
from mjlab_amd.asset_zoo.go1 import get_go1_robot_cfg
from mjlab_amd.scene.scene import Scene, SceneCfg, TerrainImporterCfg
from mjlab_amd.sensor import ContactMatch, ContactSensorCfg

KIN = ("xpos", "xquat", "xmat", "xipos", "geom_xpos", "site_xpos", "subtree_com")
SMOOTH = ("cvel", "qfrc_bias", "qfrc_actuator", "qfrc_smooth", "qacc_smooth", "actuator_force")
SOLVE = ("qacc", "qfrc_constraint")


def g1_scene(num_envs: int) -> Scene:
  feet = ContactSensorCfg(
    name="feet_ground_contact",
    primary=ContactMatch(mode="subtree", pattern=r"^(left_ankle_roll_link|right_ankle_roll_link)$", entity="robot"),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found", "force"),
    reduce="netforce",
    num_slots=1,
    track_air_time=True,
  )
  selfc = ContactSensorCfg(
    name="self_collision",
    primary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
    secondary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
    fields=("found",),
    reduce="none",
    num_slots=1,
  )
  cfg = SceneCfg(num_envs=num_envs, terrain=TerrainImporterCfg(), entities={"robot": get_g1_robot_cfg()}, sensors=(feet, selfc))
  return Scene(cfg, "cpu")


def go1_scene(num_envs: int) -> Scene:
  feet = ("FR", "FL", "RR", "RL")
  geoms = tuple(f"{n}_foot_collision" for n in feet)
  fs = ContactSensorCfg(
    name="feet_ground_contact",
    primary=ContactMatch(mode="geom", pattern=geoms, entity="robot"),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found", "force"),
    reduce="netforce",
    num_slots=1,
    track_air_time=True,
  )
  nf = ContactSensorCfg(
    name="nonfoot_ground_touch",
    primary=ContactMatch(mode="geom", entity="robot", pattern=r".*_collision\d*$", exclude=geoms),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found",),
    reduce="none",
    num_slots=1,
  )
  cfg = SceneCfg(num_envs=num_envs, terrain=TerrainImporterCfg(), entities={"robot": get_go1_robot_cfg()}, sensors=(fs, nf))
  return Scene(cfg, "cpu")


def g1_scene_model(num_envs: int, nconmax: int = 50, njmax: int = 300):
  return g1_scene(num_envs).compile(nconmax, njmax)


def go1_scene_model(num_envs: int, nconmax: int = 50, njmax: int = 300):
  return go1_scene(num_envs).compile(nconmax, njmax)


def random_states(m, n: int, rng: np.random.Generator, drop: float = 0.06) -> dict:
  """Keyframe stance perturbed: base height (feet in/above the ground), yaw,
  joint offsets, random velocities and PD targets."""
  qpos = np.tile(m.key_qpos, (n, 1)).astype(np.float64)
  qpos[:, 2] += rng.uniform(-drop, 0.02, n)
  yaw = rng.uniform(-np.pi, np.pi, n)
  qpos[:, 3] = np.cos(yaw / 2)
  qpos[:, 4:6] = 0.0
  qpos[:, 6] = np.sin(yaw / 2)
  qpos[:, 7:] += rng.uniform(-0.15, 0.15, (n, m.nq - 7))
  qvel = rng.normal(0, 0.3, (n, m.nv))
  ctrl = np.tile(m.key_ctrl, (n, 1)) + rng.uniform(-0.3, 0.3, (n, m.nu))
  return {"qpos": qpos, "qvel": qvel, "ctrl": ctrl}


def _bound(ref: np.ndarray, rel: float) -> float:
  return rel * (1.0 + float(np.abs(ref).max(initial=0.0)))


def compare_step(got: dict, ref: dict, worlds: np.ndarray | None = None, dt: float = 0.005) -> dict:
  """Compare one step's outputs (arrays shaped (nworld, -1)). Returns
  {"maxerr": {field: max|d|}, "failures": [...], "int_mismatch_worlds": [...]}."""
  n = got["qpos"].shape[0]
  sel = np.arange(n) if worlds is None else worlds
  failures: list[str] = []
  maxerr: dict[str, float] = {}
  bad_int = []
  for w in sel:
    nc, ne = int(ref["ncon"][w, 0]), int(ref["nefc"][w, 0])
    ok = int(got["ncon"][w, 0]) == nc and int(got["nefc"][w, 0]) == ne
    ok = ok and np.array_equal(got["contact_geom"][w, : 2 * nc], ref["contact_geom"][w, : 2 * nc])
    ok = ok and np.array_equal(got["efc_type"][w, :ne], ref["efc_type"][w, :ne])
    ok = ok and np.array_equal(got["efc_id"][w, :ne], ref["efc_id"][w, :ne])
    if not ok:
      bad_int.append(int(w))
  if bad_int:
    failures.append(f"integer outputs differ in worlds {bad_int[:8]}")
  good = np.array([w for w in sel if w not in set(bad_int)], dtype=int)

  def check(name: str, tol: float) -> None:
    a, b = got[name][good], ref[name][good]
    e = float(np.abs(a - b).max(initial=0.0))
    maxerr[name] = e
    if not np.isfinite(a).all() or e > tol:
      failures.append(f"{name}: max|d|={e:.3e} > {tol:.3e}")

  for k in KIN:
    check(k, 5e-5)
  for k in SMOOTH:
    check(k, _bound(ref[k][good], 1e-4))
  for k in SOLVE:
    check(k, _bound(ref[k][good], 2e-2))
  qv_tol = _bound(ref["qvel"][good], 1e-2)
  check("qvel", qv_tol)
  check("qpos", 1e-4 + dt * qv_tol)
  check("sensordata", _bound(ref["sensordata"][good], 2e-2))
  return {"maxerr": maxerr, "failures": failures, "int_mismatch_worlds": bad_int}
