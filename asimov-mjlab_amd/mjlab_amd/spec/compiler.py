"""Compile a :class:`Spec` into flat model arrays (the ``MjModel`` analogue).

Replaces ``MjSpec.compile()`` (called at ``src/mjlab/scene/scene.py:42-43``)
for the feature subset mjlab's G1/Go1 tasks use. The steps mirror MuJoCo's
compiler (MuJoCo 3.x, ``user_model.cc`` / ``engine_setconst.c``, published
algorithm, not vendored in the reference):

1. depth-first body order, joint/dof/geom/site addresses;
2. ``fromto`` capsules, inertia from geoms when a body has no ``<inertial>``;
3. autolimits for joints, actuator ``inheritrange``/``ctrlrange``/``forcerange``;
4. ``qpos0`` (free joint = body pose, ball = identity, hinge/slide = ``ref``);
5. ``mj_setConst``: ``dof_invweight0``, ``body_invweight0``, ``meaninertia``
   from the mass matrix at ``qpos0``;
6. the filtered geom-pair table (weld filter, parent filter, contype/conaffinity,
   ``<exclude>``), each pair ordered so geom types ascend (MuJoCo collision
   table convention; the contact normal points from geom1 to geom2);
7. sensor addresses (``sensordata`` layout in declaration order).

Outputs are numpy arrays named exactly as in ``include/mjh_fields.h``.
"""

from __future__ import annotations

import math
import warnings
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from mjlab_amd.spec.spec import GEOM_TYPES, JOINT_TYPES, Spec
from mjlab_amd.utils import rot

MINVAL = 1e-15
# the general convex pairs: GJK + EPA, one contact (csrc/mjh_convex.h; MuJoCo's mjc_Convex)
CONVEX_PAIRS = {(2, 4), (3, 4), (4, 4), (3, 5), (4, 5), (5, 5), (4, 6), (5, 6)}
SUPPORTED_PAIRS = {(0, 2), (0, 3), (0, 4), (0, 5), (0, 6), (2, 2), (2, 3), (2, 5), (3, 3), (2, 6), (3, 6),
                   (6, 6)} | CONVEX_PAIRS
# pairs that need the box, cylinder, ellipsoid or convex narrowphase functions (Model.nboxpair counts them)
BOX_PAIRS = {(2, 6), (3, 6), (6, 6), (0, 4), (0, 5), (2, 5)} | CONVEX_PAIRS

# Sensor type codes used by the kernels (order is ours; names follow mjtSensor).
SENSOR_TYPES = {
  "accelerometer": 1,
  "velocimeter": 2,
  "gyro": 3,
  "force": 4,
  "torque": 5,
  "magnetometer": 6,
  "rangefinder": 7,
  "jointpos": 9,
  "jointvel": 10,
  "actuatorpos": 13,
  "actuatorvel": 14,
  "actuatorfrc": 15,
  "jointactuatorfrc": 16,
  "ballquat": 18,
  "ballangvel": 19,
  "framepos": 30,
  "framequat": 31,
  "subtreecom": 34,
  "subtreelinvel": 35,
  "subtreeangmom": 36,
  "contact": 40,
  "framexaxis": 41,
  "frameyaxis": 42,
  "framezaxis": 43,
  "framelinvel": 44,
  "frameangvel": 45,
  "framelinacc": 46,
  "frameangacc": 47,
  "jointlimitpos": 20,
  "jointlimitvel": 21,
  "jointlimitfrc": 22,
  "e_potential": 48,
  "e_kinetic": 49,
  "clock": 50,
}
SENSOR_DIMS = {
  "accelerometer": 3,
  "velocimeter": 3,
  "gyro": 3,
  "force": 3,
  "torque": 3,
  "magnetometer": 3,
  "rangefinder": 1,
  "jointpos": 1,
  "jointvel": 1,
  "actuatorpos": 1,
  "actuatorvel": 1,
  "actuatorfrc": 1,
  "jointactuatorfrc": 1,
  "ballquat": 4,
  "ballangvel": 3,
  "framepos": 3,
  "framequat": 4,
  "subtreecom": 3,
  "subtreelinvel": 3,
  "subtreeangmom": 3,
  "framexaxis": 3,
  "frameyaxis": 3,
  "framezaxis": 3,
  "framelinvel": 3,
  "frameangvel": 3,
  "framelinacc": 3,
  "frameangacc": 3,
  "jointlimitpos": 1,
  "jointlimitvel": 1,
  "jointlimitfrc": 1,
  "e_potential": 1,
  "e_kinetic": 1,
  "clock": 1,
}
# the sensor types the step kernel evaluates on every path (the benchmark tasks'
# set); the others count into Model.nsensor_ext and set their group's bit in
# Model.sensor_ext_mask (a model size: mjh_step.hip's kExt* groups)
BASE_SENSOR_CODES = {1, 2, 3, 9, 10, 34, 35, 36, 40}
SENSOR_EXT_GROUPS = {48: 1, 49: 1, 4: 2, 5: 2, 30: 4, 41: 4, 42: 4, 43: 4, 31: 8, 44: 16, 45: 16, 46: 32, 47: 32,
                     20: 64, 21: 64, 22: 64, 13: 128, 14: 128, 15: 128, 16: 128, 18: 256, 19: 256, 50: 512, 7: 1024,
                     6: 2048}
# sensors whose values are unit quaternions or axes: no cutoff (mjDATATYPE_QUATERNION / _AXIS)
SENSOR_NO_CUTOFF = {"framequat", "ballquat", "framexaxis", "frameyaxis", "framezaxis"}
# Contact sensor data fields: bit -> width (src/mjlab/sensor/contact_sensor.py:16-34).
CONTACT_FIELD_DIMS = [1, 3, 3, 1, 3, 3, 3]
OBJ_CODES = {"": 0, "body": 1, "xbody": 2, "joint": 3, "geom": 5, "site": 6, "actuator": 19}
QPOS_WIDTH = {0: 7, 1: 4, 2: 1, 3: 1}
DOF_WIDTH = {0: 6, 1: 3, 2: 1, 3: 1}


@dataclass
class _Named:
  id: int
  name: str
  attrs: dict[str, Any] = field(default_factory=dict)

  def __getattr__(self, k):
    try:
      return self.__dict__["attrs"][k]
    except KeyError as e:
      raise AttributeError(k) from e


class Model:
  """Compiled model: numpy arrays + sizes + options + names.

  Attribute names follow ``mjModel`` (and ``include/mjh_fields.h``). Named
  accessors ``model.joint(name)``, ``model.sensor(name)`` ... return objects
  whose fields are 1-element arrays, like MuJoCo's named access that mjlab uses
  (``src/mjlab/entity/entity.py:621-624``, ``contact_sensor.py:210-214``).
  """

  # leading static world sites (a Scene's env-origin sites): the Simulation
  # writes their poses once and the step kernel sees only the sites after them
  nsite_origin = 0
  nsensor_ext = 0
  sensor_ext_mask = 0
  magnetic = np.array([0.0, -0.5, 0.0])  # models built before the option existed

  def __init__(self) -> None:
    self.names: dict[str, list[str]] = {}

  def _index(self, kind: str, name: str) -> int:
    names = self.names[kind]
    if name not in names:
      raise KeyError(f"{kind} '{name}' not found")
    return names.index(name)

  def body(self, name: str) -> _Named:
    i = self._index("body", name)
    return _Named(i, name, {"parentid": self.body_parentid[i : i + 1], "pos": self.body_pos[i],
                            "quat": self.body_quat[i], "mass": self.body_mass[i : i + 1],
                            "mocapid": self.body_mocapid[i : i + 1]})

  @property
  def nkey(self) -> int:
    return 0 if getattr(self, "key_qpos", None) is None else 1

  def key(self, name: str) -> _Named:
    """The entity keyframe (``init_state``) merged at compile time (entity.py:145-166)."""
    if self.nkey == 0 or name != "init_state":
      raise KeyError(f"key '{name}' not found")
    return _Named(0, name, {"qpos": np.asarray(self.key_qpos), "ctrl": np.asarray(self.key_ctrl)})

  @property
  def opt(self):
    """``mjModel.opt`` view (mjtIntegrator / mjtSolver / mjtCone codes)."""
    from types import SimpleNamespace

    return SimpleNamespace(timestep=self.timestep, gravity=np.asarray(self.gravity), magnetic=np.asarray(self.magnetic),
                           impratio=self.impratio,
                           tolerance=self.tolerance, ls_tolerance=self.ls_tolerance, iterations=self.iterations,
                           ls_iterations=self.ls_iterations, integrator=self.integrator, solver=self.solver,
                           cone=self.cone)

  def joint(self, name: str) -> _Named:
    i = self._index("joint", name)
    return _Named(
      i,
      name,
      {
        "type": self.jnt_type[i : i + 1],
        "qposadr": self.jnt_qposadr[i : i + 1],
        "dofadr": self.jnt_dofadr[i : i + 1],
        "bodyid": self.jnt_bodyid[i : i + 1],
      },
    )

  def geom(self, name: str) -> _Named:
    i = self._index("geom", name)
    return _Named(i, name, {"bodyid": self.geom_bodyid[i : i + 1]})

  def site(self, name: str) -> _Named:
    i = self._index("site", name)
    return _Named(i, name, {"bodyid": self.site_bodyid[i : i + 1]})

  def actuator(self, name: str) -> _Named:
    i = self._index("actuator", name)
    return _Named(i, name, {"trnid": self.actuator_trnid[i : i + 1]})

  def sensor(self, name: str) -> _Named:
    i = self._index("sensor", name)
    return _Named(
      i,
      name,
      {
        "adr": self.sensor_adr[i : i + 1],
        "dim": self.sensor_dim[i : i + 1],
        "type": self.sensor_type[i : i + 1],
      },
    )

  def copy(self) -> "Model":
    m = Model()
    for k, v in self.__dict__.items():
      m.__dict__[k] = v.copy() if isinstance(v, np.ndarray) else v
    m.names = {k: list(v) for k, v in self.names.items()}
    return m


def _geom_frame(g) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
  """Resolve fromto; return pos, quat, size."""
  size = np.array((list(g.size) + [0.0, 0.0, 0.0])[:3], dtype=np.float64)
  if g.fromto is not None:
    a = np.array(g.fromto[:3], dtype=np.float64)
    b = np.array(g.fromto[3:6], dtype=np.float64)
    pos = 0.5 * (a + b)
    quat = rot.quat_z2vec(b - a)
    half = 0.5 * np.linalg.norm(b - a)
    if g.type in ("capsule", "cylinder"):
      size[1] = half
    elif g.type in ("box", "ellipsoid"):
      size[2] = half
    return pos, quat, size
  q = np.array(g.quat, dtype=np.float64)
  return np.array(g.pos, dtype=np.float64), q / np.linalg.norm(q), size


def _geom_mass_inertia(gtype: str, size: np.ndarray, density: float, mass: float | None):
  """Mass and principal inertia (about the geom frame) of a primitive."""
  r = size[0]
  if gtype == "sphere":
    vol = 4.0 / 3.0 * math.pi * r**3
    m = mass if mass is not None else density * vol
    I = np.full(3, 0.4 * m * r * r)
  elif gtype == "capsule":
    h = 2.0 * size[1]
    vcyl = math.pi * r * r * h
    vsph = 4.0 / 3.0 * math.pi * r**3
    vol = vcyl + vsph
    m = mass if mass is not None else density * vol
    mcyl, msph = m * vcyl / vol, m * vsph / vol
    ixx = mcyl * (h * h / 12.0 + r * r / 4.0) + msph * (
      0.4 * r * r + h * h / 4.0 + 3.0 * h * r / 8.0
    )
    izz = 0.5 * mcyl * r * r + 0.4 * msph * r * r
    I = np.array([ixx, ixx, izz])
  elif gtype == "cylinder":
    h = 2.0 * size[1]
    vol = math.pi * r * r * h
    m = mass if mass is not None else density * vol
    ixx = m * (3 * r * r + h * h) / 12.0
    I = np.array([ixx, ixx, 0.5 * m * r * r])
  elif gtype == "box":
    vol = 8.0 * size[0] * size[1] * size[2]
    m = mass if mass is not None else density * vol
    x2, y2, z2 = (2 * size) ** 2
    I = m / 12.0 * np.array([y2 + z2, x2 + z2, x2 + y2])
  elif gtype == "ellipsoid":
    vol = 4.0 / 3.0 * math.pi * size[0] * size[1] * size[2]
    m = mass if mass is not None else density * vol
    a2, b2, c2 = size**2
    I = m / 5.0 * np.array([b2 + c2, a2 + c2, a2 + b2])
  else:  # plane, mesh (no mesh data on this path): massless
    return 0.0, np.zeros(3)
  return m, I


def _geom_rbound(gtype: str, size: np.ndarray) -> float:
  if gtype == "sphere":
    return size[0]
  if gtype == "capsule":
    return size[0] + size[1]
  if gtype == "cylinder":
    return math.hypot(size[0], size[1])
  if gtype == "box":
    return float(np.linalg.norm(size))
  if gtype == "ellipsoid":
    return float(np.max(size))
  return 0.0


def compile_spec(spec: Spec, nconmax: int = 0, njmax: int = 0) -> Model:
  m = Model()
  opt = spec.option
  bodies = spec.bodies  # DFS order, world first
  body_index = {id(b): i for i, b in enumerate(bodies)}
  parent = np.zeros(len(bodies), dtype=np.int32)
  for b in bodies:
    for c in b.children:
      parent[body_index[id(c)]] = body_index[id(b)]
  nbody = len(bodies)

  # --- joints / dofs ---
  jnt_list, dof_list = [], []
  body_jntadr = np.full(nbody, -1, np.int32)
  body_jntnum = np.zeros(nbody, np.int32)
  body_dofadr = np.full(nbody, -1, np.int32)
  body_dofnum = np.zeros(nbody, np.int32)
  nq = 0
  for bi, b in enumerate(bodies):
    if b.joints:
      body_jntadr[bi] = len(jnt_list)
      body_jntnum[bi] = len(b.joints)
    for j in b.joints:
      t = JOINT_TYPES[j.type]
      if t == 0 and (bi == 0 or len(b.joints) != 1 or parent[bi] != 0):
        raise ValueError("free joint must be the only joint of a world child body")
      jid = len(jnt_list)
      dofadr = len(dof_list)
      if body_dofadr[bi] < 0:
        body_dofadr[bi] = dofadr
      for _ in range(DOF_WIDTH[t]):
        dof_list.append((bi, jid))
      body_dofnum[bi] += DOF_WIDTH[t]
      jnt_list.append((bi, j, t, nq, dofadr))
      nq += QPOS_WIDTH[t]
  njnt, nv = len(jnt_list), len(dof_list)

  # --- geoms / sites (body order) ---
  geoms = [(bi, g) for bi, b in enumerate(bodies) for g in b.geoms]
  sites = [(bi, s) for bi, b in enumerate(bodies) for s in b.sites]
  ngeom, nsite = len(geoms), len(sites)

  # --- sizes / options ---
  m.nq, m.nv, m.nu, m.na = nq, nv, len(spec.actuators), 0
  m.nbody, m.njnt, m.ngeom, m.nsite = nbody, njnt, ngeom, nsite
  m.nmocap = 0
  m.timestep = opt.timestep
  m.gravity = np.array(opt.gravity, np.float64)
  m.magnetic = np.array(opt.magnetic, np.float64)
  m.impratio = opt.impratio
  m.tolerance = opt.tolerance
  m.ls_tolerance = opt.ls_tolerance
  m.iterations = opt.iterations
  m.ls_iterations = opt.ls_iterations
  m.integrator = {"euler": 0, "implicitfast": 3}[opt.integrator]
  m.cone = {"pyramidal": 0, "elliptic": 1}[opt.cone]
  m.solver = {"pgs": 0, "cg": 1, "newton": 2}[opt.solver]
  m.jacobian = {"dense": 0, "sparse": 1, "auto": 2}[opt.jacobian]
  m.disableflags = 0
  m.contact_sensor_maxmatch = 64
  # MuJoCo Warp's parallel line search (Option.ls_parallel / ls_parallel_min_step):
  # off in a bare model as in mjwarp.put_model; SimulationCfg.ls_parallel sets it
  m.ls_parallel = 0
  m.ls_parallel_min_step = 1e-6

  # --- bodies ---
  m.body_parentid = parent
  m.body_jntadr, m.body_jntnum = body_jntadr, body_jntnum
  m.body_dofadr, m.body_dofnum = body_dofadr, body_dofnum
  m.body_pos = np.array([b.pos for b in bodies], np.float64)
  m.body_quat = np.array([np.array(b.quat) / np.linalg.norm(b.quat) for b in bodies])
  m.body_mocapid = np.full(nbody, -1, np.int32)
  nmocap = 0
  for bi, b in enumerate(bodies):
    if b.mocap:
      # MuJoCo: mocap bodies are static children of the world (no joints)
      if parent[bi] != 0 or body_jntnum[bi] != 0:
        raise ValueError(f"mocap body '{b.name}' must be a child of the world body without joints")
      m.body_mocapid[bi] = nmocap
      nmocap += 1
  m.nmocap = nmocap
  # weld / root ids
  weld = np.zeros(nbody, np.int32)
  root = np.zeros(nbody, np.int32)
  for i in range(1, nbody):
    weld[i] = i if body_jntnum[i] > 0 else weld[parent[i]]
    root[i] = i if parent[i] == 0 else root[parent[i]]
  m.body_weldid, m.body_rootid = weld, root

  # inertia
  ipos = np.zeros((nbody, 3))
  iquat = np.tile([1.0, 0.0, 0.0, 0.0], (nbody, 1))
  mass = np.zeros(nbody)
  inertia = np.zeros((nbody, 3))
  for bi, b in enumerate(bodies):
    if bi == 0:
      continue
    if b.inertial is not None:
      ipos[bi] = b.inertial.pos
      q = np.array(b.inertial.quat, np.float64)
      iquat[bi] = q / np.linalg.norm(q)
      mass[bi] = b.inertial.mass
      inertia[bi] = b.inertial.diaginertia
      continue
    # inertia from geoms (inertiafromgeom="auto")
    parts = []
    for g in b.geoms:
      gp, gq, gs = _geom_frame(g)
      gm, gI = _geom_mass_inertia(g.type, gs, g.density, g.mass)
      if gm > 0:
        parts.append((gm, gp, rot.quat_to_mat(gq), gI))
    M = sum(p[0] for p in parts)
    if M <= 0:
      continue
    com = sum(p[0] * p[1] for p in parts) / M
    Itot = np.zeros((3, 3))
    for gm, gp, R, gI in parts:
      d = gp - com
      Itot += R @ np.diag(gI) @ R.T + gm * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    w, V = np.linalg.eigh(Itot)
    if np.linalg.det(V) < 0:
      V[:, 0] = -V[:, 0]
    ipos[bi], iquat[bi], mass[bi], inertia[bi] = com, rot.mat_to_quat(V), M, w
  m.body_ipos, m.body_iquat, m.body_mass, m.body_inertia = ipos, iquat, mass, inertia
  sub = mass.copy()
  for i in range(nbody - 1, 0, -1):
    sub[parent[i]] += sub[i]
  m.body_subtreemass = sub

  # chains / masks (GPU helpers)
  chains = []
  for i in range(nbody):
    c, k = [], i
    while k != 0:
      c.append(int(k))
      k = int(parent[k])
    chains.append(c[::-1])
  m.body_chainadr = np.zeros(nbody, np.int32)
  m.body_chainnum = np.zeros(nbody, np.int32)
  flat = []
  for i, c in enumerate(chains):
    m.body_chainadr[i] = len(flat)
    m.body_chainnum[i] = len(c)
    flat.extend(c)
  m.body_chain = np.array(flat if flat else [0], np.int32)
  m.nchain = len(flat) if flat else 1
  dofmask = np.zeros(nbody, np.int64)
  treemask = np.zeros(nbody, np.int64)
  for i in range(nbody):
    dm, tm = 0, 0
    for k in chains[i]:
      tm |= 1 << int(k)
      for d in range(int(body_dofadr[k]), int(body_dofadr[k] + body_dofnum[k])):
        dm |= 1 << d
    # nv/nbody > 63 cannot be represented; the device path refuses such models
    # (mjh_model_check), the mask is then a poison value.
    dofmask[i] = dm if nv <= 63 else -1
    treemask[i] = tm if nbody <= 63 else -1
  m.body_dofmask, m.body_treemask = dofmask, treemask

  # --- joints ---
  m.jnt_type = np.array([t for _, _, t, _, _ in jnt_list], np.int32)
  m.jnt_qposadr = np.array([q for _, _, _, q, _ in jnt_list], np.int32)
  m.jnt_dofadr = np.array([d for _, _, _, _, d in jnt_list], np.int32)
  m.jnt_bodyid = np.array([b for b, _, _, _, _ in jnt_list], np.int32)
  m.jnt_pos = np.array([j.pos for _, j, _, _, _ in jnt_list], np.float64).reshape(njnt, 3)
  m.jnt_axis = np.array([j.axis for _, j, _, _, _ in jnt_list], np.float64).reshape(njnt, 3)
  rng = np.array([j.range for _, j, _, _, _ in jnt_list], np.float64).reshape(njnt, 2)
  lim = np.zeros(njnt, np.int32)
  for k, (_, j, t, _, _) in enumerate(jnt_list):
    if j.limited == "true":
      lim[k] = 1
    elif j.limited == "auto" and spec.autolimits and t != 0:
      lim[k] = int(rng[k, 0] < rng[k, 1])
  m.jnt_range, m.jnt_limited = rng, lim
  m.jnt_solref = np.array([j.solref_limit for _, j, _, _, _ in jnt_list], np.float64).reshape(njnt, 2)
  m.jnt_solimp = np.array([j.solimp_limit for _, j, _, _, _ in jnt_list], np.float64).reshape(njnt, 5)
  m.jnt_margin = np.array([j.margin for _, j, _, _, _ in jnt_list], np.float64)
  m.jnt_stiffness = np.array([j.stiffness for _, j, _, _, _ in jnt_list], np.float64)
  if any(t == 0 and j.stiffness != 0 for _, j, t, _, _ in jnt_list):
    raise NotImplementedError("free-joint springs (stiffness on a free joint) are not supported")

  # qpos0 / qpos_spring
  qpos0 = np.zeros(nq)
  qspring = np.zeros(nq)
  for bi, j, t, qa, _ in jnt_list:
    if t == 0:
      qpos0[qa : qa + 3] = m.body_pos[bi]
      qpos0[qa + 3 : qa + 7] = m.body_quat[bi]
      qspring[qa : qa + 7] = qpos0[qa : qa + 7]
    elif t == 1:  # ball: the identity rotation (MuJoCo ignores ref / springref here)
      qpos0[qa : qa + 4] = [1.0, 0.0, 0.0, 0.0]
      qspring[qa : qa + 4] = qpos0[qa : qa + 4]
    else:
      qpos0[qa] = j.ref
      qspring[qa] = j.springref
  m.qpos0, m.qpos_spring = qpos0, qspring

  # --- dofs ---
  m.dof_bodyid = np.array([b for b, _ in dof_list], np.int32)
  m.dof_jntid = np.array([j for _, j in dof_list], np.int32)
  dpar = np.full(nv, -1, np.int32)
  for d in range(nv):
    bi, jid = dof_list[d]
    if d > 0 and dof_list[d - 1][0] == bi:
      dpar[d] = d - 1
    else:
      k = parent[bi]
      while k != 0 and body_dofnum[k] == 0:
        k = parent[k]
      dpar[d] = body_dofadr[k] + body_dofnum[k] - 1 if k != 0 else -1
  m.dof_parentid = dpar
  m.dof_armature = np.array([jnt_list[j][1].armature for _, j in dof_list], np.float64)
  m.dof_damping = np.array([jnt_list[j][1].damping for _, j in dof_list], np.float64)
  m.dof_frictionloss = np.array([jnt_list[j][1].frictionloss for _, j in dof_list], np.float64)
  m.dof_solref = np.array([jnt_list[j][1].solref_friction for _, j in dof_list], np.float64).reshape(nv, 2)
  m.dof_solimp = np.array([jnt_list[j][1].solimp_friction for _, j in dof_list], np.float64).reshape(nv, 5)

  # --- geoms ---
  gpos, gquat, gsize = [], [], []
  for _, g in geoms:
    p, q, s = _geom_frame(g)
    gpos.append(p)
    gquat.append(q)
    gsize.append(s)
  m.geom_type = np.array([GEOM_TYPES[g.type] for _, g in geoms], np.int32)
  m.geom_contype = np.array([g.contype for _, g in geoms], np.int32)
  m.geom_conaffinity = np.array([g.conaffinity for _, g in geoms], np.int32)
  m.geom_condim = np.array([g.condim for _, g in geoms], np.int32)
  m.geom_bodyid = np.array([b for b, _ in geoms], np.int32)
  m.geom_priority = np.array([g.priority for _, g in geoms], np.int32)
  m.geom_size = np.array(gsize, np.float64).reshape(ngeom, 3)
  m.geom_pos = np.array(gpos, np.float64).reshape(ngeom, 3)
  m.geom_quat = np.array(gquat, np.float64).reshape(ngeom, 4)
  m.geom_friction = np.array([g.friction for _, g in geoms], np.float64).reshape(ngeom, 3)
  m.geom_solmix = np.array([g.solmix for _, g in geoms], np.float64)
  m.geom_solref = np.array([g.solref for _, g in geoms], np.float64).reshape(ngeom, 2)
  m.geom_solimp = np.array([g.solimp for _, g in geoms], np.float64).reshape(ngeom, 5)
  m.geom_margin = np.array([g.margin for _, g in geoms], np.float64)
  m.geom_gap = np.array([g.gap for _, g in geoms], np.float64)
  m.geom_rgba = np.array([g.rgba for _, g in geoms], np.float64).reshape(ngeom, 4)
  m.geom_group = np.array([g.group for _, g in geoms], np.int32)
  m.geom_rbound = np.array([_geom_rbound(g.type, s) for (_, g), s in zip(geoms, gsize)])
  for (_, g), t in zip(geoms, m.geom_type):
    if t == GEOM_TYPES["mesh"] and (g.contype or g.conaffinity):
      raise NotImplementedError(f"mesh collision geom '{g.name}' is not supported")

  # --- sites ---
  m.site_bodyid = np.array([b for b, _ in sites], np.int32)
  m.site_pos = np.array([s.pos for _, s in sites], np.float64).reshape(nsite, 3)
  m.site_quat = np.array(
    [np.array(s.quat) / np.linalg.norm(s.quat) for _, s in sites], np.float64
  ).reshape(nsite, 4)

  # --- names ---
  m.names = {
    "body": [b.name for b in bodies],
    "joint": [j.name for _, j, _, _, _ in jnt_list],
    "geom": [g.name for _, g in geoms],
    "site": [s.name for _, s in sites],
    "actuator": [a.name for a in spec.actuators],
    "sensor": [s.name for s in spec.sensors],
  }

  # --- actuators ---
  nu = m.nu
  m.actuator_trntype = np.zeros(nu, np.int32)
  m.actuator_trnid = np.zeros(nu, np.int32)
  m.actuator_gear = np.ones(nu)
  m.actuator_gainprm = np.zeros((nu, 10))
  m.actuator_biasprm = np.zeros((nu, 10))
  m.actuator_ctrlrange = np.zeros((nu, 2))
  m.actuator_ctrllimited = np.zeros(nu, np.int32)
  m.actuator_forcerange = np.zeros((nu, 2))
  m.actuator_forcelimited = np.zeros(nu, np.int32)
  for i, a in enumerate(spec.actuators):
    jid = m.names["joint"].index(a.joint)
    if m.jnt_type[jid] not in (2, 3):
      raise NotImplementedError("actuators must drive hinge/slide joints")
    m.actuator_trnid[i] = jid
    m.actuator_gear[i] = a.gear
    m.actuator_gainprm[i, :3] = a.gainprm[:3]
    m.actuator_biasprm[i, :3] = a.biasprm[:3]
    cr = np.array(a.ctrlrange, np.float64)
    if a.inheritrange > 0:
      lo, hi = m.jnt_range[jid]
      mid, half = 0.5 * (lo + hi), 0.5 * (hi - lo) * a.inheritrange
      cr = np.array([mid - half, mid + half])
    m.actuator_ctrlrange[i] = cr
    if a.ctrllimited == "true" or (a.ctrllimited == "auto" and cr[0] < cr[1]):
      m.actuator_ctrllimited[i] = 1
    fr = np.array(a.forcerange, np.float64)
    m.actuator_forcerange[i] = fr
    if a.forcelimited == "true" or (a.forcelimited == "auto" and fr[0] < fr[1]):
      m.actuator_forcelimited[i] = 1

  # --- sensors ---
  _compile_sensors(m, spec)

  # --- set const (invweight0, meaninertia) ---
  _set_const(m)

  # --- collision pairs ---
  _compile_pairs(m, spec)

  # --- capacities ---
  m.nconmax = int(nconmax) if nconmax else max(32, 4 * len(m.pair_geom1))
  m.njmax = int(njmax) if njmax else max(64, 4 * m.nconmax + m.njnt + m.nv)

  # keyframe (first key), used by Entity defaults
  m.key_qpos = None
  m.key_ctrl = None
  return m


def _compile_sensors(m: Model, spec: Spec) -> None:
  ns = len(spec.sensors)
  m.nsensor = ns
  m.sensor_type = np.zeros(ns, np.int32)
  m.sensor_objtype = np.zeros(ns, np.int32)
  m.sensor_objid = np.zeros(ns, np.int32)
  m.sensor_reftype = np.zeros(ns, np.int32)
  m.sensor_refid = np.full(ns, -1, np.int32)
  m.sensor_adr = np.zeros(ns, np.int32)
  m.sensor_dim = np.zeros(ns, np.int32)
  m.sensor_intprm = np.zeros((ns, 3), np.int32)
  m.sensor_cutoff = np.zeros(ns)
  lookup = {
    "body": "body",
    "xbody": "body",
    "site": "site",
    "geom": "geom",
    "joint": "joint",
    "actuator": "actuator",
  }
  adr = 0
  for i, s in enumerate(spec.sensors):
    m.sensor_type[i] = SENSOR_TYPES[s.type]
    m.sensor_objtype[i] = OBJ_CODES[s.objtype]
    m.sensor_objid[i] = m.names[lookup[s.objtype]].index(s.objname) if s.objtype else -1
    if s.type in ("jointpos", "jointvel", "jointactuatorfrc") and m.jnt_type[m.sensor_objid[i]] not in (2, 3):
      raise NotImplementedError(f"{s.type} sensor '{s.name}' needs a hinge or slide joint (MuJoCo: ballquat / ballangvel)")
    if s.type in ("ballquat", "ballangvel") and m.jnt_type[m.sensor_objid[i]] != 1:
      raise ValueError(f"{s.type} sensor '{s.name}' needs a ball joint")
    if s.reftype and s.type in ("framelinacc", "frameangacc"):
      raise ValueError(f"{s.type} sensor '{s.name}': MuJoCo's acceleration frame sensors take no reference frame")
    if s.reftype:
      m.sensor_reftype[i] = OBJ_CODES[s.reftype]
      m.sensor_refid[i] = m.names[lookup[s.reftype]].index(s.refname)
    if s.type == "contact":
      bits, reduce, nslot = s.intprm
      width = sum(CONTACT_FIELD_DIMS[k] for k in range(7) if bits & (1 << k))
      if reduce == 3:
        nslot = 1
      dim = width * nslot
      m.sensor_intprm[i] = [bits, reduce, nslot]
    else:
      dim = SENSOR_DIMS[s.type]
    m.sensor_adr[i] = adr
    m.sensor_dim[i] = dim
    m.sensor_cutoff[i] = s.cutoff
    adr += dim
  m.nsensordata = adr
  # the step kernel keeps each sensor's metadata packed in four lane registers
  # (mjh_step.hip MJH_SENS_PRELOAD 2): the fields must fit their bit ranges
  for i in range(ns):
    ip = np.asarray(m.sensor_intprm).reshape(-1, 3)[i]
    ok = (0 <= int(m.sensor_objtype[i]) < 64 and 0 <= int(m.sensor_reftype[i]) < 64 and -1 <= int(m.sensor_objid[i]) < 65535
          and -1 <= int(m.sensor_refid[i]) < 65535 and 0 <= int(m.sensor_dim[i]) < 65536 and 0 <= int(m.sensor_type[i]) < 256
          and 0 <= int(ip[0]) < 128 and 0 <= int(ip[1]) < 8 and 0 <= int(ip[2]) < 65536)
    if not ok:
      raise NotImplementedError(f"sensor {i}: metadata outside the device's packed ranges")
  # sensors outside the benchmark tasks' set (a size, so it is part of the
  # specialised kernels' plans: an instance built for a model without them
  # carries none of their code)
  m.nsensor_ext = int(sum(1 for t in m.sensor_type if int(t) not in BASE_SENSOR_CODES))
  m.sensor_ext_mask = 0
  for t in m.sensor_type:
    if int(t) not in BASE_SENSOR_CODES:
      if int(t) not in SENSOR_EXT_GROUPS:
        raise NotImplementedError(f"sensor type {int(t)} has no device evaluation")
      m.sensor_ext_mask |= SENSOR_EXT_GROUPS[int(t)]


def _kinematics0(m: Model):
  """Float64 FK + com + cdof + CRB at qpos0 (for mj_setConst only)."""
  nb = m.nbody
  xpos = np.zeros((nb, 3))
  xquat = np.tile([1.0, 0, 0, 0], (nb, 1))
  xanchor = np.zeros((m.njnt, 3))
  xaxis = np.zeros((m.njnt, 3))
  q = m.qpos0
  for i in range(1, nb):
    p = m.body_parentid[i]
    if m.body_jntnum[i] == 1 and m.jnt_type[m.body_jntadr[i]] == 0:
      j = m.body_jntadr[i]
      qa = m.jnt_qposadr[j]
      xpos[i] = q[qa : qa + 3]
      xquat[i] = q[qa + 3 : qa + 7] / np.linalg.norm(q[qa + 3 : qa + 7])
      xanchor[j] = xpos[i]
      xaxis[j] = [0, 0, 1]
      continue
    xpos[i] = xpos[p] + rot.rotate(xquat[p], m.body_pos[i])
    xquat[i] = rot.quat_mul(xquat[p], m.body_quat[i])
    for j in range(m.body_jntadr[i], m.body_jntadr[i] + m.body_jntnum[i]):
      xaxis[j] = rot.rotate(xquat[i], m.jnt_axis[j])
      xanchor[j] = rot.rotate(xquat[i], m.jnt_pos[j]) + xpos[i]
      # qpos == qpos0 here: joint displacement is zero
    xquat[i] /= np.linalg.norm(xquat[i])
  xmat = np.array([rot.quat_to_mat(x) for x in xquat])
  xipos = np.array([xpos[i] + xmat[i] @ m.body_ipos[i] for i in range(nb)])
  ximat = np.array([xmat[i] @ rot.quat_to_mat(m.body_iquat[i]) for i in range(nb)])
  # subtree com
  msum = m.body_mass.copy()
  mp = m.body_mass[:, None] * xipos
  for i in range(nb - 1, 0, -1):
    msum[m.body_parentid[i]] += msum[i]
    mp[m.body_parentid[i]] += mp[i]
  com = np.where(msum[:, None] > MINVAL, mp / np.maximum(msum, MINVAL)[:, None], xipos)
  # cdof
  cdof = np.zeros((m.nv, 6))
  for j in range(m.njnt):
    b = m.jnt_bodyid[j]
    da = m.jnt_dofadr[j]
    off = com[m.body_rootid[b]] - xanchor[j]
    t = m.jnt_type[j]
    if t == 0:
      for k in range(3):
        cdof[da + k, 3 + k] = 1.0
      for k in range(3):
        ax = xmat[b][:, k]
        cdof[da + 3 + k, :3] = ax
        cdof[da + 3 + k, 3:] = np.cross(ax, off)
    elif t == 1:  # ball: rotations about the body's axes
      for k in range(3):
        ax = xmat[b][:, k]
        cdof[da + k, :3] = ax
        cdof[da + k, 3:] = np.cross(ax, off)
    elif t == 3:
      cdof[da, :3] = xaxis[j]
      cdof[da, 3:] = np.cross(xaxis[j], off)
    elif t == 2:
      cdof[da, 3:] = xaxis[j]
  # spatial inertia about subtree_com[root], 6x6 blocks [[I, h×],[−h×... ]]
  def spatial(i):
    R = ximat[i]
    d = xipos[i] - com[m.body_rootid[i]]
    mass = m.body_mass[i]
    I = R @ np.diag(m.body_inertia[i]) @ R.T + mass * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    h = mass * d
    hx = np.array([[0, -h[2], h[1]], [h[2], 0, -h[0]], [-h[1], h[0], 0]])
    S = np.zeros((6, 6))
    S[:3, :3] = I
    S[:3, 3:] = hx
    S[3:, :3] = -hx
    S[3:, 3:] = mass * np.eye(3)
    return S

  crb = np.array([spatial(i) if i > 0 else np.zeros((6, 6)) for i in range(nb)])
  for i in range(nb - 1, 0, -1):
    if m.body_parentid[i] > 0:
      crb[m.body_parentid[i]] += crb[i]
  M = np.zeros((m.nv, m.nv))
  for i in range(m.nv):
    buf = crb[m.dof_bodyid[i]] @ cdof[i]
    j = i
    while j >= 0:
      M[i, j] = M[j, i] = cdof[j] @ buf
      j = m.dof_parentid[j]
    M[i, i] += m.dof_armature[i]
  return xipos, com, cdof, M


def _set_const(m: Model) -> None:
  nv = m.nv
  m.dof_invweight0 = np.zeros(nv)
  m.body_invweight0 = np.zeros((m.nbody, 2))
  if nv == 0:
    m.meaninertia = 1.0
    return
  xipos, com, cdof, M = _kinematics0(m)
  Minv = np.linalg.inv(M)
  for j in range(m.njnt):
    da = m.jnt_dofadr[j]
    if m.jnt_type[j] == 0:
      m.dof_invweight0[da : da + 3] = np.mean(np.diag(Minv)[da : da + 3])
      m.dof_invweight0[da + 3 : da + 6] = np.mean(np.diag(Minv)[da + 3 : da + 6])
    elif m.jnt_type[j] == 1:  # ball: the mean over its three dofs (mj_setConst)
      m.dof_invweight0[da : da + 3] = np.mean(np.diag(Minv)[da : da + 3])
    else:
      m.dof_invweight0[da] = Minv[da, da]
  for b in range(1, m.nbody):
    if m.body_weldid[b] == 0:
      continue
    jacp = np.zeros((3, nv))
    jacr = np.zeros((3, nv))
    k = b
    while k > 0:
      for d in range(m.body_dofadr[k], m.body_dofadr[k] + m.body_dofnum[k]):
        jacr[:, d] = cdof[d, :3]
        jacp[:, d] = cdof[d, 3:] + np.cross(cdof[d, :3], xipos[b] - com[m.body_rootid[b]])
      k = m.body_parentid[k]
    Ap = jacp @ Minv @ jacp.T
    Ar = jacr @ Minv @ jacr.T
    m.body_invweight0[b] = [np.trace(Ap) / 3.0, np.trace(Ar) / 3.0]
  m.meaninertia = float(np.trace(M) / nv)


def _compile_pairs(m: Model, spec: Spec) -> None:
  bid = {n: i for i, n in enumerate(m.names["body"])}
  excl = set()
  m.excludes = [tuple(e) for e in spec.excludes]
  for a, b in spec.excludes:
    i, j = bid[a], bid[b]
    excl.add((min(i, j), max(i, j)))
  pairs = []
  colgeoms = set()
  for g1 in range(m.ngeom):
    for g2 in range(g1 + 1, m.ngeom):
      ct1, ca1 = m.geom_contype[g1], m.geom_conaffinity[g1]
      ct2, ca2 = m.geom_contype[g2], m.geom_conaffinity[g2]
      if not ((ct1 & ca2) or (ct2 & ca1)):
        continue
      b1, b2 = m.geom_bodyid[g1], m.geom_bodyid[g2]
      w1, w2 = m.body_weldid[b1], m.body_weldid[b2]
      if w1 == w2:
        continue
      pw1 = m.body_weldid[m.body_parentid[w1]]
      pw2 = m.body_weldid[m.body_parentid[w2]]
      if w1 != 0 and w2 != 0 and (w1 == pw2 or w2 == pw1):
        continue
      if (min(b1, b2), max(b1, b2)) in excl:
        continue
      t1, t2 = m.geom_type[g1], m.geom_type[g2]
      if t1 == 0 and t2 == 0:
        continue
      if t1 > t2:
        g1_, g2_ = g2, g1
      else:
        g1_, g2_ = g1, g2
      pairs.append((g1_, g2_))
      colgeoms.add(g1)
      colgeoms.add(g2)
  # geom-type pairs with a narrowphase in the HIP step (and the oracle):
  # plane-{sphere,capsule,ellipsoid,cylinder,box}, sphere-{sphere,capsule,cylinder,box},
  # capsule-{capsule,box}, box-box.
  # Other pairs stay in the table (the kernels return no contact for them)
  # and are reported here instead of being silently ignored.
  unsupported = sorted({(int(m.geom_type[a]), int(m.geom_type[b])) for a, b in pairs
                        if (int(m.geom_type[a]), int(m.geom_type[b])) not in SUPPORTED_PAIRS})
  m.unsupported_pair_types = unsupported
  if unsupported:
    inv = {v: k for k, v in GEOM_TYPES.items()}
    warnings.warn("collision pairs without a narrowphase on the HIP path (no contacts are generated): "
                  + ", ".join(f"{inv[a]}-{inv[b]}" for a, b in unsupported), UserWarning, stacklevel=3)
  m.npair = len(pairs)
  m.nboxpair = sum(1 for a, b in pairs if (int(m.geom_type[a]), int(m.geom_type[b])) in BOX_PAIRS)
  m.pair_geom1 = np.array([p[0] for p in pairs] or [0], np.int32)
  m.pair_geom2 = np.array([p[1] for p in pairs] or [0], np.int32)
  cg = sorted(colgeoms)
  m.ncolgeom = max(1, len(cg))
  m.colgeom_id = np.array(cg or [0], np.int32)
  slot = np.full(m.ngeom, -1, np.int32)
  for k, g in enumerate(cg):
    slot[g] = k
  m.geom_colslot = slot
