"""Ball joints (MuJoCo mjJNT_BALL: a normalised quaternion in qpos, three
rotational dofs about the body's axes, mju_quatIntegrate, the rotation-angle
cone limit of mj_instantiateLimit, the mju_subQuat spring) in the oracle
(oracle.c kinematics / com_pos / com_vel / passive / make_constraint /
integration) against closed forms that do not come from either restatement:

* a ball joint released in a plane moves exactly as a hinge does;
* a conical pendulum (isotropic bob) precesses at omega^2 = g / (L cos theta)
  with a constant tilt;
* a torsional ball spring on an isotropic body oscillates at sqrt(k / I) at
  any amplitude (the torque is -k times the rotation vector);
* a ball limit row has the Jacobian -(unit rotation axis) and holds an
  inverted pendulum at the cone angle.

The HIP step is checked against the oracle in
tests/test_gpu_parity.py::test_ball_joint_parity."""

import numpy as np
import pytest

from mjlab_amd.spec.compiler import compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from mjlab_amd.utils import rot
from oracle.oracle import Oracle


def _model(xml):
  return compile_spec(read_mjcf_string(xml), 8, 64)


def _roll(m, st, n):
  orc = Oracle(m)
  out = None
  for _ in range(n):
    out = orc.run(1, st, integrate=True)
    st = {k: out[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
  return st, out


PLANAR = """<mujoco><option timestep="0.001" gravity="0 0 -9.81"/><worldbody>
<body name="rod" pos="0 0 1"><joint name="j" type="{jtype}" axis="0 1 0"/>
<geom type="capsule" fromto="0 0 0 0.3 0 -0.4" size="0.03" mass="1.3" contype="0" conaffinity="0"/></body>
</worldbody></mujoco>"""


def test_ball_in_a_plane_moves_as_a_hinge():
  """Released from a tilt about y with zero velocity, gravity keeps the motion
  in the x-z plane: the ball quaternion stays (cos(q/2), 0, sin(q/2), 0) of the
  hinge angle q at every step (300 steps, float64, 1e-9)."""
  mb, mh = _model(PLANAR.format(jtype="ball")), _model(PLANAR.format(jtype="hinge"))
  assert mb.nq == 4 and mb.nv == 3 and mh.nq == 1
  th0 = 0.4
  sb = {"qpos": np.array([[np.cos(th0 / 2), 0, np.sin(th0 / 2), 0]])}
  sh = {"qpos": np.array([[th0]])}
  ob, oh = Oracle(mb), Oracle(mh)
  for _ in range(300):
    rb, rh = ob.run(1, sb, integrate=True), oh.run(1, sh, integrate=True)
    sb = {k: rb[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    sh = {k: rh[k] for k in ("qpos", "qvel", "qacc_warmstart", "time")}
    q = rh["qpos"][0, 0]
    np.testing.assert_allclose(rb["qpos"][0], [np.cos(q / 2), 0, np.sin(q / 2), 0], atol=1e-9)
    np.testing.assert_allclose(rb["qvel"][0], [0, rh["qvel"][0, 0], 0], atol=1e-9)
  assert abs(q - th0) > 0.1  # it swung


def test_conical_pendulum_precession():
  """A 1 kg sphere (isotropic inertia) at L = 0.5 below a ball joint, tilted
  by 0.6 rad and spun about the vertical at omega = sqrt(g / (L cos theta)):
  the tilt stays at 0.6 rad and the bob's azimuth advances at omega (1 s of
  0.2 ms steps; the isotropic inertia adds no gyroscopic torque)."""
  L, th, g = 0.5, 0.6, 9.81
  xml = f"""<mujoco><option timestep="0.0002" gravity="0 0 {-g}" integrator="Euler"/><worldbody>
  <body name="bob" pos="0 0 2"><joint type="ball"/>
  <geom type="sphere" pos="0 0 {-L}" size="0.05" mass="1" contype="0" conaffinity="0"/></body>
  </worldbody></mujoco>"""
  m = _model(xml)
  om = np.sqrt(g / (L * np.cos(th)))
  q = rot.axis_angle_to_quat(np.array([1.0, 0, 0]), th)  # tilt about x: the bob swings towards +y
  w_local = rot.quat_to_mat(q).T @ np.array([0, 0, om])  # ball qvel: the body-frame angular velocity
  st = {"qpos": q[None], "qvel": w_local[None]}
  T = 1.0
  st, _ = _roll(m, st, int(round(T / m.timestep)))
  R = rot.quat_to_mat(st["qpos"][0] / np.linalg.norm(st["qpos"][0]))
  bob = R @ np.array([0, 0, -L])
  tilt = np.arccos(-bob[2] / L)
  assert tilt == pytest.approx(th, abs=2e-3)
  az0 = np.arctan2(*(rot.quat_to_mat(q) @ np.array([0, 0, -L]))[[1, 0]])
  az = np.arctan2(bob[1], bob[0])
  assert np.mod(az - az0, 2 * np.pi) == pytest.approx(np.mod(om * T, 2 * np.pi), abs=5e-3)


def test_ball_spring_period_at_large_amplitude():
  """A sphere centred on its ball joint (I = 2/5 m r^2), no gravity, spring
  stiffness k, released at 1.2 rad about an oblique axis: the rotation angle
  follows 1.2 cos(sqrt(k / I) t) (half a period of 0.1 ms steps)."""
  k, mass, r = 0.8, 2.0, 0.1
  I = 0.4 * mass * r * r
  xml = f"""<mujoco><option timestep="0.0001" gravity="0 0 0" integrator="Euler"/><worldbody>
  <body name="s" pos="0 0 1"><joint type="ball" stiffness="{k}"/>
  <geom type="sphere" size="{r}" mass="{mass}" contype="0" conaffinity="0"/></body>
  </worldbody></mujoco>"""
  m = _model(xml)
  ax = np.array([1.0, 2.0, -0.5])
  ax /= np.linalg.norm(ax)
  a0 = 1.2
  st = {"qpos": rot.axis_angle_to_quat(ax, a0)[None]}
  w = np.sqrt(k / I)
  n = int(round(np.pi / w / m.timestep))
  st, _ = _roll(m, st, n)
  q = st["qpos"][0] / np.linalg.norm(st["qpos"][0])
  ang = 2 * np.arctan2(np.linalg.norm(q[1:]), q[0])
  axis = q[1:] / np.linalg.norm(q[1:])
  # half a period: the angle is back to a0 about the opposite axis
  assert ang == pytest.approx(a0 * abs(np.cos(w * n * m.timestep)), abs=2e-3)
  np.testing.assert_allclose(axis, -ax, atol=1e-6)


INVERTED = """<mujoco><compiler angle="radian"/><option timestep="0.002" gravity="0 0 -9.81"/><worldbody>
<body name="stick" pos="0 0 1"><joint name="j" type="ball" range="0 0.5" limited="true"/>
<geom type="sphere" pos="0 0 0.6" size="0.05" mass="1" contype="0" conaffinity="0"/></body>
</worldbody></mujoco>"""


def test_ball_limit_row_jacobian_and_rest_on_the_cone():
  """An inverted 1 kg bob at 0.6 m above a ball joint limited to 0.5 rad:
  past the cone one limit row with J = -(unit rotation axis) on the three
  dofs; released at 0.1 rad it falls onto the cone and rests there, the row's
  generalised force holding the gravity torque m g L sin(angle)."""
  m = _model(INVERTED)
  assert m.jnt_limited[0] == 1 and m.jnt_range[0, 1] == pytest.approx(0.5)
  ax = np.array([1.0, 1.0, 0.0]) / np.sqrt(2)
  st = {"qpos": rot.axis_angle_to_quat(ax, 0.52)[None]}
  out = Oracle(m).run(1, st, integrate=False, debug=True)
  assert out["nefc"][0, 0] == 1
  J = out["efc_J"][0].reshape(m.njmax, m.nv)[0]
  np.testing.assert_allclose(J, -ax, atol=1e-12)
  assert out["efc_pos"][0, 0] == pytest.approx(0.5 - 0.52, abs=1e-12)
  # released inside the cone: it falls onto the limit and stays
  st = {"qpos": rot.axis_angle_to_quat(ax, 0.1)[None]}
  st, out = _roll(m, st, 1500)
  q = st["qpos"][0] / np.linalg.norm(st["qpos"][0])
  ang = 2 * np.arctan2(np.linalg.norm(q[1:]), q[0])
  assert 0.5 < ang < 0.53
  assert np.abs(st["qvel"][0]).max() < 1e-4
  tq = 9.81 * 0.6 * np.sin(ang)
  assert np.linalg.norm(out["qfrc_constraint"][0]) == pytest.approx(tq, rel=1e-3)


def test_ball_joint_model_round_trip_and_entity_indexing():
  """The NaN guard's MJCF (model_to_mjcf) keeps ball joints (type, range,
  identity qpos0, invweight0), and an entity's joint addresses cover a ball
  joint's 4 qpos / 3 dofs (reference entity.py:631-633)."""
  from mjlab_amd.spec.mjcf import model_to_mjcf

  m = _model(INVERTED)
  m2 = _model(model_to_mjcf(m))
  for k in ("jnt_type", "jnt_qposadr", "jnt_dofadr", "jnt_range", "jnt_limited", "qpos0", "dof_invweight0"):
    np.testing.assert_allclose(np.asarray(getattr(m, k)), np.asarray(getattr(m2, k)), rtol=1e-6, atol=1e-9, err_msg=k)
  np.testing.assert_allclose(m.qpos0, [1, 0, 0, 0])

  from mjlab_amd.entity import Entity, EntityCfg
  from mjlab_amd.spec.mjcf import read_mjcf_string

  xml = """<mujoco><worldbody><body name="root"><freejoint/><geom type="box" size="0.1 0.1 0.1" mass="1"/>
  <body name="a" pos="0.2 0 0"><joint name="ball" type="ball"/><geom type="sphere" size="0.05" mass="0.2"/>
  <body name="b" pos="0.1 0 0"><joint name="hinge" axis="0 0 1"/><geom type="sphere" size="0.04" mass="0.1"/>
  </body></body></body></worldbody></mujoco>"""
  ent = Entity(EntityCfg(spec_fn=lambda: read_mjcf_string(xml)))
  model = ent.compile()
  ix = ent._compute_indexing(model, "cpu")
  assert ix.joint_q_adr.tolist() == [7, 8, 9, 10, 11] and ix.joint_v_adr.tolist() == [6, 7, 8, 9]
