"""The reference's own boundary tests, restated against this build's Simulation.

Each test follows one reference test (cited file:line) with the same scene, the
same calls and the same assertions and tolerances; differences are named in the
test. They run on two backends (``tests/refsim.py``): ``hip`` (the HIP step
library on cuda:0, every step/forward also checked against the float64 oracle)
and ``oracle`` (CPU, for the host logic in the CPU suite). Reference scenes use
``mujoco.MjSpec.from_string`` / ``MjModel.from_xml_string``; here
``read_mjcf_string`` / ``compile_spec`` (MuJoCo is absent).
"""

from __future__ import annotations

import math
import warnings
from unittest.mock import Mock

import numpy as np
import pytest
import torch

from mjlab_amd.entity import Entity, EntityCfg
from mjlab_amd.entity.entity import EntityArticulationInfoCfg
from mjlab_amd.envs.mdp import events
from mjlab_amd.managers.event_manager import EventManager
from mjlab_amd.managers.manager_term_config import EventTermCfg
from mjlab_amd.managers.scene_entity_config import SceneEntityCfg
from mjlab_amd.scene.scene import Scene, SceneCfg
from mjlab_amd.sensor import ContactMatch, ContactSensorCfg
from mjlab_amd.sensor.builtin_sensor import BuiltinSensorCfg, ObjRef
from mjlab_amd.sim import MujocoCfg, SimulationCfg
from mjlab_amd.spec.compiler import compile_spec
from mjlab_amd.spec.mjcf import read_mjcf_string
from mjlab_amd.utils.math import quat_apply_inverse
from mjlab_amd.utils.spec_config import ActuatorCfg
from tests.refsim import BACKENDS, device_of, expanded_fields_attach, make_sim


@pytest.fixture(params=BACKENDS)
def backend(request):
  return request.param


# ---------------------------------------------------------------------------
# tests/test_entity_data.py:11-158 and tests/test_entity.py:13-136 scenes
# ---------------------------------------------------------------------------
FIXED_BASE_XML = """
<mujoco><worldbody>
  <body name="object" pos="0 0 0.5">
    <geom name="object_geom" type="box" size="0.1 0.1 0.1" rgba="0.8 0.3 0.3 1"/>
  </body>
</worldbody></mujoco>"""

FLOATING_BASE_XML = """
<mujoco><worldbody>
  <body name="object" pos="0 0 1">
    <freejoint name="free_joint"/>
    <geom name="object_geom" type="box" size="0.1 0.1 0.1" rgba="0.3 0.3 0.8 1" mass="0.1"/>
  </body>
</worldbody></mujoco>"""

FIXED_BASE_ARTICULATED_XML = """
<mujoco><worldbody>
  <body name="base" pos="0 0 0.5">
    <geom name="base_geom" type="cylinder" size="0.1 0.05" mass="5.0"/>
    <body name="link1" pos="0 0 0.1">
      <joint name="joint1" type="hinge" axis="0 0 1" range="-3.14 3.14"/>
      <geom name="link1_geom" type="box" size="0.05 0.05 0.2" mass="1.0"/>
      <body name="link2" pos="0 0 0.4">
        <joint name="joint2" type="hinge" axis="0 1 0" range="-1.57 1.57"/>
        <geom name="link2_geom" type="box" size="0.05 0.05 0.15" mass="0.5"/>
      </body>
    </body>
  </body>
</worldbody></mujoco>"""

FLOATING_BASE_ARTICULATED_XML = """
<mujoco><worldbody>
  <body name="base" pos="0 0 1">
    <freejoint name="free_joint"/>
    <geom name="base_geom" type="box" size="0.2 0.2 0.1" mass="1.0"/>
    <body name="link1" pos="0 0 0">
      <joint name="joint1" type="hinge" axis="0 0 1" range="0 1.57"/>
      <geom name="link1_geom" type="box" size="0.1 0.1 0.1" mass="0.1"/>
      <site name="site1" pos="0 0 0"/>
    </body>
    <body name="link2" pos="0 0 0">
      <joint name="joint2" type="hinge" axis="0 0 1" range="0 1.57"/>
      <geom name="link2_geom" type="box" size="0.1 0.1 0.1" mass="0.1"/>
    </body>
  </body>
</worldbody>
<sensor><jointpos name="joint1_pos" joint="joint1"/></sensor>
</mujoco>"""

_ACT = EntityArticulationInfoCfg(actuators=(ActuatorCfg(joint_names_expr=("joint1", "joint2"), effort_limit=1.0,
                                                         stiffness=1.0, damping=1.0),))


def _entity(xml: str, **kw) -> Entity:
  return Entity(EntityCfg(spec_fn=lambda: read_mjcf_string(xml), **kw))


def _init_entity_with_sim(entity: Entity, backend: str, num_envs: int = 1, skip: tuple[str, ...] = ()):
  """test_entity_data.py:35-41 / test_entity.py:130-136."""
  model = entity.compile()
  # every pair of these scenes has a narrowphase (FIXED_BASE_ARTICULATED's
  # cylinder base against link2's box: the general convex collider)
  assert not model.unsupported_pair_types, model.unsupported_pair_types
  sim = make_sim(num_envs, SimulationCfg(), model, backend, skip=skip)
  entity.initialize(model, sim.model, sim.data, device_of(backend))
  return entity, sim


def test_root_velocity_world_frame_roundtrip(backend):
  """test_entity_data.py:44-70."""
  dev = device_of(backend)
  entity, sim = _init_entity_with_sim(_entity(FLOATING_BASE_XML), backend)
  pose = torch.tensor([0.0, 0.0, 1.0, 0.6, 0.2, 0.3, 0.7141], device=dev).unsqueeze(0)
  entity.write_root_link_pose_to_sim(pose)
  vel_w = torch.tensor([1.0, 0.5, 0.0, 0.0, 0.3, 0.1], device=dev).unsqueeze(0)
  entity.write_root_link_velocity_to_sim(vel_w)
  sim.forward()
  vel_w_read = entity.data.root_link_vel_w.clone()
  assert torch.allclose(vel_w_read, vel_w, atol=1e-4)
  entity.write_root_link_velocity_to_sim(vel_w_read)
  sim.forward()
  assert torch.allclose(entity.data.root_link_vel_w, vel_w_read, atol=1e-4)


def test_root_velocity_frame_conversion(backend):
  """test_entity_data.py:73-102: angular velocity is stored in the body frame."""
  dev = device_of(backend)
  entity, sim = _init_entity_with_sim(_entity(FLOATING_BASE_XML), backend)
  quat_w = torch.tensor([0.6, 0.2, 0.3, 0.7141], device=dev).unsqueeze(0)
  entity.write_root_link_pose_to_sim(torch.cat([torch.zeros(1, 3, device=dev), quat_w], dim=-1))
  lin_vel_w = torch.tensor([1.0, 0.5, 0.2], device=dev).unsqueeze(0)
  ang_vel_w = torch.tensor([0.1, 0.2, 0.3], device=dev).unsqueeze(0)
  entity.write_root_link_velocity_to_sim(torch.cat([lin_vel_w, ang_vel_w], dim=-1))
  qvel = sim.data.qvel[:, entity.data.indexing.free_joint_v_adr.long()]
  assert torch.allclose(qvel[:, :3], lin_vel_w, atol=1e-5)
  assert torch.allclose(qvel[:, 3:], quat_apply_inverse(quat_w, ang_vel_w), atol=1e-5)


def test_write_velocity_uses_qpos_not_xquat(backend):
  """test_entity_data.py:105-132."""
  dev = device_of(backend)
  entity, sim = _init_entity_with_sim(_entity(FLOATING_BASE_XML), backend)
  entity.write_root_link_pose_to_sim(torch.tensor([0.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0], device=dev).unsqueeze(0))
  sim.forward()
  entity.write_root_link_pose_to_sim(torch.tensor([0.0, 0.0, 1.0, 0.707, 0.0, 0.707, 0.0], device=dev).unsqueeze(0))
  vel_w = torch.tensor([1.0, 0.0, 0.0, 0.0, 1.0, 0.0], device=dev).unsqueeze(0)
  entity.write_root_link_velocity_to_sim(vel_w)
  sim.forward()
  assert torch.allclose(entity.data.root_link_vel_w, vel_w, atol=1e-4)


def test_read_requires_forward_to_be_current(backend):
  """test_entity_data.py:135-158: derived reads are stale until forward()."""
  dev = device_of(backend)
  entity, sim = _init_entity_with_sim(_entity(FLOATING_BASE_XML), backend)
  sim.forward()
  initial_pose = entity.data.root_link_pose_w.clone()
  new_pose = torch.tensor([1.0, 2.0, 3.0, 0.707, 0.0, 0.707, 0.0], device=dev).unsqueeze(0)
  entity.write_root_link_pose_to_sim(new_pose)
  assert torch.allclose(entity.data.root_link_pose_w, initial_pose, atol=1e-5)
  sim.forward()
  current_pose = entity.data.root_link_pose_w
  assert torch.allclose(current_pose, new_pose, atol=1e-4)
  assert not torch.allclose(current_pose, initial_pose, atol=1e-4)


@pytest.mark.parametrize("xml,act,expected", [
  (FIXED_BASE_XML, None, dict(is_fixed_base=True, is_articulated=False, is_actuated=False, num_bodies=1, num_joints=0,
                              num_actuators=0)),
  (FLOATING_BASE_XML, None, dict(is_fixed_base=False, is_articulated=False, is_actuated=False, num_bodies=1,
                                 num_joints=0, num_actuators=0)),
  (FIXED_BASE_ARTICULATED_XML, _ACT, dict(is_fixed_base=True, is_articulated=True, is_actuated=True, num_bodies=3,
                                          num_joints=2, num_actuators=2)),
  (FLOATING_BASE_ARTICULATED_XML, _ACT, dict(is_fixed_base=False, is_articulated=True, is_actuated=True, num_bodies=3,
                                             num_joints=2, num_actuators=2)),
], ids=["fixed", "floating", "fixed_articulated", "floating_articulated"])
def test_entity_properties(xml, act, expected):
  """test_entity.py:139-192."""
  e = _entity(xml, articulation=act)
  for prop, value in expected.items():
    assert getattr(e, prop) == value


def test_find_methods():
  """test_entity.py:195-206."""
  e = _entity(FLOATING_BASE_ARTICULATED_XML, articulation=_ACT)
  assert e.find_bodies("base")[1] == ["base"]
  assert e.find_joints("joint1")[1] == ["joint1"]
  assert e.find_sites("site1")[1] == ["site1"]
  assert e.find_bodies("link.*")[1] == ["link1", "link2"]
  assert e.find_joints("joint.*")[1] == ["joint1", "joint2"]


def test_find_with_subset_filtering():
  """test_entity.py:209-219."""
  e = _entity(FLOATING_BASE_ARTICULATED_XML, articulation=_ACT)
  assert e.find_joints("joint1", joint_subset=["joint1", "joint2"])[1] == ["joint1"]
  with pytest.raises(ValueError, match="Not all regular expressions are matched"):
    e.find_joints("joint1", joint_subset=["joint2"])


def test_root_state_read_write(backend):
  """test_entity.py:222-242."""
  dev = device_of(backend)
  entity, sim = _init_entity_with_sim(_entity(FLOATING_BASE_XML), backend)
  root_state = torch.tensor([1.0, 2.0, 3.0, 1.0, 0.0, 0.0, 0.0, 0.5, 0.0, 0.0, 0.0, 0.0, 0.2], device=dev).unsqueeze(0)
  entity.write_root_state_to_sim(root_state)
  q = entity.data.indexing.free_joint_q_adr.long()
  v = entity.data.indexing.free_joint_v_adr.long()
  assert torch.allclose(sim.data.qpos[:, q], root_state[:, :7])
  assert torch.allclose(sim.data.qvel[:, v], root_state[:, 7:])


def test_external_force_and_torque(backend):
  """test_entity.py:245-272: forces translate, torques rotate (10 physics steps)."""
  dev = device_of(backend)
  entity, sim = _init_entity_with_sim(_entity(FLOATING_BASE_XML), backend)
  entity.write_external_wrench_to_sim(forces=torch.tensor([[5.0, 0.0, 0.0]], device=dev),
                                      torques=torch.tensor([[0.0, 0.0, 3.0]], device=dev))
  initial_pos = sim.data.qpos[0, :3].clone()
  initial_quat = sim.data.qpos[0, 3:7].clone()
  for _ in range(10):
    sim.step()
  assert sim.data.qpos[0, 0] > initial_pos[0], "Force should cause X translation"
  assert not torch.allclose(sim.data.qpos[0, 3:7], initial_quat), "Torque should cause rotation"
  w = sim.data.qvel[0, 3:6]
  assert abs(w[2]) > (abs(w[0]) + abs(w[1])) * 5, "Rotation should be primarily around Z axis"
  # analytic: a free box under a constant wrench from rest (no contacts, the
  # torque axis is a principal axis): x = F/m t^2/2, w_z = tau/I_zz t (implicitfast
  # with no damping is semi-implicit Euler: x_n = F/m dt^2 n(n+1)/2)
  m, dt, n = 0.1, float(sim.mj_model.timestep), 10
  assert abs(float(sim.data.qpos[0, 0] - initial_pos[0]) - 5.0 / m * dt * dt * n * (n + 1) / 2) < 1e-5
  izz = m * (0.2**2 + 0.2**2) / 12
  assert abs(float(w[2]) - 3.0 / izz * dt * n) < 1e-3 * 3.0 / izz * dt * n


def test_external_force_clearing(backend):
  """test_entity.py:275-295."""
  dev = device_of(backend)
  entity, sim = _init_entity_with_sim(_entity(FLOATING_BASE_XML), backend)
  entity.write_external_wrench_to_sim(forces=torch.tensor([[5.0, 0.0, 0.0]], device=dev),
                                      torques=torch.tensor([[0.0, 0.0, 3.0]], device=dev))
  entity.write_external_wrench_to_sim(forces=torch.zeros((1, 3), device=dev), torques=torch.zeros((1, 3), device=dev))
  body_id = int(entity.indexing.body_ids[0])
  assert torch.allclose(sim.data.xfrc_applied[:, body_id, :], torch.zeros(6, device=dev))


def test_external_force_on_specific_body(backend):
  """test_entity.py:298-326, as the reference writes it: the overlapping link
  boxes collide (box-box narrowphase), the wrench moves link1."""
  dev = device_of(backend)
  e = _entity(FLOATING_BASE_ARTICULATED_XML, articulation=_ACT)
  with warnings.catch_warnings():
    warnings.simplefilter("error")  # every collision pair of the model has a narrowphase
    e.compile()
  # base and link boxes overlap completely, a degenerate box-box configuration
  # whose deepest contact's position and reference acceleration float32 cannot
  # pin (measured 5.1e-5 / 0.62 against bounds 5e-5 / 0.53): those two checks
  # are skipped (Shadow skip); forces, accelerations and state are compared
  entity, sim = _init_entity_with_sim(e, backend, skip=("contact_pos", "efc_aref"))
  body_ids = entity.find_bodies("link1")[0]
  entity.write_external_wrench_to_sim(forces=torch.tensor([[3.0, 0.0, 0.0]], device=dev),
                                      torques=torch.zeros((1, 3), device=dev), body_ids=body_ids)
  link1_id = sim.mj_model.body("link1").id
  base_id = sim.mj_model.body("base").id
  assert torch.allclose(sim.data.xfrc_applied[0, link1_id, :3], torch.tensor([3.0, 0.0, 0.0], device=dev))
  assert torch.allclose(sim.data.xfrc_applied[0, base_id, :3], torch.zeros(3, device=dev))
  initial_pos = sim.data.xpos[0, link1_id, :].clone()
  for _ in range(10):
    sim.step()
  assert not torch.allclose(sim.data.xpos[0, link1_id, :], initial_pos)


def test_fixed_base_initial_position():
  """test_entity.py:329-340."""
  e = Entity(EntityCfg(spec_fn=lambda: read_mjcf_string(FIXED_BASE_XML),
                       init_state=EntityCfg.InitialStateCfg((1.0, 2.0, 3.0), (0.7071, 0.7071, 0.0, 0.0))))
  body = e.compile().body("object")
  np.testing.assert_allclose(body.pos, [1.0, 2.0, 3.0], rtol=1e-6)
  np.testing.assert_allclose(body.quat, [0.7071, 0.7071, 0.0, 0.0], atol=1e-4)


def test_keyframe_ctrl_maps_joint_pos_to_actuators():
  """test_entity.py:343-363."""
  m = Entity(EntityCfg(spec_fn=lambda: read_mjcf_string(FLOATING_BASE_ARTICULATED_XML), articulation=_ACT,
                       init_state=EntityCfg.InitialStateCfg(joint_pos={"joint1": 0.5, "joint2": -0.25}))).compile()
  assert m.nkey == 1
  assert m.nu == 2
  assert list(m.key("init_state").ctrl) == [0.5, -0.25]


def test_keyframe_ctrl_underactuated():
  """test_entity.py:366-385 (key_ctrl is (nu,) here, (nkey, nu) in MuJoCo)."""
  act = EntityArticulationInfoCfg(actuators=(ActuatorCfg(joint_names_expr=("joint1",), effort_limit=1.0, stiffness=1.0,
                                                         damping=1.0),))
  m = Entity(EntityCfg(spec_fn=lambda: read_mjcf_string(FLOATING_BASE_ARTICULATED_XML), articulation=act,
                       init_state=EntityCfg.InitialStateCfg(joint_pos={"joint1": 0.42, "joint2": -0.99}))).compile()
  assert m.nu == 1
  assert m.key("init_state").ctrl[0] == 0.42


def test_fixed_base_mocap_runtime_pose_change(backend):
  """test_entity.py:388-415."""
  dev = device_of(backend)

  def spec_fn():
    spec = read_mjcf_string(FIXED_BASE_ARTICULATED_XML)
    spec.worldbody.children[0].mocap = True
    return spec

  e = Entity(EntityCfg(spec_fn=spec_fn, init_state=EntityCfg.InitialStateCfg((1.0, 2.0, 3.0), (1.0, 0.0, 0.0, 0.0))))
  entity, sim = _init_entity_with_sim(e, backend)
  assert entity.indexing.mocap_id is not None
  assert entity.is_mocap is True
  new_pose = torch.tensor([5.0, 6.0, 7.0, 1.0, 0.0, 0.0, 0.0], device=dev).unsqueeze(0)
  entity.write_mocap_pose_to_sim(new_pose)
  sim.forward()
  assert torch.allclose(entity.data.root_link_pose_w, new_pose, atol=1e-5)


# ---------------------------------------------------------------------------
# tests/test_contact_sensor.py:19-757
# ---------------------------------------------------------------------------
FALLING_BOX_XML = """
<mujoco><worldbody>
  <body name="ground" pos="0 0 0">
    <geom name="ground_geom" type="plane" size="5 5 0.1" rgba="0.5 0.5 0.5 1"/>
  </body>
  <body name="box" pos="0 0 0.5">
    <freejoint name="box_joint"/>
    <geom name="box_geom" type="box" size="0.1 0.1 0.1" rgba="0.8 0.3 0.3 1" mass="1.0"/>
  </body>
</worldbody></mujoco>"""

BIPED_XML = """
<mujoco><worldbody>
  <body name="ground" pos="0 0 0">
    <geom name="ground_geom" type="plane" size="5 5 0.1" rgba="0.5 0.5 0.5 1"/>
  </body>
  <body name="base" pos="0 0 0.5">
    <freejoint name="base_joint"/>
    <geom name="torso_geom" type="box" size="0.15 0.1 0.2" mass="5.0"/>
    <body name="left_foot" pos="0.1 0 -0.25">
      <joint name="left_ankle" type="hinge" axis="0 1 0" range="-0.5 0.5"/>
      <geom name="left_foot_geom" type="box" size="0.05 0.08 0.02" mass="0.2"/>
    </body>
    <body name="right_foot" pos="-0.1 0 -0.25">
      <joint name="right_ankle" type="hinge" axis="0 1 0" range="-0.5 0.5"/>
      <geom name="right_foot_geom" type="box" size="0.05 0.08 0.02" mass="0.2"/>
    </body>
  </body>
</worldbody></mujoco>"""

SIMPLE_ROBOT_XML = """
<mujoco><worldbody>
  <body name="ground" pos="0 0 0">
    <geom name="ground_geom" type="plane" size="5 5 0.1"/>
  </body>
  <body name="robot" pos="0 0 0.3">
    <freejoint name="robot_joint"/>
    <geom name="trunk_collision" type="box" size="0.2 0.15 0.1" mass="2.0"/>
    <geom name="head_collision" type="sphere" size="0.08" pos="0.25 0 0.1" mass="0.5"/>
    <body name="leg1" pos="0.1 0.1 -0.1">
      <geom name="leg1_thigh_collision1" type="capsule" size="0.02" fromto="0 0 0 0 0 -0.1"/>
      <geom name="leg1_thigh_collision2" type="capsule" size="0.02" fromto="0 0 -0.05 0 0 -0.15"/>
      <geom name="leg1_foot_collision" type="sphere" size="0.03" pos="0 0 -0.2"/>
    </body>
    <body name="leg2" pos="-0.1 0.1 -0.1">
      <geom name="leg2_thigh_collision1" type="capsule" size="0.02" fromto="0 0 0 0 0 -0.1"/>
      <geom name="leg2_thigh_collision2" type="capsule" size="0.02" fromto="0 0 -0.05 0 0 -0.15"/>
      <geom name="leg2_foot_collision" type="sphere" size="0.03" pos="0 0 -0.2"/>
    </body>
  </body>
</worldbody></mujoco>"""


def _scene_with_sensors(xml: str, entity_name: str, sensors: tuple, backend: str, num_envs: int = 2, njmax: int = 50,
                        skip: tuple[str, ...] = ()):
  """test_contact_sensor.py:102-130 (create_scene_with_sensor)."""
  dev = device_of(backend)
  scene = Scene(SceneCfg(num_envs=num_envs, env_spacing=3.0, entities={entity_name: EntityCfg(
    spec_fn=lambda: read_mjcf_string(xml))}, sensors=sensors), dev)
  model = scene.compile()
  sim = make_sim(num_envs, SimulationCfg(njmax=njmax), model, backend, skip=skip)
  scene.initialize(sim.mj_model, sim.model, sim.data)
  return scene, sim


def _place(entity, sim, z: float) -> torch.Tensor:
  rs = torch.zeros((sim.num_envs, 13), device=sim.device)
  rs[:, 2] = z
  rs[:, 3] = 1.0
  entity.write_root_state_to_sim(rs)
  return rs


def _settle(sim, n: int = 30) -> None:
  for _ in range(n):
    sim.step()


def _box_sensor(fields=("found", "force"), **kw) -> ContactSensorCfg:
  return ContactSensorCfg(name="box_contact", primary=ContactMatch(mode="geom", pattern="box_geom", entity="box"),
                          secondary=None, fields=fields, **kw)


def _feet(**kw) -> ContactMatch:
  return ContactMatch(mode="geom", pattern=kw.pop("pattern", ("left_foot_geom", "right_foot_geom")), entity="biped", **kw)


def test_basic_contact_detection(backend):
  """test_contact_sensor.py:147-188."""
  scene, sim = _scene_with_sensors(FALLING_BOX_XML, "box", (_box_sensor(),), backend)
  sensor = scene["box_contact"]
  _place(scene["box"], sim, 0.11)
  _settle(sim)
  data = sensor.data
  assert data.found is not None and data.force is not None
  assert data.found.shape == (2, 1)
  assert data.force.shape[-1] == 3
  assert torch.any(data.found > 0)
  assert torch.any(torch.abs(data.force[data.found > 0]) > 0)
  # numeric pin (not in the reference test): a 1 kg box at rest carries its
  # weight; maxforce reports the largest of its corner contacts in the contact
  # frame (normal first), and the four corners share m*g
  fn = data.force[..., 0]
  assert torch.all(fn > 0.2 * 9.81) and torch.all(fn < 9.81 + 0.5)


def test_contact_fields(backend):
  """test_contact_sensor.py:191-231. The box rests on four corner contacts
  carrying near-equal forces, so the maxforce reduction's pick (and with it
  pos/torque) may differ between float32 and float64 while every force agrees:
  the shadow skips sensordata here and the test checks what is determined."""
  scene, sim = _scene_with_sensors(
    FALLING_BOX_XML, "box", (_box_sensor(fields=("found", "force", "torque", "dist", "pos", "normal")),), backend,
    skip=("sensordata",))
  _place(scene["box"], sim, 0.105)
  _settle(sim, 10)
  data = scene["box_contact"].data
  for f in ("found", "force", "torque", "dist", "pos", "normal"):
    assert getattr(data, f) is not None
  for f in ("force", "torque", "pos", "normal"):
    assert getattr(data, f).shape[-1] == 3
  assert len(data.dist.shape) == 2
  # numeric pin (after the box has landed: 10 steps cover 2 of its 5 mm drop):
  # normal (0, 0, -1): the sensor reports it primary (box) -> secondary (the
  # ground), docs/api/sensors.md:166; contact point on the plane, small penetration
  _settle(sim, 60)
  data = scene["box_contact"].data
  assert torch.all(data.found > 0)
  assert torch.allclose(data.normal[:, 0], torch.tensor([0.0, 0.0, -1.0], device=sim.device).expand(2, 3), atol=1e-3)
  assert torch.all(data.pos[:, 0, 2].abs() < 2e-3) and torch.all(data.dist.abs() < 2e-3)


def test_multi_slot_pattern_matching(backend):
  """test_contact_sensor.py:239-278."""
  cfg = ContactSensorCfg(name="feet_contact", primary=_feet(), secondary=None, fields=("found", "force"),
                         track_air_time=True)
  scene, sim = _scene_with_sensors(BIPED_XML, "biped", (cfg,), backend)
  _place(scene["biped"], sim, 0.25)
  _settle(sim, 20)
  data = scene["feet_contact"].data
  assert data.found.shape == (2, 2)
  assert data.force.shape == (2, 2, 3)
  assert hasattr(data, "current_air_time")
  assert data.current_air_time.shape == (2, 2)


def test_regex_pattern_matching(backend):
  """test_contact_sensor.py:281-320."""
  cfg = ContactSensorCfg(name="all_feet_contact", primary=_feet(pattern=r".*foot_geom$"), secondary=None,
                         fields=("found", "force"))
  scene, sim = _scene_with_sensors(BIPED_XML, "biped", (cfg,), backend)
  assert scene["all_feet_contact"].data.found.shape == (2, 2)
  _place(scene["biped"], sim, 0.24)
  _settle(sim, 20)
  data = scene["all_feet_contact"].data
  assert torch.any(data.found > 0)
  assert data.force is not None and data.force.shape == (2, 2, 3)


@pytest.mark.parametrize("reduce_mode", ["none", "mindist", "maxforce", "netforce"])
def test_reduce_modes(backend, reduce_mode):
  """test_contact_sensor.py:328-354 (+ one step and a numeric check per mode)."""
  scene, sim = _scene_with_sensors(FALLING_BOX_XML, "box", (_box_sensor(fields=("force",), reduce=reduce_mode,
                                                                        num_slots=1),), backend)
  data = scene["box_contact"].data
  assert len(data.force.shape) == 3
  assert data.force.shape[-1] == 3
  if backend == "hip":
    _place(scene["box"], sim, 0.1)
    _settle(sim, 30)
    f = scene["box_contact"].data.force[:, 0]
    if reduce_mode == "netforce":  # the whole weight, in the global frame, along +z
      assert torch.allclose(f[:, 2], torch.full((2,), 9.81, device=f.device), rtol=0.05)
    else:  # one corner's contact-frame force: normal component > 0
      assert torch.all(f[:, 0] > 0)


def test_reduce_modes_multiple_contacts(backend):
  """test_contact_sensor.py:357-389."""
  cfg = ContactSensorCfg(name="feet_contact", primary=_feet(), secondary=None, fields=("found", "force", "dist"),
                         reduce="mindist", num_slots=1)
  scene, sim = _scene_with_sensors(BIPED_XML, "biped", (cfg,), backend)
  _place(scene["biped"], sim, 0.25)
  _settle(sim, 20)
  data = scene["feet_contact"].data
  assert data.found.shape == (2, 2)
  assert data.force.shape == (2, 2, 3)


@pytest.mark.parametrize("exclude,expected", [
  (("leg1_foot_collision", "leg2_foot_collision"), 6),  # test_contact_sensor.py:397-424
  ((r".*thigh_collision\d+",), 4),  # :427-452
  (("trunk_collision", r".*foot_collision"), 5),  # :455-483
])
def test_exclude_patterns(exclude, expected):
  cfg = ContactSensorCfg(name="s", primary=ContactMatch(mode="geom", pattern=r".*_collision\d*$", entity="robot",
                                                        exclude=exclude), secondary=None, fields=("found",))
  scene, _ = _scene_with_sensors(SIMPLE_ROBOT_XML, "robot", (cfg,), "oracle")
  assert scene["s"].data.found.shape == (2, expected)


def test_body_mode_contacts():
  """test_contact_sensor.py:491-506."""
  cfg = ContactSensorCfg(name="body_contact", primary=ContactMatch(mode="body", pattern="base", entity="biped"),
                         secondary=None, fields=("found",))
  scene, _ = _scene_with_sensors(BIPED_XML, "biped", (cfg,), "oracle")
  assert scene["body_contact"].data.found.shape[1] == 1


def test_subtree_mode_contacts(backend):
  """test_contact_sensor.py:509-534."""
  cfg = ContactSensorCfg(name="subtree_contact", primary=ContactMatch(mode="subtree", pattern="base", entity="biped"),
                         secondary=None, fields=("found",))
  scene, sim = _scene_with_sensors(BIPED_XML, "biped", (cfg,), backend)
  _place(scene["biped"], sim, 0.2)
  _settle(sim, 30)
  assert torch.any(scene["subtree_contact"].data.found > 0)


def test_air_time_tracking(backend):
  """test_contact_sensor.py:542-605."""
  cfg = ContactSensorCfg(name="feet_contact", primary=_feet(), secondary=None, fields=("found",), track_air_time=True)
  scene, sim = _scene_with_sensors(BIPED_XML, "biped", (cfg,), backend)
  sensor, biped = scene["feet_contact"], scene["biped"]
  rs = _place(biped, sim, 0.24)
  _settle(sim, 30)
  assert torch.any(sensor.data.found > 0)
  rs[:, 2] = 1.0
  biped.write_root_state_to_sim(rs)
  _settle(sim, 20)
  data2 = sensor.data
  assert torch.all(data2.found == 0)
  assert hasattr(data2, "current_air_time") and hasattr(data2, "last_air_time")
  rs[:, 2] = 0.24
  biped.write_root_state_to_sim(rs)
  _settle(sim, 30)
  assert torch.any(sensor.data.found > 0)


def test_multiple_sensors():
  """test_contact_sensor.py:613-649."""
  l = ContactSensorCfg(name="left_foot_contact", primary=_feet(pattern="left_foot_geom"), secondary=None,
                       fields=("found", "force"))
  r = ContactSensorCfg(name="right_foot_contact", primary=_feet(pattern="right_foot_geom"), secondary=None,
                       fields=("found", "force"))
  scene, _ = _scene_with_sensors(BIPED_XML, "biped", (l, r), "oracle", njmax=40)
  assert scene["left_foot_contact"].data.found.shape == (2, 1)
  assert scene["right_foot_contact"].data.found.shape == (2, 1)


def test_no_contacts(backend):
  """test_contact_sensor.py:657-685."""
  scene, sim = _scene_with_sensors(FALLING_BOX_XML, "box", (_box_sensor(),), backend)
  _place(scene["box"], sim, 5.0)
  sim.step()
  data = scene["box_contact"].data
  assert torch.all(data.found == 0)
  assert torch.all(data.force == 0)


def test_num_slots_greater_than_one(backend):
  """test_contact_sensor.py:688-757."""
  s1 = ContactSensorCfg(name="feet_contact_single", primary=_feet(), secondary=None, fields=("found", "force", "normal"),
                        num_slots=1)
  s3 = ContactSensorCfg(name="feet_contact_triple", primary=_feet(), secondary=None, fields=("found", "force", "normal"),
                        num_slots=3)
  scene, sim = _scene_with_sensors(BIPED_XML, "biped", (s1, s3), backend, njmax=40)
  _place(scene["biped"], sim, 0.25)
  _settle(sim, 20)
  d1, d3 = scene["feet_contact_single"].data, scene["feet_contact_triple"].data
  assert d1.found.shape == (2, 2) and d1.force.shape == (2, 2, 3) and d1.normal.shape == (2, 2, 3)
  assert d3.found.shape == (2, 6) and d3.force.shape == (2, 6, 3) and d3.normal.shape == (2, 6, 3)
  # numeric pin: slot 0 of the 3-slot maxforce sensor is the 1-slot sensor's
  # record (same top-1), and found counts the matches before reduction
  assert torch.equal(d3.found.view(2, 2, 3)[..., 0], d1.found)
  assert torch.allclose(d3.force.view(2, 2, 3, 3)[:, :, 0], d1.force, atol=1e-6)


# ---------------------------------------------------------------------------
# tests/test_builtin_sensor.py:23-139
# ---------------------------------------------------------------------------
ARTICULATED_ROBOT_XML = """
<mujoco><worldbody>
  <geom name="floor" type="plane" size="5 5 0.1" pos="0 0 0"/>
  <body name="base" pos="0 0 1">
    <freejoint name="free_joint"/>
    <geom name="base_geom" type="box" size="0.2 0.2 0.1" mass="5.0"/>
    <site name="base_site" pos="0 0 0"/>
    <body name="link1" pos="0.3 0 0">
      <joint name="joint1" type="hinge" axis="0 0 1" range="-1.57 1.57"/>
      <geom name="link1_geom" type="box" size="0.1 0.1 0.1" mass="1.0"/>
      <site name="link1_site" pos="0 0 0"/>
    </body>
  </body>
</worldbody></mujoco>"""


def _robot_scene(sensor_cfg, backend):
  dev = device_of(backend)
  scene = Scene(SceneCfg(num_envs=2, env_spacing=3.0, entities={"robot": EntityCfg(
    spec_fn=lambda: read_mjcf_string(ARTICULATED_ROBOT_XML))}, sensors=(sensor_cfg,)), dev)
  model = scene.compile()
  sim = make_sim(2, SimulationCfg(njmax=20), model, backend)
  scene.initialize(sim.mj_model, sim.model, sim.data)
  return scene, sim


def test_jointpos_sensor(backend):
  """test_builtin_sensor.py:70-100."""
  cfg = BuiltinSensorCfg(name="joint1_pos", sensor_type="jointpos", obj=ObjRef(type="joint", name="joint1",
                                                                                 entity="robot"))
  scene, sim = _robot_scene(cfg, backend)
  sensor = scene["robot/joint1_pos"]
  sim.step()
  data = sensor.data
  assert isinstance(data, torch.Tensor)
  assert data.shape == (2, 1)
  # numeric pin: jointpos = qpos of joint1 before integration (sensor_pos stage)
  assert torch.allclose(data[:, 0], torch.zeros(2, device=sim.device), atol=1e-6)


def test_accelerometer_sensor(backend):
  """test_builtin_sensor.py:103-138. The robot drops 0.2 s without reaching the
  floor: a free-falling accelerometer reads gravity-compensated cacc, which is
  zero up to rounding; the reference asserts only ``any(|a| > 0)``, which its
  rounding satisfies. Here the robot is additionally stepped onto the floor
  (0.6 s) so the reading is the support force, and it is checked numerically."""
  cfg = BuiltinSensorCfg(name="base_accel", sensor_type="accelerometer", obj=ObjRef(type="site", name="base_site",
                                                                                    entity="robot"))
  scene, sim = _robot_scene(cfg, backend)
  sensor = scene["robot/base_accel"]
  for _ in range(100):
    sim.step()
  data = sensor.data
  assert isinstance(data, torch.Tensor)
  assert data.shape == (2, 3)
  assert torch.all(data.abs() < 1e-2)  # free fall
  for _ in range(300):
    sim.step()
  # at rest on the floor: the proper acceleration is +g along the body z axis
  assert torch.allclose(sensor.data[:, 2], torch.full((2,), 9.81, device=sim.device), atol=0.2)


def test_builtin_sensor_types_beyond_the_benchmark_set(backend):
  """The remaining BuiltinSensorCfg types of builtin_sensor.py:30-110 through the
  same Scene path (not in the reference's test file; numeric pins from the
  scene): framepos of link1's site in the base frame is the joint offset
  (0.3, 0, 0) whatever the hinge angle; e_potential of the 6 kg robot at
  z = 1 m is m g z; e_kinetic at rest is 0; clock reads the data time before
  the step; the base site's rangefinder (z up) sees nothing (-1); the force
  at link1's site carries link1's weight while the robot falls freely (0 up to
  rounding)."""
  cfgs = (
    BuiltinSensorCfg(name="l1_in_base", sensor_type="framepos", obj=ObjRef(type="site", name="link1_site", entity="robot"),
                     ref=ObjRef(type="xbody", name="base", entity="robot")),
    BuiltinSensorCfg(name="epot", sensor_type="e_potential"),
    BuiltinSensorCfg(name="ekin", sensor_type="e_kinetic"),
    BuiltinSensorCfg(name="clk", sensor_type="clock"),
    BuiltinSensorCfg(name="range_up", sensor_type="rangefinder", obj=ObjRef(type="site", name="base_site", entity="robot")),
    BuiltinSensorCfg(name="l1_force", sensor_type="force", obj=ObjRef(type="site", name="link1_site", entity="robot")),
  )
  dev = device_of(backend)
  scene = Scene(SceneCfg(num_envs=2, env_spacing=3.0, entities={"robot": EntityCfg(
    spec_fn=lambda: read_mjcf_string(ARTICULATED_ROBOT_XML))}, sensors=cfgs), dev)
  model = scene.compile()
  assert model.nsensor_ext == 6  # all outside the benchmark set: the generic kernel instance
  sim = make_sim(2, SimulationCfg(njmax=20), model, backend)
  scene.initialize(sim.mj_model, sim.model, sim.data)
  sim.step()
  d = {k: scene[k].data for k in ("robot/l1_in_base", "epot", "ekin", "clk", "robot/range_up", "robot/l1_force")}
  assert d["robot/l1_in_base"].shape == (2, 3) and d["epot"].shape == (2, 1)
  assert torch.allclose(d["robot/l1_in_base"], torch.tensor([[0.3, 0.0, 0.0]] * 2, device=dev), atol=1e-5)
  assert torch.allclose(d["epot"][:, 0], torch.full((2,), 6 * 9.81, device=dev), rtol=1e-5)
  assert torch.allclose(d["ekin"][:, 0], torch.zeros(2, device=dev), atol=1e-9)
  assert torch.allclose(d["clk"][:, 0], torch.zeros(2, device=dev))
  assert torch.equal(d["robot/range_up"][:, 0], torch.full((2,), -1.0, device=dev))
  assert torch.allclose(d["robot/l1_force"], torch.zeros(2, 3, device=dev), atol=1e-3)
  sim.step()
  assert torch.allclose(scene["clk"].data[:, 0], torch.full((2,), float(model.timestep), device=dev), atol=1e-7)


def test_builtin_sensor_cfg_validation():
  """builtin_sensor.py:206-259 (the reference's cfg checks)."""
  with pytest.raises(ValueError, match="requires obj.type='site'"):
    BuiltinSensorCfg(name="a", sensor_type="accelerometer", obj=ObjRef(type="body", name="base"))
  with pytest.raises(ValueError, match="does not support ref"):
    BuiltinSensorCfg(name="a", sensor_type="jointpos", obj=ObjRef(type="joint", name="j"),
                     ref=ObjRef(type="body", name="b"))
  assert BuiltinSensorCfg(name="a", sensor_type="gyro", obj=ObjRef(type="site", name="s", entity="robot")).name == \
    "robot/a"


# ---------------------------------------------------------------------------
# tests/test_events.py:21-119
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dev", [pytest.param("cpu"), pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_reset_joints_by_offset(dev):
  """test_events.py:21-66, with the reference's Mock entity."""
  env = Mock()
  env.num_envs = 2
  env.device = dev
  ent = Mock()
  ent.data.default_joint_pos = torch.zeros((2, 3), device=dev)
  ent.data.default_joint_vel = torch.zeros((2, 3), device=dev)
  ent.data.soft_joint_pos_limits = torch.tensor([[[-0.5, 0.5]] * 3] * 2, device=dev)
  ent.write_joint_state_to_sim = Mock()
  env.scene = {"robot": ent}
  events.reset_joints_by_offset(env, torch.tensor([0], device=dev), position_range=(0.3, 0.3),
                                velocity_range=(0.2, 0.2), asset_cfg=SceneEntityCfg("robot", joint_ids=slice(None)))
  jp, jv = ent.write_joint_state_to_sim.call_args[0][:2]
  assert torch.allclose(jp, torch.ones_like(jp) * 0.3)
  assert torch.allclose(jv, torch.ones_like(jv) * 0.2)
  events.reset_joints_by_offset(env, torch.tensor([1], device=dev), position_range=(1.0, 1.0),
                                velocity_range=(0.0, 0.0), asset_cfg=SceneEntityCfg("robot", joint_ids=slice(None)))
  jp = ent.write_joint_state_to_sim.call_args[0][0]
  assert torch.allclose(jp, torch.ones_like(jp) * 0.5)


def test_class_based_event_with_domain_randomization():
  """test_events.py:69-119."""

  class CustomRandomizer:
    def __init__(self, cfg, env):
      self.cfg, self.env = cfg, env

    def __call__(self, env, env_ids, field, ranges):
      pass

  env = Mock()
  env.num_envs = 4
  env.device = "cpu"
  env.scene = {}
  env.sim = Mock()
  cfg = {
    "custom_dr": EventTermCfg(mode="startup", func=CustomRandomizer, domain_randomization=True,
                              params={"field": "geom_friction", "ranges": (0.3, 1.2)}),
    "standard_dr": EventTermCfg(mode="reset", func=events.randomize_field, domain_randomization=True,
                                params={"field": "body_mass", "ranges": (0.8, 1.2)}),
    "regular_event": EventTermCfg(mode="reset", func=events.reset_joints_by_offset,
                                  params={"position_range": (-0.1, 0.1), "velocity_range": (0.0, 0.0)}),
  }
  manager = EventManager(cfg, env)
  assert "geom_friction" in manager.domain_randomization_fields
  assert "body_mass" in manager.domain_randomization_fields
  assert len(manager.domain_randomization_fields) == 2


# ---------------------------------------------------------------------------
# tests/test_sim.py:17-82
# ---------------------------------------------------------------------------
SIM_ROBOT_XML = """
<mujoco><worldbody>
  <body name="base" pos="0 0 1">
    <freejoint name="free_joint"/>
    <geom name="base_geom" type="box" size="0.1 0.1 0.1" mass="1.0" friction="0.5 0.01 0.005"/>
    <body name="foot1" pos="0.2 0 0">
      <joint name="joint1" type="hinge" axis="0 0 1" range="0 1.57"/>
      <geom name="foot1_geom" type="box" size="0.05 0.05 0.05" mass="0.1" friction="0.5 0.01 0.005"/>
    </body>
    <body name="foot2" pos="-0.2 0 0">
      <joint name="joint2" type="hinge" axis="0 0 1" range="0 1.57"/>
      <geom name="foot2_geom" type="box" size="0.05 0.05 0.05" mass="0.1" friction="0.5 0.01 0.005"/>
    </body>
  </body>
</worldbody></mujoco>"""

MJ_INT_EULER, MJ_SOL_CG = 0, 1
MJ_SOL_PGS = 0


def test_simulation_config_is_piped(backend):
  """test_sim.py:43-82, as the reference writes it (solver="cg"); solver="pgs"
  is piped too (MuJoCo's mjSOL_PGS, pyramidal cones), PGS with elliptic cones
  is refused rather than silently replaced."""
  model = compile_spec(read_mjcf_string(SIM_ROBOT_XML))
  cfg = SimulationCfg(contact_sensor_maxmatch=128, ls_parallel=False,
                      mujoco=MujocoCfg(timestep=0.02, integrator="euler", solver="cg", iterations=7,
                                       ls_iterations=14, gravity=(0, 0, 7.5)))
  sim = make_sim(1, cfg, model, backend)
  assert sim.mj_model.opt.timestep == cfg.mujoco.timestep
  assert sim.mj_model.opt.integrator == MJ_INT_EULER
  assert sim.mj_model.opt.solver == MJ_SOL_CG
  assert sim.mj_model.opt.iterations == cfg.mujoco.iterations
  assert tuple(sim.mj_model.opt.gravity) == cfg.mujoco.gravity
  np.testing.assert_almost_equal(sim.model.opt.timestep[0].cpu().numpy(), cfg.mujoco.timestep)
  np.testing.assert_almost_equal(sim.model.opt.gravity[0].cpu().numpy(), cfg.mujoco.gravity)
  assert sim.model.opt.integrator == MJ_INT_EULER
  assert sim.model.opt.solver == MJ_SOL_CG
  assert sim.model.opt.iterations == cfg.mujoco.iterations
  assert sim.wp_model.opt.contact_sensor_maxmatch == cfg.contact_sensor_maxmatch
  assert sim.wp_model.opt.ls_parallel == cfg.ls_parallel
  # the piped options reach the step: one Euler step under +7.5 gravity
  sim.step()
  assert abs(float(sim.data.qvel[0, 2]) - 7.5 * 0.02) < 1e-5
  pgs = make_sim(1, SimulationCfg(mujoco=MujocoCfg(solver="pgs")), compile_spec(read_mjcf_string(SIM_ROBOT_XML)), backend)
  assert pgs.mj_model.opt.solver == MJ_SOL_PGS and pgs.model.opt.solver == MJ_SOL_PGS
  pgs.step()
  with pytest.raises(NotImplementedError):
    make_sim(1, SimulationCfg(mujoco=MujocoCfg(solver="pgs", cone="elliptic")), compile_spec(read_mjcf_string(SIM_ROBOT_XML)),
             backend)


# ---------------------------------------------------------------------------
# tests/test_domain_randomization.py:19-144
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("field,ranges,operation,asset_names,axes,seed", [
  ("geom_friction", (0.3, 1.2), "abs", {"geom_names": [".*"]}, [0], 123),
  ("body_mass", (0.8, 1.2), "scale", {"body_names": [".*"]}, None, 456),
  ("dof_damping", (0.1, 0.5), "abs", {"joint_names": [".*"]}, None, 789),
])
def test_randomize_field(backend, field, ranges, operation, asset_names, axes, seed):
  """test_domain_randomization.py:91-144 (+ on the HIP backend: one step with
  the randomised per-world field, checked against the oracle fed the same
  per-world values)."""
  torch.manual_seed(seed)
  dev = device_of(backend)
  n = 4
  scene = Scene(SceneCfg(num_envs=n, entities={"robot": EntityCfg(spec_fn=lambda: read_mjcf_string(SIM_ROBOT_XML))}),
                dev)
  model = scene.compile()
  sim = make_sim(n, SimulationCfg(), model, backend)
  scene.initialize(model, sim.model, sim.data)
  sim.expand_model_fields(("geom_friction", "body_mass", "dof_damping"))
  expanded_fields_attach(sim)

  class Env:
    pass

  env = Env()
  env.scene, env.sim, env.num_envs, env.device = scene, sim, n, dev
  robot = scene["robot"]
  if field == "geom_friction":
    idx = robot.indexing.geom_ids
    model_field = sim.model.geom_friction[:, idx[0], 0]
  elif field == "body_mass":
    idx = robot.indexing.body_ids
    model_field = sim.model.body_mass[:, idx[0]]
  else:
    idx = robot.indexing.joint_v_adr
    sim.model.dof_damping[:, idx.long()] = 0.0
    model_field = sim.model.dof_damping[:, idx[0]]
  initial = model_field.clone()
  sc = SceneEntityCfg("robot", **asset_names)
  sc.resolve(scene)
  events.randomize_field(env, env_ids=None, field=field, ranges=ranges, operation=operation, asset_cfg=sc, axes=axes)
  new = model_field
  assert not torch.all(new == initial)
  if operation == "abs":
    assert torch.all((new >= ranges[0]) & (new <= ranges[1]))
  else:
    assert torch.all((new >= ranges[0] * initial) & (new <= ranges[1] * initial))
  assert len(torch.unique(new)) >= 2
  if backend == "hip":
    sim.data.qvel[:, 6:] = 1.0  # joint velocities so that damping acts
    sim.step()  # shadowed: per-world fields must reach the kernel
