"""Mocap bodies (entity.py:101-104, 582-595; data.py:178-187): compiler ids,
the EntityData write, and the oracle's kinematics (pose from mocap_pos/quat)."""

import numpy as np
import pytest
import torch

from mjlab_amd.entity.entity import EntityCfg
from mjlab_amd.spec.mjcf import read_mjcf_string
from oracle.oracle import Oracle
from tests.scenes import g1_mocap_scene, mocap_states


def test_compiler_assigns_mocap_ids():
  m = g1_mocap_scene(2).compile(50, 300)
  ids = np.nonzero(m.body_mocapid >= 0)[0]
  assert m.nmocap == 1 and len(ids) == 1
  b = int(ids[0])
  assert m.body_parentid[b] == 0 and m.body_jntnum[b] == 0 and m.body_weldid[b] == 0
  # the ball collides with the robot, never with the (static) terrain plane
  g = [i for i in range(m.ngeom) if m.geom_bodyid[i] == b]
  pairs = {(int(a), int(c)) for a, c in zip(m.pair_geom1, m.pair_geom2)}
  assert any(g[0] in p for p in pairs)
  plane = [i for i in range(m.ngeom) if m.geom_type[i] == 0]
  assert not any({g[0], plane[0]} == set(p) for p in pairs)


def test_mocap_body_must_be_static_world_child():
  xml = ('<mujoco><worldbody><body name="a" mocap="true"><joint name="j" type="hinge"/>'
         '<geom type="sphere" size="0.1"/></body></worldbody></mujoco>')
  from mjlab_amd.scene.scene import Scene, SceneCfg

  sc = Scene(SceneCfg(num_envs=1, entities={"a": EntityCfg(spec_fn=lambda: read_mjcf_string(xml))}), "cpu")
  with pytest.raises(ValueError, match="mocap body"):
    sc.compile(10, 10)


def test_oracle_mocap_kinematics():
  m = g1_mocap_scene(4).compile(50, 300)
  st = mocap_states(m, 4, np.random.default_rng(3))
  ref = Oracle(m).run(4, st, integrate=False)
  b = int(np.nonzero(m.body_mocapid >= 0)[0][0])
  np.testing.assert_allclose(ref["xpos"].reshape(4, -1, 3)[:, b], st["mocap_pos"][:, :3], atol=1e-12)
  q = st["mocap_quat"][:, :4] / np.linalg.norm(st["mocap_quat"][:, :4], axis=1, keepdims=True)
  np.testing.assert_allclose(ref["xquat"].reshape(4, -1, 4)[:, b], q, atol=1e-12)


def test_entity_write_mocap_pose_cpu():
  """The write lands in the entity's mocap slot (Simulation data on CPU)."""
  from mjlab_amd.sim import Simulation, SimulationCfg

  sc = g1_mocap_scene(3)
  m = sc.compile(50, 300)
  sim = Simulation(3, SimulationCfg(nconmax=50, njmax=300), m, "cpu")
  sc.initialize(sim.mj_model, sim.model, sim.data)
  ball = sc["ball"]
  assert ball.is_fixed_base and ball.is_mocap and ball.indexing.mocap_id == 0
  b = int(np.nonzero(m.body_mocapid >= 0)[0][0])
  # mj_resetData: mocap poses start at the body's model pose
  torch.testing.assert_close(sim.data.mocap_pos[:, 0], torch.tensor(m.body_pos[b], dtype=torch.float32).expand(3, 3))
  pose = torch.tensor([[1.0, 2.0, 3.0, 1.0, 0.0, 0.0, 0.0], [4.0, 5.0, 6.0, 0.0, 1.0, 0.0, 0.0]])
  mask = torch.tensor([True, False, True])
  ball.write_mocap_pose_to_sim(pose[[0, 0, 1]], env_ids=mask)
  assert torch.equal(sim.data.mocap_pos[:, 0], torch.tensor([[1.0, 2.0, 3.0], list(m.body_pos[b]), [4.0, 5.0, 6.0]]))
  assert torch.equal(sim.data.mocap_quat[2, 0], torch.tensor([0.0, 1.0, 0.0, 0.0]))
  robot = sc["robot"]
  with pytest.raises(ValueError, match="non-mocap"):
    robot.data.write_mocap_pose(pose[:1].expand(3, -1))
