"""Entity write API (restates tests/test_entity.py:222-242 and the velocity
frame conventions of entity/data.py:95-106) on CPU tensors."""

import math

import torch

from mjlab_amd.scene.scene import Scene
from mjlab_amd.sim import Simulation, SimulationCfg
from tests.scenes import g1_scene


def setup(n=3):
  sc = g1_scene(n)
  m = sc.compile(50, 300)
  sim = Simulation(n, SimulationCfg(nconmax=50, njmax=300), m, "cpu")
  sc.initialize(m, sim.model, sim.data)
  return sc["robot"], sim


def test_root_state_write_identity_quat():
  robot, sim = setup(1)
  rs = torch.tensor([[1.0, 2.0, 3.0, 1.0, 0.0, 0.0, 0.0, 0.5, 0.0, 0.0, 0.0, 0.0, 0.2]])
  robot.write_root_state_to_sim(rs)
  ix = robot.data.indexing
  assert torch.allclose(sim.data.qpos[:, ix.free_joint_q_adr.long()], rs[:, :7])
  assert torch.allclose(sim.data.qvel[:, ix.free_joint_v_adr.long()], rs[:, 7:])


def test_root_angular_velocity_is_stored_in_body_frame():
  robot, sim = setup(1)
  yaw = math.pi / 2
  q = [math.cos(yaw / 2), 0.0, 0.0, math.sin(yaw / 2)]
  rs = torch.tensor([[0.0, 0.0, 1.0, *q, 0.3, 0.0, 0.0, 1.0, 0.0, 0.0]])
  robot.write_root_state_to_sim(rs)
  v = sim.data.qvel[0, robot.data.indexing.free_joint_v_adr.long()]
  assert torch.allclose(v[:3], torch.tensor([0.3, 0.0, 0.0]))  # linear stays world
  assert torch.allclose(v[3:], torch.tensor([0.0, -1.0, 0.0]), atol=1e-6)  # world x -> body -y


def test_masked_and_indexed_writes_agree():
  robot, sim = setup(4)
  jp = torch.randn(4, robot.num_joints)
  mask = torch.tensor([True, False, True, False])
  before = robot.data.joint_pos.clone()
  robot.write_joint_position_to_sim(jp, env_ids=mask)
  after = robot.data.joint_pos
  assert torch.equal(after[mask], jp[mask]) and torch.equal(after[~mask], before[~mask])
  jp2 = torch.randn(2, robot.num_joints)
  robot.write_joint_position_to_sim(jp2, env_ids=torch.tensor([1, 3]))
  assert torch.equal(robot.data.joint_pos[[1, 3]], jp2)


def test_clear_state_zeroes_applied_wrenches_and_ctrl():
  robot, sim = setup(2)
  sim.data.xfrc_applied.fill_(1.0)
  sim.data.ctrl.fill_(1.0)
  robot.clear_state(torch.tensor([True, False]))
  bids = robot.data.indexing.body_ids.long()
  assert (sim.data.xfrc_applied[0, bids] == 0).all() and (sim.data.xfrc_applied[1, bids] == 1).all()
  assert (sim.data.ctrl[0] == 0).all() and (sim.data.ctrl[1] == 1).all()


def test_bridge_is_pointer_stable():
  _, sim = setup(1)
  import pytest

  with pytest.raises(AttributeError):
    sim.data.qpos = torch.zeros(1, 36)
