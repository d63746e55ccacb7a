"""SimulationCfg.nconmax as the reference defines it: the size of a contact
pool shared by the worlds ("Contacts exist in large heterogenous arrays: one
world may have more than nconmax contacts", /root/reference/src/mjlab/sim/
sim.py:81-85; MuJoCo Warp allocates nconmax x nworld). Each world gets
max(nconmax, njmax) contact slots (CPU: the sizes and
buffer shapes; the GPU keeps-more test is
tests/test_gpu_parity.py::test_pooled_contacts_one_world_exceeds_nconmax)."""

from mjlab_amd.sim import Simulation, SimulationCfg
from tests.scenes import g1_scene_model


def test_per_world_slots_from_the_pool():
  m = g1_scene_model(4)
  s = Simulation(4, SimulationCfg(nconmax=50, njmax=300), m, "cpu")
  assert (m.ncon_share, m.nconmax) == (50, 300)
  assert tuple(s.data.contact_dist.shape) == (4, 300)
  Simulation(64, SimulationCfg(nconmax=50, njmax=300), m, "cpu")
  assert (m.ncon_share, m.nconmax) == (50, 300)  # independent of the world count
  Simulation(2, SimulationCfg(nconmax=400, njmax=300), m, "cpu")
  assert (m.ncon_share, m.nconmax) == (400, 400)
  # nconmax unset: the model's share is kept (not the previous Simulation's slot count)
  Simulation(2, SimulationCfg(njmax=100), m, "cpu")
  assert (m.ncon_share, m.nconmax) == (400, 400)
  Simulation(2, SimulationCfg(nconmax=3, njmax=100), m, "cpu")
  assert (m.ncon_share, m.nconmax) == (3, 100)
