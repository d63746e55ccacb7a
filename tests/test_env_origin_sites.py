"""Env-origin sites as the reference compiles them (terrain_importer.py:95-120:
one transparent sphere site per env origin on the world body, so the model has
nsite = num_envs + robot sites and the robot's site ids start at num_envs).
They are static: the Simulation writes their poses once into the wide
(num_envs, nsite) site_xpos / site_xmat and the kernel's model view starts
after them (mjh_data.site_wstride / site_off, ABI 14). CPU checks here; the HIP
step's site outputs are compared with the oracle's full arrays in every GPU
parity test (tests/scenes.py KIN), and tests/test_gpu_env.py checks the static
block survives env steps."""

import numpy as np
import torch

from mjlab_amd.sim import Simulation, SimulationCfg
from mjlab_amd.tasks import load_env_cfg
from tests.scenes import g1_scene


def test_scene_compiles_one_site_per_env_origin_first():
  n = 8
  scene = g1_scene(n)
  m = scene.compile(50, 300)
  assert m.nsite_origin == n and m.nsite == n + 6
  assert m.names["site"][:n] == [f"env_origin_{i}" for i in range(n)]
  assert (np.asarray(m.site_bodyid)[:n] == 0).all()
  np.testing.assert_allclose(np.asarray(m.site_pos)[:n], scene.env_origins.cpu().numpy(), atol=1e-6)
  # the robot's sites follow: reference ids num_envs + k
  assert m.site("robot/left_foot").id == n + m.names["site"][n:].index("robot/left_foot")
  sim = Simulation(n, SimulationCfg(nconmax=50, njmax=300), m, "cpu")
  assert tuple(sim.data.site_xpos.shape) == (n, n + 6, 3) and tuple(sim.data.site_xmat.shape) == (n, n + 6, 3, 3)
  assert sim.ksizes["nsite"] == 6 and sim.sizes["nsite"] == n + 6
  origins = scene.env_origins.cpu()
  for w in range(n):  # every world row holds all origins (static, written once)
    torch.testing.assert_close(sim.data.site_xpos[w, :n].cpu(), origins)
  torch.testing.assert_close(sim.data.site_xmat[:, :n].cpu(), torch.eye(3).expand(n, n, 3, 3))
  assert sim._dstruct.site_wstride == n + 6 and sim._dstruct.site_off == n


def test_env_entity_site_ids_are_the_reference_indices():
  """In the velocity env, the robot's EntityData site ids are num_envs + k and
  its site reads take those columns of sim.data.site_xpos."""
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = 4
  from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv

  env = ManagerBasedRlEnv(cfg, device="cpu")
  robot = env.scene["robot"]
  ids = robot.indexing.site_ids.tolist()
  assert ids == list(range(4, 4 + len(ids))) and env.sim.mj_model.nsite == 4 + len(ids)
  assert env.sim.mj_model.names["site"][0] == "env_origin_0"
