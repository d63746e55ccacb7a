"""Capture safety of graph owners (utils/capture.py).

Round 4's GPU run aborted inside an env-step capture while the cyclic
collector finalised earlier tests' objects (``gpurun_out/r04m/gputests.log:34``):
the destructor of a captured ``torch.cuda.CUDAGraph`` (an old env's or
Simulation's) ran inside another capture. Graph owners now hold only handles
(``GraphSlot``); a dying owner's graphs are retired and destroyed at the next
safe point. This test constructs that hazard on purpose: a Simulation and an
env holding captured graphs, dropped in reference cycles, collected INSIDE a
new capture. It runs in a child process so that a regression shows as a
failed test, not as an aborted test session."""

import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]

CHILD = r"""
import gc, sys
sys.path.insert(0, "asimov-mjlab_amd"); sys.path.insert(0, ".")
import torch
from mjlab_amd.envs.manager_based_rl_env import ManagerBasedRlEnv
from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
from mjlab_amd.tasks import load_env_cfg
from mjlab_amd.utils import capture
from tests.scenes import g1_scene_model

dev = "cuda:0"
cfg = SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.005))
old_sim = Simulation(8, cfg, g1_scene_model(8), dev)
old_sim.step()                      # replays its captured step graph
assert old_sim.step_graph is not None and old_sim.forward_graph is not None
old_sim.cycle = old_sim             # only the cyclic collector can free it
ecfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
ecfg.scene.num_envs = 16
old_env = ManagerBasedRlEnv(ecfg, device=dev)
old_env.reset()
act = torch.zeros(16, old_env.action_manager.total_action_dim, device=dev)
for _ in range(3):
  old_env.step(act)                 # the env step is captured on its 2nd call
assert old_env._graph is not None
old_env.cycle = old_env

new = Simulation(8, cfg, g1_scene_model(8), dev)
g = torch.cuda.CUDAGraph()
gc.disable()
with torch.cuda.graph(g):
  new._launch_step()
  del old_sim, old_env
  found = gc.collect()              # both owners die here, inside the capture
  retired = capture.retired_count()
  assert capture.release_retired() == 0   # nothing is destroyed while capturing
  new._launch_step()
gc.enable()
g.replay()
torch.cuda.synchronize()
assert found > 0, found
assert retired >= 3, retired        # step + forward graphs of the Simulations, the env step
assert capture.release_retired() >= 3   # released at the next safe point
torch.cuda.synchronize()
print("CAPTURE-SAFE OK", found, retired)
"""


def test_graph_owners_collected_inside_a_capture():
  env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
  r = subprocess.run([sys.executable, "-c", CHILD], cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
  tail = (r.stdout + r.stderr)[-3000:]
  assert r.returncode == 0, tail
  assert "CAPTURE-SAFE OK" in r.stdout, tail
