"""Per-iteration solver comparison for selected worlds of the N=4096 parity
scenario: GPU forward vs float64 oracle with the iteration cap set to k."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np

from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
from oracle.oracle import Oracle
from tests.scenes import g1_scene_model, random_states
from tests.test_gpu_parity import get, put

W = [2809, 1928, 1230, 2246, 949, 5]
st_full = random_states(g1_scene_model(4096), 4096, np.random.default_rng(11))
st = {k: v[W] for k, v in st_full.items()}
n = len(W)
for k in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,5,10,100").split(",")]:
  m = g1_scene_model(n)
  sim = Simulation(n, SimulationCfg(nconmax=50, njmax=300, mujoco=MujocoCfg(timestep=0.005, iterations=k, ls_iterations=20)), m, "cuda:0")
  put(sim, st)
  sim.forward()
  g = get(sim, n)
  r = Oracle(m).run(n, st, integrate=False)
  rel = np.abs(g["qacc"] - r["qacc"]).max(1) / (1 + np.abs(r["qacc"]).max(1))
  print(k, "gpu_it", g["solver_niter"][:, 0].tolist(), "or_it", r["solver_niter"][:, 0].tolist(), "rel", " ".join(f"{x:.1e}" for x in rel))
