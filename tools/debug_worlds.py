"""Dump input state + GPU outputs of the N=4096 parity scenario for offline
analysis (gpurun_out/full4096.npz: inputs and the solver-related outputs)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np

from tests.scenes import g1_scene_model, random_states
from tests.test_gpu_parity import get, make_sim, put

n = 4096
m = g1_scene_model(n)
st = random_states(m, n, np.random.default_rng(11))
sim = make_sim(m, n)
put(sim, st)
sim.step()
got = get(sim, n)
Path("gpurun_out").mkdir(exist_ok=True)
keep = ("qacc", "qvel", "qpos", "qfrc_constraint", "sensordata", "solver_niter", "nefc", "ncon", "efc_force", "qacc_smooth")
np.savez_compressed("gpurun_out/full4096.npz", **{f"gpu_{k}": got[k] for k in keep})
print("ok")
