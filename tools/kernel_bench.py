"""Time the physics step kernel alone at the bench size (diagnostic tool).

usage: [MJH_LIB=<lib.so>] [MJH_SPEC=0] [MJH_BALANCE=1] [MJH_LS_PARALLEL=0] python tools/kernel_bench.py [N] [launches] [task]
Builds the task's model exactly as the env does (so the model-specialised
instance is used unless MJH_SPEC=0), settles random states for 20 steps, then
times `launches` step launches with HIP events and reports ms/launch,
world-steps/s, mean nefc and iterations.
"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np
import torch

from mjlab_amd.scene.scene import Scene
from mjlab_amd.sim import Simulation, native
from mjlab_amd.tasks import load_env_cfg
from tests.scenes import random_states

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 40
task = sys.argv[3] if len(sys.argv) > 3 else "Mjlab-Velocity-Flat-Unitree-G1"
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
cfg.sim.balance_worlds = os.environ.get("MJH_BALANCE", "0") == "1"  # A/B: cost-sorted world order
cfg.sim.ls_parallel = os.environ.get("MJH_LS_PARALLEL", "1") == "1"  # A/B: parallel vs exact line search
m = Scene(cfg.scene, device="cuda:0").compile()
sim = Simulation(n, cfg.sim, m, "cuda:0")
st = random_states(m, n, np.random.default_rng(0), drop=0.03)
for k, v in st.items():
  t = getattr(sim.data, k)
  t.copy_(torch.as_tensor(v, dtype=t.dtype, device="cuda:0").view_as(t))
for _ in range(20):
  sim.step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(launches):
  sim.step()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / launches
spec = native.lib().mjh_spec_index(ctypes.addressof(sim._mstruct)) if os.environ.get("MJH_SPEC") != "0" else -1
print(f"{os.environ.get('MJH_LIB', 'libmjh.so')} spec={spec} balance={int(cfg.sim.balance_worlds)} "
      f"ls_parallel={int(cfg.sim.ls_parallel)}: {task} N={n} {ms:.3f} ms/launch  {n / ms * 1e3:,.0f} world-steps/s  "
      f"nefc {sim.data.nefc.float().mean().item():.1f}  niter {sim.data.solver_niter.float().mean().item():.2f}  "
      f"lds {sim.scratch_bytes()} rcap {sim.efc_capacity()} flags {int((sim.data.flags != 0).sum())}")
