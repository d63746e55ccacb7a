"""Bitwise comparison of two step-library builds on the same inputs (diagnostic, GPU box).

usage: python tools/lib_diff.py dump <out.npz> [task] [n] [steps]   (MJH_LIB selects the build)
       python tools/lib_diff.py cmp <a.npz> <b.npz>
Runs `steps` physics steps of the task's model from seeded random states and saves the
data arrays; `cmp` reports, per field, the count of differing elements.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))

if sys.argv[1] == "cmp":
  a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
  bad = 0
  for k in a.files:
    d = int(np.sum(a[k].view(np.uint8) != b[k].view(np.uint8))) if a[k].shape == b[k].shape else -1
    if d:
      bad += 1
      print(f"{k:28s} differing bytes {d}")
  print("identical" if not bad else f"{bad} fields differ")
  sys.exit(0)

import torch  # noqa: E402

from mjlab_amd.scene.scene import Scene  # noqa: E402
from mjlab_amd.sim import Simulation  # noqa: E402
from mjlab_amd.tasks import load_env_cfg  # noqa: E402
from tests.scenes import random_states  # noqa: E402

out = sys.argv[2]
task = sys.argv[3] if len(sys.argv) > 3 else "Mjlab-Velocity-Flat-Unitree-G1"
n = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
cfg = load_env_cfg(task)
cfg.scene.num_envs = n
m = Scene(cfg.scene, device="cuda:0").compile()
sim = Simulation(n, cfg.sim, m, "cuda:0")
st = random_states(m, n, np.random.default_rng(0), drop=0.03)
for k, v in st.items():
  t = getattr(sim.data, k)
  t.copy_(torch.as_tensor(v, dtype=t.dtype, device="cuda:0").view_as(t))
for _ in range(steps):
  sim.step()
torch.cuda.synchronize()
np.savez(out, **{k: getattr(sim.data, k).detach().cpu().numpy() for k in sim.data.fields()})
print("saved", out)
