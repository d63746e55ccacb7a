"""Re-run the GPU trajectory parity scenario and dump the first non-borderline
integer mismatch (input state + both outputs of that world) to
gpurun_out/mismatch.npz for offline analysis with the oracle."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np
import torch

from oracle.oracle import INPUTS, Oracle
from tests.scenes import g1_scene_model, int_mismatch_reason, random_states
from tests.test_gpu_parity import get, make_sim, put

n = 64
m = g1_scene_model(n)
sim = make_sim(m, n)
put(sim, random_states(m, n, np.random.default_rng(2), drop=0.03))
orc = Oracle(m)
for k in range(60):
  cur = get(sim, n)
  state = {f: cur[f] for f in INPUTS if f in cur}
  sim.step()
  nxt = get(sim, n)
  ref = orc.run(n, state, integrate=True)
  for w in range(n):
    r = int_mismatch_reason(nxt, ref, w)
    if r is not None:
      print(k, w, r)
      if not r[1]:
        out = {f"in_{f}": v[w] for f, v in state.items()}
        out.update({f"gpu_{f}": v[w] for f, v in nxt.items()})
        out.update({f"ref_{f}": v[w] for f, v in ref.items()})
        Path("gpurun_out").mkdir(exist_ok=True)
        np.savez("gpurun_out/mismatch.npz", **out)
        sys.exit(0)
print("no non-borderline mismatch")
