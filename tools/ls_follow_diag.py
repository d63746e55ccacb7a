"""Diagnostics: the device's recorded step-size choices (solver_lstrace) and the
oracle replaying them (follow mode), G1 256 worlds, parity-test seed."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import numpy as np  # noqa: E402

from oracle.oracle import Oracle  # noqa: E402
from tests.scenes import compare_step, g1_scene_model, random_states  # noqa: E402
from tests.test_gpu_parity import get, make_sim, put  # noqa: E402


def dec(t, k=10):
  return [(int(t[i // 5]) >> (6 * (i % 5))) & 63 for i in range(k)]


n = 256
m = g1_scene_model(n)
st = random_states(m, n, np.random.default_rng(1))
sim = make_sim(m, n, ls_parallel=True)
put(sim, st)
sim.step()
got = get(sim, n)
free = Oracle(m).run(n, st, integrate=True)
fol = Oracle(m).run(n, st, integrate=True, follow=got)
rep = compare_step(got, fol)
print("failures", rep["failures"][:4])
ex = fol["ls_excess"][:, 0]
for w in np.argsort(-ex)[:6]:
  print(f"world {w} excess {ex[w]:.3e} freegap {free['ls_gap'][w, 0]:.3e} niter gpu {got['solver_niter'][w, 0]} free {free['solver_niter'][w, 0]} "
        f"follow {fol['solver_niter'][w, 0]} nefc gpu {got['nefc'][w, 0]} oracle {free['nefc'][w, 0]}")
  print("   gpu ", dec(got["solver_lstrace"][w]), got["solver_lstrace"][w])
  print("   free", dec(free["solver_lstrace"][w]))
  print("   fol ", dec(fol["solver_lstrace"][w]))
