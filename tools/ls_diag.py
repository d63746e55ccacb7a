"""Diagnostics: per-world solver agreement of the HIP step with the oracle
under both line searches (G1, 256 worlds, tests/test_gpu_parity seeds)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import numpy as np  # noqa: E402

from oracle.oracle import Oracle  # noqa: E402
from tests.scenes import g1_scene_model, random_states  # noqa: E402
from tests.test_gpu_parity import get, make_sim, put  # noqa: E402

n = 256
for lsp in (True, False):
  m = g1_scene_model(n)
  st = random_states(m, n, np.random.default_rng(1))
  sim = make_sim(m, n, ls_parallel=lsp)
  put(sim, st)
  sim.step()
  got = get(sim, n)
  ref = Oracle(m).run(n, st, integrate=True)
  for k in ("qacc", "sensordata", "efc_force"):
    d = np.abs(got[k] - ref[k]).max(1) / (1 + np.abs(ref[k]).max(1))
    o = np.argsort(-d)[:6]
    print(f"ls_parallel={lsp} {k}: worst rel {np.round(d[o], 5)} worlds {o} niter gpu {got['solver_niter'][o, 0]} "
          f"oracle {ref['solver_niter'][o, 0]} gap {ref['ls_gap'][o, 0]}")
  print("niter mean gpu", got["solver_niter"].mean(), "oracle", ref["solver_niter"].mean(),
        "differs", int((got["solver_niter"] != ref["solver_niter"]).sum()))
