"""Per-world GPU-vs-oracle diagnostics for one configuration (diagnostic tool)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd")); sys.path.insert(0, str(ROOT))
import numpy as np, torch
from tests.test_gpu_parity import make_sim, put, get, DEV
from tests.scenes import g1_scene_model, random_states, compare_step
from oracle.oracle import Oracle

n = 128
m = g1_scene_model(n)
sim = make_sim(m, n, expand=("geom_friction",))
rng = np.random.default_rng(3)
fr = sim.model.geom_friction
mode = sys.argv[1] if len(sys.argv) > 1 else "rand"
if mode == "rand":
  fr[:, :, 0] = torch.as_tensor(rng.uniform(0.3, 1.2, (n, fr.shape[1])), dtype=torch.float32, device=DEV)
else:
  rng.uniform(0.3, 1.2, (n, fr.shape[1]))
st = random_states(m, n, rng)
put(sim, st)
sim.step()
got = get(sim, n)
ref = Oracle(m, overrides={"geom_friction": fr.cpu().numpy()}).run(n, st, integrate=True)
rep = compare_step(got, ref)
print(mode, rep["failures"], rep["int_mismatch_worlds"])
e = np.abs(got["qacc"] - ref["qacc"]).max(axis=1)
for w in np.argsort(-e)[:8]:
  print(w, f"err {e[w]:.3e}", "niter", got["solver_niter"][w, 0], ref["solver_niter"][w, 0], "nefc", got["nefc"][w, 0], ref["nefc"][w,0], "ncon", ref["ncon"][w, 0],
        "maxqacc", np.abs(ref["qacc"][w]).max())
print("median err", np.median(e))
