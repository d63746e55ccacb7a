"""Diagnostics (profile build, MJH_LIB=.../libmjh_prof.so): the parallel line
search's candidate costs at solver iteration 0, HIP vs the float64 oracle, for
the worlds whose first choices differ (G1, 256 worlds, parity-test seed)."""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mjlab_amd.sim import native  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from tests.scenes import g1_scene_model, random_states  # noqa: E402
from tests.test_gpu_parity import get, make_sim, put  # noqa: E402

n = 256
L = native.lib()
buf = torch.zeros(n * 32, dtype=torch.float32, device="cuda:0")
L.mjh_set_lsdbg_buffer.argtypes = [ctypes.c_void_p]
assert L.mjh_set_lsdbg_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
m = g1_scene_model(n)
st = random_states(m, n, np.random.default_rng(1))
sim = make_sim(m, n, ls_parallel=True)
put(sim, st)
buf.zero_()
sim.step()
got = get(sim, n)
gc = buf.view(n, 32).cpu().numpy()[:, :20]
orc = Oracle(m)
oc = np.zeros((n, 64))
orc.lib.oracle_set_lscost.argtypes = [ctypes.c_void_p, ctypes.c_int]
orc.lib.oracle_set_lscost(oc.ctypes.data, 0)
ref = orc.run(n, st, integrate=True, follow=got)
orc.lib.oracle_set_lscost(None, 0)
oc = oc[:, :20]
g0 = got["solver_lstrace"][:, 0] & 63
r0 = np.argmin(oc, axis=1)
diff = np.nonzero((g0 != r0) & (got["nefc"][:, 0] > 0))[0]
print("worlds whose first step-size choice differs:", len(diff), "of", int((got["nefc"][:, 0] > 0).sum()))
rel = np.abs(gc - oc).max(1) / (1e-9 + np.abs(oc).max(1))
print("candidate-cost max rel diff over worlds: median", np.median(rel), "max", rel.max(), "world", int(np.argmax(rel)))
for w in list(diff[:4]) + [int(np.argmax(rel))]:
  print(f"world {w} gpu choice {g0[w]} oracle argmin {r0[w]} nefc {got['nefc'][w, 0]}")
  print("   gpu   ", np.array2string(gc[w], precision=6, max_line_width=250))
  print("   oracle", np.array2string(oc[w], precision=6, max_line_width=250))
