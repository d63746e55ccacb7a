"""Diagnostics (profile build, MJH_LIB=.../libmjh_prof.so): the step-size index
the parallel line search picks at each solver iteration, HIP vs oracle, for the
worlds whose solver outputs differ most (G1, 256 worlds, parity-test seed)."""
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
buf = torch.zeros(n * 32, dtype=torch.int64, device="cuda:0")
L = native.lib()
L.mjh_set_profile_buffer.argtypes = [ctypes.c_void_p]
assert L.mjh_set_profile_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
m = g1_scene_model(n)
st = random_states(m, n, np.random.default_rng(1))
sim = make_sim(m, n, ls_parallel=True)
put(sim, st)
buf.zero_()
sim.step()
got = get(sim, n)
tr = buf.view(n, 32)[:, 30].cpu().numpy()
ref = Oracle(m).run(n, st, integrate=True)
f32 = Oracle(m, "f32").run(n, st, integrate=True)


def dec(x, k):
  return [int((int(x) >> (5 * i)) & 31) for i in range(k)]


d = np.abs(got["efc_force"] - ref["efc_force"]).max(1) / (1 + np.abs(ref["efc_force"]).max(1))
same = sum(dec(tr[w], 10)[: ref["solver_niter"][w, 0]] == dec(ref["ls_trace"][w, 0], 10)[: ref["solver_niter"][w, 0]]
           for w in range(n))
print("worlds whose chosen step sizes match the oracle's over its iterations:", same, "/", n)
for w in np.argsort(-d)[:6]:
  print(f"world {w} rel {d[w]:.4f} niter gpu {got['solver_niter'][w, 0]} f64 {ref['solver_niter'][w, 0]} "
        f"f32 {f32['solver_niter'][w, 0]} nefc {ref['nefc'][w, 0]} gap {ref['ls_gap'][w, 0]:.3e}")
  print("   gpu", dec(tr[w], 10))
  print("   f64", dec(ref["ls_trace"][w, 0], 10))
  print("   f32", dec(f32["ls_trace"][w, 0], 10))
