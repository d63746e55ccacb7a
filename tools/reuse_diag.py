"""Diagnostics: position reuse on/off on the mocap scene, per-world differences."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import numpy as np  # noqa: E402

from tests.scenes import g1_mocap_scene, mocap_states  # noqa: E402
from tests.test_gpu_parity import get, put  # noqa: E402
from tests.test_gpu_reuse import _make  # noqa: E402

n = 32
m = g1_mocap_scene(n).compile(50, 300)
st = mocap_states(m, n, np.random.default_rng(13))
on, off = _make(m, n, True), _make(m, n, False)
for s in (on, off):
  put(s, st)
for tag, edit in (("forward+step", False), ("forward+mocap edit+step", True)):
  for s in (on, off):
    s.forward()
    if edit:
      s.data.mocap_pos[::2] += 0.01
    s.step()
  a, b = get(on, n), get(off, n)
  for k in ("qpos", "qvel", "qacc", "ncon", "nefc", "geom_xpos", "efc_aref", "efc_D", "sensordata", "qfrc_constraint"):
    d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64)).max(1)
    print(tag, k, "worlds differing:", np.nonzero(d)[0].tolist()[:12], "max", d.max())
