"""numpy restatement of the env layer's device random stream (TEST INFRASTRUCTURE).

Follows ``asimov-mjlab_amd/csrc/mjh_rng.h`` (``mjh::Rng``): element ``idx`` of
the U[0, 1) draw keyed (seed, key, step) is a splitmix64 finalizer chain, 24
random bits per float. The fixture generators (tools/make_golden_events.py)
use it to hand the reference's functions exactly the draws the fused HIP
kernels consume; the GPU tests check it against ``mjh_uniform_draws``.
"""

from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def _mix64_int(z: int) -> int:
  z &= M64
  z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
  z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
  return z ^ (z >> 31)


def _mix64_arr(z: np.ndarray) -> np.ndarray:
  z = z.astype(np.uint64)
  with np.errstate(over="ignore"):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
  return z ^ (z >> np.uint64(31))


def base(seed: int, key: int, step: int) -> int:
  return _mix64_int(seed ^ _mix64_int(key ^ _mix64_int(step + GOLDEN)))


def u01(seed: int, key: int, step: int, idx) -> np.ndarray:
  """float32 draws for element indices ``idx`` (any integer array shape)."""
  b = np.uint64(base(seed, key, step))
  i = np.asarray(idx, dtype=np.uint64)
  with np.errstate(over="ignore"):
    z = b + (i + np.uint64(1)) * np.uint64(GOLDEN)
  return ((_mix64_arr(z) >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)).astype(np.float32)


def site_hash(site: str) -> int:
  """FNV-1a of the call-site name (mjlab_amd.envops._site_hash)."""
  h = 1469598103934665603
  for ch in site.encode():
    h = ((h ^ ch) * 1099511628211) & M64
  return h


def site_key(site: str, salt: int) -> int:
  """Key of the ``salt``-th rng_args call of an env (mjlab_amd.envops.rng_args)."""
  return (site_hash(site) ^ (salt * GOLDEN)) & M64
