"""Model-specialised step kernels for any model (launch plugins).

MuJoCo Warp compiles its kernels for whatever model ``put_model`` receives (the
reference's ``Simulation`` puts any scene, ``src/mjlab/sim/sim.py:116-147``). The
library here ships specialised instances for the benchmark models only
(csrc/mjh_spec_table.h); every other model would run the generic instance, whose
addresses and sizes are runtime values (far more registers, spills and private
scratch). This module closes that gap the MI355X way: when a Simulation's launch
plan matches no built-in specialisation, it renders a one-plan table, compiles
``csrc/mjh_step.hip`` with ``-DMJH_PLUGIN`` for gfx950 (hipcc, ~20 s, once per
plan: the library is cached under ``mjlab_amd/_jit/`` keyed by the plan, the
kernel sources and the compile flags) and registers the plugin's launch entry
with the main library (``mjh_register_spec_plugin``). The main library still
packs the model image and orders the worlds; the plugin launches its instance.

Ineligible models (elliptic cones, PGS: the built-in specialisations decline
them too) and non-slab data keep the generic instance. A failed compile keeps
the generic instance and says why (``Simulation.kernel_instance()``), never a
CPU path.
"""

from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
import sys
import time
from pathlib import Path

from mjlab_amd.sim import native
from mjlab_amd.sim.spec_table import layout_ints, plan_of, render

PKG = Path(__file__).resolve().parents[1]
CSRC = PKG.parent / "csrc"
INCLUDE = PKG.parents[1] / "include"
JIT_DIR = Path(os.environ.get("MJH_JIT_DIR", str(PKG / "_jit")))
FLAGS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-DMJH_PLUGIN")
_SOURCES = ("mjh_step.hip", "mjh_math.h", "mjh_convex.h", "mjh_rng.h")
_LOADED: dict[str, ctypes.CDLL] = {}  # plugin libraries stay loaded (their entry points are registered)


def _source_key() -> str:
  """The kernel sources, headers and flags a plugin is compiled from."""
  h = hashlib.sha256()
  h.update(" ".join(FLAGS).encode())
  for name in _SOURCES:
    h.update((CSRC / name).read_bytes())
  for hdr in sorted(INCLUDE.glob("*.h")):
    h.update(hdr.read_bytes())
  return h.hexdigest()[:10]


def _key(plan: list[int]) -> str:
  return hashlib.sha256(" ".join(map(str, plan)).encode()).hexdigest()[:14] + "_" + _source_key()


def plugin_path(plan: list[int]) -> Path:
  return JIT_DIR / f"libmjh_spec_{_key(plan)}.so"


def prune_stale() -> list[Path]:
  """Remove cached plugins compiled from other kernel sources (never loadable again)."""
  cur = _source_key()
  gone = []
  for f in JIT_DIR.glob("libmjh_spec_*"):
    if not f.name.split(".")[0].endswith("_" + cur):
      f.unlink(missing_ok=True)
      gone.append(f)
  return gone


def compile_plugin(plan: list[int], name: str = "model", log=print) -> Path:
  """Build (or find in the cache) the plugin library for one launch plan."""
  out = plugin_path(plan)
  if out.exists():
    return out
  JIT_DIR.mkdir(parents=True, exist_ok=True)
  table = out.with_suffix(".table.h")
  table.write_text(render([plan], [name], layout_ints(native.lib()), origin="mjlab_amd/sim/jit.py"))
  hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
  tmp = out.with_suffix(f".{os.getpid()}.tmp")
  cmd = [hipcc, *FLAGS, f"-I{INCLUDE}", f'-DMJH_SPEC_TABLE="{table}"', "-o", str(tmp), str(CSRC / "mjh_step.hip")]
  t0 = time.time()
  log(f"[mjlab_amd.jit] compiling a specialised step kernel for {name} (plan {out.stem[12:]}) ...")
  r = subprocess.run(cmd, capture_output=True, text=True)
  if r.returncode != 0:
    raise RuntimeError(f"plugin compile failed: {' '.join(cmd)}\n{r.stderr[-4000:]}")
  os.replace(tmp, out)  # atomic: a concurrent builder of the same plan sees a whole file
  log(f"[mjlab_amd.jit] built {out.name} in {time.time() - t0:.0f} s")
  prune_stale()
  return out


def register(path: Path, plan: list[int]) -> int:
  """Load a plugin library, check its ABI and plan, register its launch entry."""
  lib = _LOADED.get(str(path))
  if lib is None:
    lib = ctypes.CDLL(str(path))
    _LOADED[str(path)] = lib
  if lib.mjh_plugin_abi() != native.ABI_VERSION:
    raise RuntimeError(f"{path.name}: plugin ABI {lib.mjh_plugin_abi()} != {native.ABI_VERSION}")
  buf = (ctypes.c_int * len(plan))()
  if lib.mjh_plugin_plan(buf, len(plan)) != len(plan) or list(buf) != plan:
    raise RuntimeError(f"{path.name}: built for another launch plan")
  arr = (ctypes.c_int * len(plan))(*plan)
  fn = ctypes.cast(lib.mjh_plugin_step, ctypes.c_void_p).value
  k = native.lib().mjh_register_spec_plugin(ctypes.c_void_p(fn), arr, len(plan))
  if k < 0:
    raise RuntimeError(native.lib().mjh_last_error().decode())
  return k


def eligible(model) -> bool:
  """The built-in specialisations' conditions (find_spec): pyramidal cones, Newton or CG."""
  return int(getattr(model, "cone", 0)) != 1 and int(getattr(model, "solver", 2)) != 0


def ensure(mstruct_addr: int, model, name: str = "model", compile_missing: bool = True, log=None) -> dict:
  """The kernel instance this model's launches use, building a plugin if needed.

  Returns {"kind": "builtin"|"plugin"|"generic", "index": k, "path": ..., "reason": ...}."""
  log = log or (lambda msg: print(msg, file=sys.stderr, flush=True))
  L = native.lib()
  k = int(L.mjh_spec_index(mstruct_addr))
  if k >= 0:
    return {"kind": "builtin", "index": k}
  if not eligible(model):
    return {"kind": "generic", "index": -1, "reason": "elliptic cones or PGS: generic instances only"}
  plan = plan_of(L, mstruct_addr)
  path = plugin_path(plan)
  if not path.exists():
    if not compile_missing:
      return {"kind": "generic", "index": -1, "reason": f"no plugin built for this plan ({path.name})"}
    try:
      compile_plugin(plan, name, log)
    except Exception as e:  # noqa: BLE001 - the generic instance still runs; say why
      return {"kind": "generic", "index": -1, "reason": str(e)[:400]}
  kp = register(path, plan)
  return {"kind": "plugin", "index": kp, "path": str(path)}
