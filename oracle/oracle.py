"""ctypes driver for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg. Builds the oracle's model/data structs from the same X-macro field list as
the product ABI (mjlab_amd.sim.abi), with float64 (or float32) reals.
"""

from __future__ import annotations

import ctypes
import subprocess
import sys
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
REPO = ORACLE_DIR.parent
sys.path.insert(0, str(REPO / "asimov-mjlab_amd"))

from mjlab_amd.sim import abi  # noqa: E402

# Data fields the caller provides (the step's inputs); the rest are outputs.
INPUTS = ("qpos", "qvel", "act", "qacc_warmstart", "ctrl", "qfrc_applied", "xfrc_applied", "mocap_pos", "mocap_quat", "time")


def build(force: bool = False) -> None:
  libs = [ORACLE_DIR / "liboracle_f64.so", ORACLE_DIR / "liboracle_f32.so"]
  if force or not all(p.exists() for p in libs):
    subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, capture_output=True)


class Oracle:
  def __init__(self, model, precision: str = "f64", overrides: dict | None = None) -> None:
    build()
    self.model = model
    self._overrides = overrides
    self._f32 = None
    self.real = ctypes.c_double if precision == "f64" else ctypes.c_float
    self.dtype = np.float64 if precision == "f64" else np.float32
    self.lib = ctypes.CDLL(str(ORACLE_DIR / f"liboracle_{precision}.so"))
    self.lib.oracle_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    self.lib.oracle_set_debug.argtypes = [ctypes.c_void_p] * 4
    self.lib.oracle_set_follow.argtypes = [ctypes.c_int]
    self.lib.oracle_set_lscost.argtypes = [ctypes.c_void_p, ctypes.c_int]
    self.lib.oracle_set_decisions.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    self.lib.oracle_sizeof_model.restype = ctypes.c_size_t
    self.lib.oracle_sizeof_data.restype = ctypes.c_size_t
    MS = abi.model_struct(self.real, device=False)
    DS = abi.data_struct(self.real, device=False)
    assert ctypes.sizeof(MS) == self.lib.oracle_sizeof_model(), "oracle model struct layout mismatch"
    assert ctypes.sizeof(DS) == self.lib.oracle_sizeof_data(), "oracle data struct layout mismatch"
    self.sizes = abi.model_sizes(model)
    self._keep = []
    ms = MS()
    for k, v in self.sizes.items():
      setattr(ms, k, v)
    for k, v in abi.model_options(model).items():
      setattr(ms, k, v)
    arrays = abi.model_host_arrays(model)
    overrides = overrides or {}
    for f in abi.model_array_fields():
      a = arrays[f.name]
      stride = 0
      if f.name in overrides:
        a = np.asarray(overrides[f.name]).reshape(-1)
        stride = abi.count(f, self.sizes)
      if f.ctype == "float":
        a = a.astype(self.dtype)
      a = np.ascontiguousarray(a)
      self._keep.append(a)
      setattr(ms, f.name, a.ctypes.data)
      if f.kind == "MW":
        setattr(ms, f.name + "_wstride", stride)
    self.ms = ms

  def run(self, nworld: int, state: dict, integrate: bool = True, nthreads: int = 1, debug: bool = False,
          follow: dict | None = None) -> dict:
    """One step (or forward) of `nworld` worlds from `state`. debug=True also
    returns the mass matrix ``qM`` (nworld, nv*nv) and the constraint Jacobian
    ``efc_J`` (nworld, njmax*nv; rows < nefc) of the forward pass. Always
    returned (solver diagnostics, (nworld, 1) each): ``ls_gap``, the smallest
    relative cost gap between the best and the runner-up step size over the
    parallel line searches (inf: none ran); ``solver_capped``, 1 if the solver
    stopped at the iteration cap unconverged (the step-size choices are in
    ``solver_lstrace``). The debug globals are per process: not
    for concurrent run() calls.

    follow: the device's outputs of the same step (``solver_niter``,
    ``solver_lstrace``). Under the parallel line search each world then replays
    the device's discrete choices (iteration count, step-size index per
    iteration) and ``ls_excess`` (nworld, 1) replaces ``ls_gap``: the worst
    relative float64 cost excess of a replayed choice over the argmin. A float64
    follow run also replays the step in the float32 build and returns its
    outputs under ``f32`` — the same algorithm and choices at float32: each
    world's own rounding sensitivity, which the parity checker uses as a floor.

    Also returned: the solver's own decision inputs, evaluated at every
    iteration in follow mode too (the oracle never takes them from the device
    for the check): ``solver_conv`` (nworld, 15, 4) = improvement, gradient
    (both scaled by 1 / (meaninertia nv), the test is ``< tolerance``), the
    scaled cost magnitude |old| + |cost| and the scaled norm of the gradient's
    terms' magnitudes |Ma| + |qfrc_smooth| + |qfrc_constraint| per iteration
    (NaN where none ran), and
    ``warm_costs`` (nworld, 2) = the cost at qacc_warmstart and at qacc_smooth
    (the solve starts from qacc_smooth when the first is larger)."""
    if follow is not None:
      state = dict(state, solver_niter=np.asarray(follow["solver_niter"]).reshape(nworld, -1),
                   solver_lstrace=np.asarray(follow["solver_lstrace"]).reshape(nworld, -1))
    DS = abi.data_struct(self.real, device=False)
    ds = DS()
    ds.nworld = nworld
    out = {}
    for f in abi.data_array_fields():
      n = max(1, abi.count(f, self.sizes))
      dt = self.dtype if f.ctype == "float" else np.int32
      if f.name in state:
        a = np.ascontiguousarray(np.asarray(state[f.name], dtype=dt).reshape(nworld, -1)).copy()
        if a.shape[1] != n and abi.count(f, self.sizes) != 0:
          raise ValueError(f"{f.name}: got {a.shape[1]} per world, expected {n}")
        if a.shape[1] == 0:
          a = np.zeros((nworld, 1), dt)
      else:
        a = np.zeros((nworld, n), dt)
      out[f.name] = a
      setattr(ds, f.name, a.ctypes.data)
    nv, nj = self.sizes["nv"], self.sizes["njmax"]
    out["ls_gap"] = np.zeros((nworld, 1), self.dtype)
    out["ls_trace"] = np.zeros((nworld, 1), np.int64)
    if debug:
      out["qM"] = np.zeros((nworld, nv * nv), self.dtype)
      out["efc_J"] = np.zeros((nworld, nj * nv), self.dtype)
    self.lib.oracle_set_debug(out["qM"].ctypes.data if debug else None, out["efc_J"].ctypes.data if debug else None,
                              out["ls_gap"].ctypes.data, out["ls_trace"].ctypes.data)
    out["solver_conv"] = np.full((nworld, 15, 4), np.nan, self.dtype)
    out["warm_costs"] = np.full((nworld, 2), np.nan, self.dtype)
    self.lib.oracle_set_decisions(out["solver_conv"].ctypes.data, out["warm_costs"].ctypes.data)
    self.lib.oracle_set_follow(1 if follow is not None else 0)
    if follow is not None:  # every candidate cost of every replayed search (the choice check)
      out["ls_costs"] = np.full((nworld, 15, 64), np.nan, self.dtype)
      self.lib.oracle_set_lscost(out["ls_costs"].ctypes.data, -1)
    try:
      rc = self.lib.oracle_run(ctypes.addressof(self.ms), ctypes.addressof(ds), 0, nworld, int(integrate), nthreads)
    finally:
      self.lib.oracle_set_debug(None, None, None, None)
      self.lib.oracle_set_follow(0)
      self.lib.oracle_set_lscost(None, 0)
      self.lib.oracle_set_decisions(None, None)
    if rc != 0:
      raise RuntimeError(f"oracle_run failed: {rc}")
    out["solver_capped"] = out.pop("ls_trace").astype(np.int32)
    out["solver_opt"] = {"tolerance": float(self.ms.tolerance), "iterations": int(self.ms.iterations)}
    if follow is not None and self.ms.ls_parallel:
      out["ls_excess"] = out.pop("ls_gap")
    if follow is not None and self.dtype == np.float64:
      if self._f32 is None:
        self._f32 = Oracle(self.model, "f32", overrides=self._overrides)
      out["f32"] = self._f32.run(nworld, state, integrate=integrate, nthreads=nthreads, follow=follow)
    return out
