"""Why the float32 solve iterates more than the float64 oracle.

usage: python tools/iteration_analysis.py [n]      (CPU only: the oracle, both precisions)

The device's mean Newton iteration count equals the float32 oracle's (GPU test
ITERATIONS lines: G1 6.02 vs float32 6.0, float64 5.15; Go1 4.26 vs 4.2, float64 3.22).
MuJoCo's stop test is  improvement < tol  or  gradient < tol  (both scaled by
1 / (meaninertia nv), tol = 1e-8, the reference's sim.py:57). The gradient,
Ma - qfrc_smooth - qfrc_constraint, cancels terms of magnitude |Ma| + |qfrc_smooth| +
|qfrc_constraint|: in float32 its rounding floor is ~eps32 times that magnitude, which
lies above the tolerance in (nearly) every world, so a float32 solver cannot stop by
the gradient test; it stops by the improvement test, which the float32 cost difference
passes one iteration after convergence (the difference rounds to 0). The float64 solver
stops by the gradient test at the converged iterate itself. Prediction: the float64
oracle with the gradient test switched off (oracle_set_stop_mode(1)) iterates as often as
the float32 one. This prints, per model: the mean iterations of float64, float64 with the
improvement test only, and float32; the share of float64 stops decided by the gradient
test; and the share of those whose float32 gradient floor exceeds the tolerance.
"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
sys.path.insert(0, str(ROOT))
from oracle.oracle import Oracle  # noqa: E402
from tests.scenes import g1_scene_model, go1_scene_model, random_states  # noqa: E402

EPS32 = float(np.finfo(np.float32).eps)


def analyse(name: str, m, n: int, seed: int = 1) -> dict:
  from mjlab_amd.sim import MujocoCfg

  MujocoCfg(timestep=0.005, iterations=10, ls_iterations=20).apply(m)  # the GPU parity tests' options
  st = random_states(m, n, np.random.default_rng(seed))
  o64 = Oracle(m, "f64")
  r64 = o64.run(n, st, integrate=True, nthreads=8)
  o64.lib.oracle_set_stop_mode.argtypes = [ctypes.c_int]
  o64.lib.oracle_set_stop_mode(1)
  try:
    r64i = o64.run(n, st, integrate=True, nthreads=8)
  finally:
    o64.lib.oracle_set_stop_mode(0)
  r32 = Oracle(m, "f32").run(n, st, integrate=True, nthreads=8)
  tol = r64["solver_opt"]["tolerance"]
  nit = r64["solver_niter"][:, 0]
  conv = r64["solver_conv"]  # (n, 15, 4): improvement, gradient, |cost| scale, gradient-term scale
  by_grad = floor_above = stopped = 0
  for w in range(n):
    k = int(nit[w]) - 1
    if k < 0 or k >= 15 or r64["solver_capped"][w, 0]:
      continue
    impr, grad, _, gmag = conv[w, k]
    stopped += 1
    if not impr < tol and grad < tol:
      by_grad += 1
      floor_above += int(EPS32 * gmag > tol)
  res = {"model": name, "worlds": n, "f64": float(nit.mean()), "f64_improvement_only": float(r64i["solver_niter"][:, 0].mean()),
         "f32": float(r32["solver_niter"][:, 0].mean()), "f64_stops": stopped, "f64_stops_by_gradient": by_grad,
         "of_which_f32_gradient_floor_above_tol": floor_above,
         "f32_floor_above_tol_all_iters": float((EPS32 * conv[:, :, 3] > tol)[~np.isnan(conv[:, :, 3])].mean())}
  return res


def main() -> None:
  n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
  for name, fn in (("G1", g1_scene_model), ("Go1", go1_scene_model)):
    r = analyse(name, fn(n), n)
    print(f"{r['model']:4s} worlds {r['worlds']}: mean iterations float64 {r['f64']:.2f}, float64 with the improvement "
          f"test only {r['f64_improvement_only']:.2f}, float32 {r['f32']:.2f}; float64 stops by the gradient test "
          f"{r['f64_stops_by_gradient']}/{r['f64_stops']}, of which the float32 gradient floor (eps32 x |terms|) exceeds "
          f"the tolerance in {r['of_which_f32_gradient_floor_above_tol']}; floor above tolerance at "
          f"{100 * r['f32_floor_above_tol_all_iters']:.1f} % of all iterations")


if __name__ == "__main__":
  main()
