"""The north-star solver figure, measured by counter on the split step (diagnostic tool).

usage: python tools/solver_roofline.py stats.csv fetch.csv write.csv kernel_bench.log N nv > profiles/solver_roofline.json

The split build (MJH_SPLIT=1) runs each physics step as two launches: the
position stage (step_kernel<..., 1>) and the velocity / constraint-solver stage
(step_kernel<..., 2>). This takes the solver launch's average duration from
the rocprofv3 --kernel-trace --stats summary, its L2-miss fabric bytes from
separate FETCH_SIZE / WRITE_SIZE passes (per dispatch, after 20 settling
launches), and the run's mean nefc / solver iterations from kernel_bench.py's
line, and reports against the 8 TB/s HBM peak (MI355X_MICROARCH.md):
* algorithmic: SURVEY.md §8d's streamed-J model
  B_solve = iters * 4 (nefc nv + nv^2 + 6 nefc + 4 nv) + 4 (nefc + 2 nv) per world;
* counter: (FETCH_SIZE + WRITE_SIZE) per launch (an upper bound on HBM bytes:
  Infinity Cache hits included).
"""
import csv
import json
import re
import sys

stats, fetch, write, kb, n, nv = sys.argv[1:7]
n, nv = int(n), int(nv)
HBM = 8000.0


def solver_kernel(name: str) -> bool:
  return "step_kernel" in name and re.search(r",\s*2>\(", name) is not None


t_us = None
for r in csv.DictReader(open(stats)):
  if solver_kernel(r["Name"]):
    t_us = float(r["AverageNs"]) / 1e3
    name = r["Name"].split("(mjh_model")[0].replace("void (anonymous namespace)::", "")


def per_dispatch(path, counter):
  vals = {}
  for r in csv.DictReader(open(path)):
    if r["Counter_Name"] == counter and solver_kernel(r["Kernel_Name"]):
      d = int(r["Dispatch_Id"])
      vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
  v = [vals[k] for k in sorted(vals)]
  v = v[20:] or v
  return sum(v) / max(1, len(v)) * 1024.0, len(v)


fb, nf = per_dispatch(fetch, "FETCH_SIZE")
wb, nw = per_dispatch(write, "WRITE_SIZE")
line = [l for l in open(kb) if "ms/launch" in l][-1]
nefc = float(re.search(r"nefc ([\d.]+)", line).group(1))
iters = float(re.search(r"niter ([\d.]+)", line).group(1))
b_solve = iters * 4 * (nefc * nv + nv * nv + 6 * nefc + 4 * nv) + 4 * (nefc + 2 * nv)
alg = b_solve * n / (t_us * 1e-6) / 1e9
cnt = (fb + wb) / (t_us * 1e-6) / 1e9
print(json.dumps({
  "num_envs": n, "kernel": name, "launch_us": t_us, "mean_nefc": nefc, "mean_iters": iters,
  "b_solve_per_world": b_solve, "algorithmic_gbs": alg, "algorithmic_frac": alg / HBM,
  "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "counter_gbs": cnt, "counter_frac": cnt / HBM,
  "launches": [nf, nw], "peak_gbs": HBM, "task": "Mjlab-Velocity-Flat-Unitree-G1",
  "head": sys.argv[7] if len(sys.argv) > 7 else None,
  "gap": f"40% of 8 TB/s on {b_solve * n / 1e6:.1f} MB is a {b_solve * n / (0.4 * HBM * 1e9) * 1e6:.0f} us launch, "
         f"{t_us / (b_solve * n / (0.4 * HBM * 1e9) * 1e6):.1f}x faster than the measured {t_us:.0f} us: the solver is a "
         "per-world serial chain over an LDS/L2-resident hot set (DESIGN.md §4), not an HBM stream",
  "source": "tools/gpu_solver_pmc.sh: MJH_SPLIT=1 build, tools/kernel_bench.py G1 4096, rocprofv3 --stats + --pmc FETCH_SIZE / WRITE_SIZE",
}, indent=1))
