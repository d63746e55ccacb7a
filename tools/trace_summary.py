"""Summarise a rocprofv3 --kernel-trace CSV of a bench run (diagnostic tool).

Takes the last K env steps (an env step = 4 physics launches; delimited by
every 4th `step_kernel<..., true, ...>` dispatch) and splits the wall time into
physics, gated forward, env-layer kernel time and inter-kernel gaps.
usage: python tools/trace_summary.py <kernel_trace.csv> [K] [decimation]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dec = int(sys.argv[3]) if len(sys.argv) > 3 else 4
rows = list(csv.DictReader(open(path)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda x: x[0])
steps = [i for i, k in enumerate(ks) if "step_kernel" in k[2] and ", true," in k[2]]
first = steps[::dec]  # first physics launch of each env step
if len(first) < K + 2:
  K = len(first) - 2
a, b = first[-K - 1], first[-1]
win = ks[a:b]
tot = win[-1][0] - win[0][0]
cat = defaultdict(float)
names = defaultdict(lambda: [0, 0.0])
gaps = 0.0
for i, (s, e, n) in enumerate(win):
  d = e - s
  c = "physics" if ("step_kernel" in n and ", true," in n) else "forward" if "step_kernel" in n else "pack" if "pack_kernel" in n else "env"
  cat[c] += d
  if c == "env":
    names[n[:110]][0] += 1
    names[n[:110]][1] += d
  if i + 1 < len(win):
    gaps += max(0, win[i + 1][0] - e)
print(f"{K} env steps: {tot / K / 1e3:.3f} us/step wall, {len(win) / K:.1f} dispatches/step")
gl = defaultdict(lambda: [0, 0.0])
for i in range(len(win) - 1):
  g = win[i + 1][0] - win[i][1]
  if g > 2000:  # > 2 us: attribute the idle time to the (previous -> next) kernel pair
    gl[(win[i][2][:60], win[i + 1][2][:60])][0] += 1
    gl[(win[i][2][:60], win[i + 1][2][:60])][1] += g
big = sorted(gl.items(), key=lambda x: -x[1][1])[:6]
for c, v in sorted(cat.items(), key=lambda x: -x[1]):
  print(f"  {c:8s} {v / K / 1e3:9.1f} us/step")
print(f"  gaps     {gaps / K / 1e3:9.1f} us/step")
for (a, b), (c, g) in big:
  print(f"    gap {g / K / 1e3:7.1f} us/step ({c / K:.1f}/step): {a} -> {b}")
print("env kernels (per step: count, us):")
for n, (c, d) in sorted(names.items(), key=lambda x: -x[1][1])[:40]:
  print(f"  {c / K:5.1f} {d / K / 1e3:8.1f}  {n}")
