"""Ordered kernel dispatches of one steady-state env step from a rocprofv3
--kernel-trace CSV (diagnostic tool): name, duration and the gap before each.

usage: python tools/trace_order.py <kernel_trace.csv> [decimation]
The env step is delimited by every `decimation`-th physics step launch
(step_kernel<..., true, 0>); the second-to-last complete one is printed.
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
dec = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda x: x[0])


def short(n):
  n = n.replace("(anonymous namespace)::", "").replace("void ", "")
  n = re.sub(r"at::native::", "", n)
  return n.split("(")[0][:90]


# physics step launches: the fused step kernel whose forward flag is a runtime
# argument; the gated forward follows the env layer's resets, so an env step
# starts at the first of `dec` consecutive step launches after the previous forward
steps = [i for i, k in enumerate(ks) if "step_kernel" in k[2]]
firsts = []
i = 0
while i < len(steps):
  j = i
  while j + 1 < len(steps) and steps[j + 1] - steps[j] <= 2:
    j += 1
  if j - i + 1 >= dec:
    firsts.append(steps[i])
  i = j + 1
if len(firsts) < 3:
  sys.exit("not enough env steps in the trace")
a, b = firsts[-3], firsts[-2]
# include the pack launch before the first physics launch
while a > 0 and "pack_kernel" in ks[a - 1][2]:
  a -= 1
while b > 0 and "pack_kernel" in ks[b - 1][2]:
  b -= 1
prev_end = ks[a][0]
tot_gap = tot_k = 0.0
print(f"{'#':>3} {'dur us':>8} {'gap us':>7}  kernel")
for n, (s, e, name) in enumerate(ks[a:b]):
  gap = (s - prev_end) / 1e3
  print(f"{n:3d} {(e - s) / 1e3:8.2f} {gap:7.2f}  {short(name)}")
  tot_gap += max(gap, 0.0)
  tot_k += (e - s) / 1e3
  prev_end = e
print(f"{b - a} dispatches, kernel time {tot_k:.1f} us, gaps {tot_gap:.1f} us, wall {(ks[b][0] - ks[a][0]) / 1e3:.1f} us")
