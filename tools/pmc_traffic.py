"""Per-launch L2-miss (fabric) traffic of the step kernel from two rocprofv3 --pmc passes.

usage: python tools/pmc_traffic.py fetch.csv write.csv N > profiles/step_kernel_traffic.json
FETCH_SIZE / WRITE_SIZE (kilobytes) count the L2's memory-side requests, which
include Infinity Cache hits (MI355X_MICROARCH.md:297): they are L2-miss fabric
bytes, an upper bound on HBM bytes. The guide's x2 FETCH_SIZE correction
(:298) holds for wide coalesced streaming reads (16 B per lane); the step
kernel's reads are scattered per-world scratch and model-image reads, so
`bytes_per_launch` takes FETCH_SIZE as reported; the x2 figure is given as
`bytes_per_launch_fetch_x2` (upper bound). Only step launches (STEP=true)
after the first 20 (settling) are used.
"""
import csv
import json
import sys


NAMES = set()


def per_dispatch(path, counter):
  vals = {}
  for r in csv.DictReader(open(path)):
    if r["Counter_Name"] != counter or "step_kernel" not in r["Kernel_Name"] or "true" not in r["Kernel_Name"]:
      continue
    NAMES.add(r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0])
    d = int(r["Dispatch_Id"])
    vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
  ks = sorted(vals)
  return [vals[k] for k in ks]


f = per_dispatch(sys.argv[1], "FETCH_SIZE")
w = per_dispatch(sys.argv[2], "WRITE_SIZE")
n = int(sys.argv[3])
f, w = f[20:] or f, w[20:] or w
fetch_kb = sum(f) / len(f)
write_kb = sum(w) / len(w)
out = {
  "num_envs": n,
  "kernel": " + ".join(sorted(NAMES)) + " (G1, settled states, tools/kernel_bench.py)",
  "fetch_size_kb_raw": fetch_kb,
  "write_size_kb": write_kb,
  "bytes_per_launch": (fetch_kb + write_kb) * 1024.0,
  "bytes_per_launch_fetch_x2": (2.0 * fetch_kb + write_kb) * 1024.0,
  "what": "L2-miss fabric bytes per launch (FETCH_SIZE + WRITE_SIZE; Infinity Cache hits included, so an upper "
          "bound on HBM bytes; FETCH_SIZE not doubled: the reads are scattered, not 16-B/lane streaming)",
  "launches": [len(f), len(w)],
}
print(json.dumps(out, indent=1))
