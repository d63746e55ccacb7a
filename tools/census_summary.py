"""Per-env-step kernel census from a rocprofv3 --stats kernel_stats.csv:
kernels called >= K times, calls/K and µs/step, sorted by time.
usage: python tools/census_summary.py <kernel_stats.csv> <K>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2])
tot_calls = tot_us = 0.0
out = []
for r in rows:
  c = int(r["Calls"])
  if c < K:
    continue
  us = float(r["TotalDurationNs"]) / 1e3 / K
  out.append((us, c / K, float(r["AverageNs"]) / 1e3, r["Name"][:140]))
  tot_calls += c / K
  tot_us += us
out.sort(reverse=True)
print(f"per env step: {tot_calls:.1f} launches, {tot_us:.1f} us kernel time")
for us, cps, avg, name in out:
  print(f"{us:9.1f} us  {cps:6.1f}/step  avg {avg:7.1f} us  {name}")
