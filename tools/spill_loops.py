"""Spill traffic of one kernel instance by loop depth (static estimate).

usage: python tools/spill_loops.py <device.s> <kernel-symbol-substring>
Loops are the intervals [label, backward branch to it] of the instance's
assembly; an instruction's depth is the number of such intervals around it.
Prints scratch loads / stores per depth and the source lines (inline chain,
innermost mjh_step.hip line) of the spills at depth >= 1.
"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
lines, inside = [], False
with open(path) as f:
  for line in f:
    if not inside:
      head = line.split(";")[0].rstrip()
      if head.endswith(":") and sym in head and not line.startswith("\t") and not line.startswith("."):
        inside = True
      continue
    if line.startswith(".Lfunc_end"):
      break
    lines.append(line.rstrip("\n"))
labels = {}
for i, l in enumerate(lines):
  m = re.match(r"^(\.LBB\w+):", l)
  if m:
    labels[m.group(1)] = i
loops = []
for i, l in enumerate(lines):
  m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\w+)|^\s+s_branch\s+(\.LBB\w+)", l)
  if m:
    t = m.group(1) or m.group(2)
    if t in labels and labels[t] <= i:
      loops.append((labels[t], i))
depth = [0] * len(lines)
for a, b in loops:
  for i in range(a, b + 1):
    depth[i] += 1
loc = 0
by_depth = collections.Counter()
hot = collections.Counter()
for i, l in enumerate(lines):
  s = l.strip()
  if s.startswith(".loc"):
    hits = re.findall(r"mjh_step\.hip:(\d+)", s)
    loc = int(hits[0]) if hits else 0
    continue
  kind = "st" if s.startswith("scratch_store") else ("ld" if s.startswith("scratch_load") else None)
  if kind:
    by_depth[(depth[i], kind)] += 1
    if depth[i] >= 1:
      hot[(loc, depth[i], kind)] += 1
print(f"{len(loops)} loops")
for d in sorted({k[0] for k in by_depth}):
  print(f"depth {d}: loads {by_depth[(d, 'ld')]:4d} stores {by_depth[(d, 'st')]:4d}")
print("spills inside loops (line, depth, kind): count")
for (ln, d, k), n in sorted(hot.items(), key=lambda x: (-x[0][1], -x[1]))[:60]:
  print(f"  mjh_step.hip:{ln:<5d} depth {d} {k}: {n}")
