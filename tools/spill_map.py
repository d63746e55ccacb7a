"""Where a kernel instance's private-scratch (spill) traffic sits in the source.

usage: python tools/spill_map.py <device.s> <kernel-symbol-substring> [top]
The .s comes from `hipcc --cuda-device-only -S -gline-tables-only` of mjh_step.hip.
Counts scratch loads / stores (VGPR spills and private arrays) and v_readlane /
v_writelane (SGPR spills to VGPR lanes go through v_writelane/v_readlane too) per
source line (.loc), and prints the lines with the most scratch traffic.
"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
files, loc = {}, (0, 0)
st, ld = collections.Counter(), collections.Counter()
inside = False
name = None
with open(path) as f:
  for line in f:
    if line.startswith("\t.file"):
      m = re.match(r'\t\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
      if m:
        files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
      continue
    if not inside:
      head = line.split(";")[0].rstrip()
      if head.endswith(":") and sym in head and not line.startswith("\t") and not line.startswith("."):
        inside, name = True, head[:-1]
      continue
    if line.startswith(".Lfunc_end"):
      break
    s = line.strip()
    if s.startswith(".loc"):
      # the mjh_step.hip lines of the inline chain: innermost and outermost (kernel body)
      hits = re.findall(r"mjh_step\.hip:(\d+)", s)
      loc = (int(hits[0]), int(hits[-1])) if hits else (0, 0)
      continue
    if s.startswith("scratch_store") or (s.startswith("buffer_store") and "off, s[0:3]" in s):
      st[loc] += 1
    elif s.startswith("scratch_load") or (s.startswith("buffer_load") and "off, s[0:3]" in s):
      ld[loc] += 1
print("kernel:", name)
print(f"static scratch stores {sum(st.values())}, loads {sum(ld.values())}")
tot = collections.Counter()
for k in set(st) | set(ld):
  tot[k] = st[k] + ld[k]
for (inner, outer), n in tot.most_common(top):
  print(f"mjh_step.hip:{inner:<5d} (in body line {outer:<5d})  stores {st[(inner, outer)]:4d}  loads {ld[(inner, outer)]:4d}")
by_outer = collections.Counter()
for (inner, outer), n in tot.items():
  by_outer[outer // 50 * 50] += n
print("by 50-line block of the kernel body:")
for blk, n in sorted(by_outer.items()):
  print(f"  {blk:5d}-{blk + 49:5d}: {n}")
