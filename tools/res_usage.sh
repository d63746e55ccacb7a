#!/bin/bash
# Register / scratch / spill summary of the step-kernel instances (device-only compile, no GPU).
# usage: bash tools/res_usage.sh [extra hipcc flags...]
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -c -o /dev/null \
  -Rpass-analysis=kernel-resource-usage "$@" asimov-mjlab_amd/csrc/mjh_step.hip 2>&1 |
python3 -c '
import re, sys
txt = sys.stdin.read()
for b in re.split(r"remark: Function Name: ", txt)[1:]:
  name = b.split()[0]
  if "step_kernel" not in name:
    continue
  g = lambda k: (re.search(k + r": (\d+)", b) or [None, "?"])[1]
  inst = re.search(r"step_kernelILi(\d+)ELi(\d+)ELi?(n?\d+)ELb(\d)ELi(\d)", name)
  print("step_kernel<%s,%s,%s,%s,%s>" % inst.groups(), "VGPR", g("VGPRs"), "scratch", g(r"ScratchSize \[bytes/lane\]"),
        "waves", g(r"Occupancy \[waves/SIMD\]"), "VGPRspill", g("VGPRs Spill"), "SGPRspill", g("SGPRs Spill"))
'
