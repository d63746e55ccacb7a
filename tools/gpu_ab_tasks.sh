#!/bin/bash
# Same-box A/B of step-library builds on the G1 (4096 worlds) and Go1 (8192 worlds)
# kernel benches, two interleaved passes each. usage: bash tools/gpu_ab_tasks.sh <tag> <lib.so>...
set -e
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for R in 1 2; do
  for L in "$@"; do
    MJH_LIB=$L MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py 4096 40 >> $O/kb.log 2>&1
    tail -n 1 $O/kb.log
    MJH_LIB=$L MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py 8192 40 Mjlab-Velocity-Flat-Unitree-Go1 >> $O/kb.log 2>&1
    tail -n 1 $O/kb.log
  done
done
