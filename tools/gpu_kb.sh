#!/bin/bash
# Kernel-only A/B timing: specialised vs generic step instance (+ optional
# extra library variants). usage: bash tools/gpu_kb.sh <tag> [lib ...]
TAG=${1:-kb}; shift
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$TAG
mkdir -p $O
set -e
for T in Mjlab-Velocity-Flat-Unitree-G1 Mjlab-Velocity-Flat-Unitree-Go1; do
  N=4096; [ "$T" = Mjlab-Velocity-Flat-Unitree-Go1 ] && N=8192
  timeout -k 10 120 python tools/kernel_bench.py $N 40 $T >> $O/kb.log 2>&1
  MJH_SPEC=0 timeout -k 10 120 python tools/kernel_bench.py $N 40 $T >> $O/kb.log 2>&1
  MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py $N 40 $T >> $O/kb.log 2>&1
done
for L in "$@"; do
  MJH_LIB=$L timeout -k 10 120 python tools/kernel_bench.py 4096 40 >> $O/kb.log 2>&1
done
grep "ms/launch" $O/kb.log
