#!/bin/bash
# Kernel-only A/B of library variants: baseline then each variant, twice, G1 4096 and Go1 8192.
# usage: bash tools/gpu_ab.sh <tag> lib.so ...
TAG=${1:-ab}; shift
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$TAG
mkdir -p $O
set -e
L=asimov-mjlab_amd/mjlab_amd/libmjh.so
for R in 1 2; do
  for V in $L "$@"; do
    MJH_LIB=$V timeout -k 10 120 python tools/kernel_bench.py 4096 40 Mjlab-Velocity-Flat-Unitree-G1 >> $O/kb.log 2>&1
    MJH_LIB=$V timeout -k 10 120 python tools/kernel_bench.py 8192 40 Mjlab-Velocity-Flat-Unitree-Go1 >> $O/kb.log 2>&1
  done
done
grep "ms/launch" $O/kb.log
