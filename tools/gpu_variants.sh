#!/bin/bash
# Kernel-only A/B of step-library variants (tools/build_variant.py), world
# ordering on as in production. usage: bash tools/gpu_variants.sh <tag> <variant>...
TAG=${1:-var}; shift
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$TAG
mkdir -p $O
set -e
for T in Mjlab-Velocity-Flat-Unitree-G1 Mjlab-Velocity-Flat-Unitree-Go1; do
  N=4096; [ "$T" = Mjlab-Velocity-Flat-Unitree-Go1 ] && N=8192
  MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py $N 40 $T >> $O/kb.log 2>&1
  for V in "$@"; do
    MJH_BALANCE=1 MJH_LIB=asimov-mjlab_amd/mjlab_amd/variants/libmjh_$V.so timeout -k 10 120 python tools/kernel_bench.py $N 40 $T >> $O/kb.log 2>&1
  done
done
grep "ms/launch" $O/kb.log
