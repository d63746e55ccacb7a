#!/bin/bash
# A/B: parallel vs exact line search, step kernel alone (G1 4096, Go1 8192), twice each
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-lsab}
mkdir -p $O
set -e
for rep in 1 2; do
  for LS in 1 0; do
    MJH_BALANCE=1 MJH_LS_PARALLEL=$LS timeout -k 10 120 python tools/kernel_bench.py 4096 40 >> $O/kb.log 2>&1
    MJH_BALANCE=1 MJH_LS_PARALLEL=$LS timeout -k 10 120 python tools/kernel_bench.py 8192 40 Mjlab-Velocity-Flat-Unitree-Go1 >> $O/kb.log 2>&1
  done
done
grep "ms/launch" $O/kb.log
