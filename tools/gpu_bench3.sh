#!/bin/bash
# Steady-state bench lines for the three single-GPU configs (G1 4096, Go1 8192,
# tracking 4096) plus a rocprofv3 --stats run of the G1 headline command.
# usage (repo root on the GPU box): bash tools/gpu_bench3.sh <tag> [steps]
set -e
TAG=${1:-b3}
K=${2:-300}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
t() { echo "[$(date +%T)] $*"; }
for T in Mjlab-Velocity-Flat-Unitree-G1 Mjlab-Velocity-Flat-Unitree-Go1 Mjlab-Tracking-Flat-Unitree-G1; do
  t bench $T
  timeout -k 10 300 python -u bench.py --task $T --steps $K --warmup 20 --cpu-seconds 4 > $O/bench_$T.log 2>&1 || { tail -30 $O/bench_$T.log; exit 1; }
  grep '^{' $O/bench_$T.log
done
if [ "${PROF:-1}" = 1 ]; then
  t rocprof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps $K --no-cpu-baseline > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
  grep '^{' $O/bench_prof.log
  find $O/prof -name '*kernel_trace.csv' -delete
fi
t done
