#!/bin/bash
# Kernel trace of a short G1 bench and the ordered dispatches of one env step.
# usage (repo root on the box): bash tools/gpu_trace.sh <tag> [task]
set -e
TAG=${1:-trace}
T=${2:-Mjlab-Velocity-Flat-Unitree-G1}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python bench.py --task $T --steps 30 --warmup 5 --settle 60 --no-cpu-baseline > $O/trace_bench.log 2>&1
F=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python tools/trace_order.py $F > $O/trace_order.txt
python tools/trace_summary.py $F 20 > $O/trace_summary.txt
tail -3 $O/trace_order.txt
find $O/kt -name '*.csv' -delete
