#!/bin/bash
# One GPU-box pass: parity tests, env-step breakdown, profiled bench, PMC traffic.
# usage (from the repo root on the box): bash tools/gpu_round.sh <tag>
set -e
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -m pytest tests -m gpu -x -q > $O/gputests.log 2>&1
timeout -k 10 240 python tools/env_breakdown.py > $O/eb.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py > $O/bench.log 2>&1
if [ "${PMC:-1}" = 1 ]; then
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf -o f -- python tools/kernel_bench.py 4096 40 > $O/pmcf.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o w -- python tools/kernel_bench.py 4096 40 > $O/pmcw.log 2>&1
fi
echo done
