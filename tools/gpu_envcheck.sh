#!/bin/bash
# Env-layer change check on the GPU box: full GPU test suite, a kernel-trace
# breakdown of the steady-state env step, and the G1 bench line.
# usage (repo root on the box): bash tools/gpu_envcheck.sh <tag> [pytest args]
set -e
TAG=${1:-ec}
shift || true
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gputests.log | tail -30; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o t -- python bench.py --steps 60 --warmup 5 --no-cpu-baseline > $O/trb.log 2>&1
python tools/trace_summary.py $(find $O/tr -name "*kernel_trace.csv") 50 > $O/trace.txt
find $O/tr -name "*.csv" -delete
head -8 $O/trace.txt
timeout -k 10 300 python -u bench.py --cpu-seconds 2 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
