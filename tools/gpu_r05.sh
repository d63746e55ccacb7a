#!/bin/bash
# Round-5 GPU pass (repo root on the box): selected stages, each under its own time limit.
# usage: TESTS=1|k-expr BENCH="20 300" VARIANTS="v1 v2" PROF=0|1 bash tools/gpu_r05.sh <tag>
set -e
TAG=${1:-r05}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
t() { echo "[$(date +%T)] $*"; }
if [ -n "$TESTS" ]; then
  t tests
  K=(); [ "$TESTS" != 1 ] && K=(-k "$TESTS")
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${K[@]}" > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
  grep -E "PARITY TOTAL|passed|failed" $O/gputests.log | tail -4
fi
for S in $BENCH; do
  t bench $S
  timeout -k 10 400 python -u bench.py --steps $S --warmup 5 --no-cpu-baseline > $O/bench$S.log 2>&1 || { tail -30 $O/bench$S.log; exit 1; }
  grep '^{' $O/bench$S.log
done
if [ -n "$VARIANTS" ]; then
  t variants
  bash tools/gpu_variants.sh $TAG $VARIANTS
fi
if [ "${PROF:-0}" = 1 ]; then
  t rocprof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 300 --no-cpu-baseline > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
  grep '^{' $O/bench_prof.log
  find $O/prof -name '*kernel_trace.csv' -delete
fi
t done
