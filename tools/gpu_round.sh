#!/bin/bash
# One GPU-box pass: parity tests, env-step breakdown, profiled bench, PMC traffic.
# usage (from the repo root on the box): bash tools/gpu_round.sh <tag>
# Large per-dispatch traces are reduced on the box (gpurun copies back <= 64 MiB).
set -e
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
t() { echo "[$(date +%T)] $*"; }
if [ -n "$DIAG" ]; then timeout -k 10 120 python $DIAG > $O/diag.log 2>&1; tail -30 $O/diag.log; fi
if [ -n "$PHASE" ]; then
  t phase
  timeout -k 10 180 python tools/phase_profile.py 4096 > $O/phase.log 2>&1 || { tail -20 $O/phase.log; exit 1; }
  tail -40 $O/phase.log
fi
t tests
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
t breakdown
timeout -k 10 240 python tools/env_breakdown.py > $O/eb.log 2>&1 || { tail -20 $O/eb.log; exit 1; }
cat $O/eb.log
t bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
find $O/prof -name '*kernel_trace.csv' -delete
if [ "${PMC:-1}" = 1 ]; then
  t pmc
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf -o f -- python tools/kernel_bench.py 4096 40 > $O/pmcf.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o w -- python tools/kernel_bench.py 4096 40 > $O/pmcw.log 2>&1
  python tools/pmc_traffic.py $(find $O/pmcf -name '*counter_collection.csv') $(find $O/pmcw -name '*counter_collection.csv') 4096 > $O/step_kernel_traffic.json
  cat $O/step_kernel_traffic.json
  # keep the per-dispatch counter rows of the step kernel (the JSON's evidence)
  for P in pmcf pmcw; do
    F=$(find $O/$P -name '*counter_collection.csv' | head -1)
    { head -1 $F; grep 'step_kernel' $F || true; } > $O/${P}_step_kernel_rows.csv
  done
  find $O/pmcf $O/pmcw -name '*.csv' -delete
fi
du -sh $O
t done
