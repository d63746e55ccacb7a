#!/bin/bash
# Evidence refresh for the HEAD kernel: SQ counters, PMC traffic, env breakdown, profiled bench.
set -e
TAG=${1:-r03v}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
t() { echo "[$(date +%T)] $*"; }
t sq
bash tools/gpu_pmc_sq.sh ${TAG}_sq 4096 > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
cp gpurun_out/${TAG}_sq/step_kernel_sq.json profiles/step_kernel_sq.json
PMC=1 bash tools/gpu_round.sh $TAG > $O/round.log 2>&1 || { tail -30 $O/round.log; exit 1; }
cp $O/step_kernel_traffic.json profiles/step_kernel_traffic.json
grep -v '^[EW]2026' $O/round.log | tail -30
t done
