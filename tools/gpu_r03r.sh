#!/bin/bash
# Fresh-box pass: step-kernel A/B (variant libs vs the tree's), GPU suite, SQ counters
# (roofline_valu input), plain bench.  usage: bash tools/gpu_r03r.sh <tag> [lib ...]
set -e
TAG=${1:-r03r}; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
t() { echo "[$(date +%T)] $*"; }
t ab
for P in 1 2; do
  MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py 4096 40 >> $O/kb.log 2>&1
  for L in "$@"; do
    MJH_BALANCE=1 MJH_LIB=$L timeout -k 10 120 python tools/kernel_bench.py 4096 40 >> $O/kb.log 2>&1
  done
done
grep "ms/launch" $O/kb.log
[ "${AB_ONLY:-0}" = 1 ] && exit 0
t tests
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
if [ "${SQ:-1}" = 1 ]; then
  t sq
  bash tools/gpu_pmc_sq.sh ${TAG}_sq 4096 > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
  tail -3 $O/sq.log
  cp gpurun_out/${TAG}_sq/step_kernel_sq.json profiles/step_kernel_sq.json
fi
t bench
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
t done
