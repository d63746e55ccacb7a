#!/bin/bash
# A/B of the tree's library vs variants on G1 4096 and Go1 8192, then GPU suite and bench.
# usage: bash tools/gpu_r03t.sh <tag> [lib ...]
set -e
TAG=${1:-r03t}; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
t() { echo "[$(date +%T)] $*"; }
t ab
for P in 1 2; do
  for T in Mjlab-Velocity-Flat-Unitree-G1 Mjlab-Velocity-Flat-Unitree-Go1; do
    N=4096; [ "$T" = Mjlab-Velocity-Flat-Unitree-Go1 ] && N=8192
    MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py $N 40 $T >> $O/kb.log 2>&1
    for L in "$@"; do
      MJH_BALANCE=1 MJH_LIB=$L timeout -k 10 120 python tools/kernel_bench.py $N 40 $T >> $O/kb.log 2>&1
    done
  done
done
grep "ms/launch" $O/kb.log
[ "${AB_ONLY:-0}" = 1 ] && exit 0
t tests
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
t bench
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log
if [ "${PHASE:-0}" = 1 ]; then
  t phase
  timeout -k 10 180 python tools/phase_profile.py 4096 > $O/phase.log 2>&1 || { tail -20 $O/phase.log; exit 1; }
  tail -25 $O/phase.log
fi
t done
