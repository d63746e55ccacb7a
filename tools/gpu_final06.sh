#!/bin/bash
# Round-6 end-of-round GPU pass (repo root on the box), in two calls:
#   STAGE=a: GPU tests (the launch-plugin speed test printed), smoke(), the three bench
#            configs and the rocprofv3 --kernel-trace --stats run of the default command;
#   STAGE=b: PMC traffic (FETCH_SIZE, WRITE_SIZE passes), SQ counters, phase profile, and the
#            split build's solver launch (north-star figure).
# usage: STAGE=a|b bash tools/gpu_final06.sh <tag>
set -e
TAG=${1:-r06fin}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
t() { echo "[$(date +%T)] $*"; }
if [ "${STAGE:-a}" = a ]; then
  t tests
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
  grep -E "PARITY TOTAL|passed|failed" $O/gputests.log | tail -3
  t plugin speed
  timeout -k 10 300 python -u -m pytest tests/test_gpu_jit.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/jit.log 2>&1 || { tail -30 $O/jit.log; exit 1; }
  grep -h "plugin speed\|plugin parity" $O/jit.log
  t smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -n 2 $O/smoke.log
  t default bench
  timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
  grep '^{' $O/bench_default.log
  bash tools/gpu_bench3.sh $TAG
else
  t pmc traffic
  MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf -o f -- python tools/kernel_bench.py 4096 40 > $O/pmcf.log 2>&1
  MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o w -- python tools/kernel_bench.py 4096 40 > $O/pmcw.log 2>&1
  python tools/pmc_traffic.py $(find $O/pmcf -name '*counter_collection.csv') $(find $O/pmcw -name '*counter_collection.csv') 4096 > $O/step_kernel_traffic.json
  cat $O/step_kernel_traffic.json
  find $O/pmcf $O/pmcw -name '*.csv' -delete
  t sq
  bash tools/gpu_pmc_sq.sh $TAG
  t phase
  timeout -k 10 200 python -u tools/phase_profile.py 4096 > $O/phase_4096.log 2>&1
  head -14 $O/phase_4096.log
  t solver
  bash tools/gpu_solver_pmc.sh $TAG
fi
t done
