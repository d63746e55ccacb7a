#!/bin/bash
# Same-box A/B of step-library builds: kernel_bench G1 4096 (two passes each), then
# a short env bench per library. usage: bash tools/gpu_ab06.sh <tag> <lib.so>...
set -e
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for R in 1 2; do
  for L in "$@"; do
    MJH_LIB=$L MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py 4096 40 >> $O/kb.log 2>&1
    tail -1 $O/kb.log
  done
done
for L in "$@"; do
  MJH_LIB=$L timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1
  python - "$L" $O/b.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
print(f"{sys.argv[1].split('/')[-1]:24s} {j['value']:12,.0f} env-steps/s  {j['ms_per_step']:.3f} ms/step  launch {j['roofline']['launch_us']:.1f} us")
PY
done
