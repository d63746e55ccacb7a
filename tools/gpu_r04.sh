#!/bin/bash
# Round-4 occupancy study on the GPU box: the GPU suite, kernel-only and env-bench
# A/B of the worlds-per-CU variants, and per-world phase profiles (8 vs 16 per CU).
# usage (repo root on the box): bash tools/gpu_r04.sh <tag>
TAG=${1:-r04}
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
grep -E "^E |FAILED|ERROR|passed|failed|PARITY|\[cg|box pairs" $O/gputests.log | tail -25
set -e
for V in prof8 prof16; do
  MJH_LIB=asimov-mjlab_amd/mjlab_amd/variants/libmjh_$V.so timeout -k 10 150 python tools/phase_profile.py 4096 > $O/phase_$V.log 2>&1
  echo "== $V"; head -3 $O/phase_$V.log
done
bash tools/gpu_variants.sh $TAG big16 big12 go16
bash tools/gpu_libab.sh ${TAG}b big16 big12
