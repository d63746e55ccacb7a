#!/bin/bash
# Step-kernel change check on the GPU box: kernel timing (specialised/generic),
# phase profile (libmjh_prof.so, if built) and the physics parity tests.
# usage (repo root on the box): bash tools/gpu_kcheck.sh <tag>
set -e
TAG=${1:-kc}
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$TAG
mkdir -p $O
bash tools/gpu_kb.sh $TAG "${@:2}"
if [ -f asimov-mjlab_amd/mjlab_amd/libmjh_prof.so ]; then
  timeout -k 10 120 python tools/phase_profile.py 4096 > $O/phase.log 2>&1 || { tail -20 $O/phase.log; exit 1; }
  cat $O/phase.log
fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -3 $O/parity.log
