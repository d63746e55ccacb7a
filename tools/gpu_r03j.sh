#!/bin/bash
# parity suite on the default build, then line-search A/B and phase profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03j}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_split.py > $O/tests.log 2>&1 && \
bash tools/gpu_ls_ab.sh ${1:-r03j} && \
MJH_LS_PARALLEL=1 timeout -k 10 120 python tools/phase_profile.py 4096 > $O/phase.log 2>&1
