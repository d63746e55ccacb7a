#!/bin/bash
# round-3 checks: parity on the default build (both line searches), the split
# build's suites, then A/B kernel timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r03g
mkdir -p $O

timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/tests_base.log 2>&1 && \
MJH_LIB=asimov-mjlab_amd/mjlab_amd/variants/libmjh_split.so timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_env.py > $O/tests_split.log 2>&1 && \
bash tools/gpu_variants.sh r03g split p4 p4s
