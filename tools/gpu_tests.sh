#!/bin/bash
# GPU parity suite (+ optional extra pytest args) with a per-step time limit.
# usage (repo root on the GPU box): bash tools/gpu_tests.sh <tag> [pytest args...]
TAG=${1:-t}; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread "$@" > $O/gputests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|parity|passed|failed" $O/gputests.log | tail -60
exit $rc
