#!/bin/bash
# Env-step A/B: the tree's library vs variant libraries, plain bench lines (no CPU
# baseline), alternated twice; then the GPU suite.  usage: bash tools/gpu_envab.sh <tag> [lib ...]
set -e
TAG=${1:-envab}; shift
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for P in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > $O/tree_$P.log 2>&1 || { tail -20 $O/tree_$P.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('$O/tree_$P.log') if l.startswith('{')][0]); print('tree', d['value'], d['ms_per_step'])"
  for L in "$@"; do
    MJH_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > $O/var_$P.log 2>&1 || { tail -20 $O/var_$P.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$O/var_$P.log') if l.startswith('{')][0]); print('$L', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
