#!/bin/bash
# reuse tests + parity + env tests on the default build, then env bench with position reuse on/off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r03o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reuse.py tests/test_gpu_parity.py tests/test_gpu_env.py > $O/tests.log 2>&1 && \
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_reuse_$rep.json 2> $O/bench_reuse_$rep.err && \
  MJH_POS_REUSE=0 timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_noreuse_$rep.json 2> $O/bench_noreuse_$rep.err || exit 1
done
for f in $O/bench_*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['launch_us'],1))"; done
