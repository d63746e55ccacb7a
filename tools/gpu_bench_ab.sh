#!/bin/bash
# env-step bench A/B: default library vs variants (G1 velocity 4096), twice each
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-benchab}
shift
mkdir -p $O
set -e
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err
  for V in "$@"; do
    MJH_LIB=asimov-mjlab_amd/mjlab_amd/variants/libmjh_$V.so timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_${V}_$rep.json 2> $O/bench_${V}_$rep.err
  done
done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['launch_us'],1))"; done
