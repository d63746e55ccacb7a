#!/bin/bash
# Env-bench A/B of step-library builds (in-tree and variants), two passes, plus
# the rows-in-global-scratch bitwise test per variant.
# usage (repo root on the GPU box): bash tools/gpu_libab.sh <tag> <variant>...
TAG=${1:-libab}; shift
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$TAG
mkdir -p $O
set -e
LIBS="asimov-mjlab_amd/mjlab_amd/libmjh.so"
for V in "$@"; do LIBS="$LIBS asimov-mjlab_amd/mjlab_amd/variants/libmjh_$V.so"; done
for R in 1 2; do
  for L in $LIBS; do
    MJH_LIB=$L timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/b.log 2>&1
    python - "$L" $O/b.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
c = j["config"]
print(f"{sys.argv[1].split('/')[-1]:22s} {j['value']:12,.0f} env-steps/s  {j['ms_per_step']:.3f} ms/step  "
      f"launch {j['roofline']['launch_us']:.1f} us  overflow {c['efc_overflow_worlds']}  nefc {c['mean_nefc']:.1f}")
PY
  done
done | tee $O/libab.log
for V in "$@"; do
  MJH_LIB=asimov-mjlab_amd/mjlab_amd/variants/libmjh_$V.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -s \
    -k bit_identical > $O/bit_$V.log 2>&1 || true
  echo "$V: $(grep -E 'rows in global|passed|failed' $O/bit_$V.log | tr '\n' ' ')"
done
