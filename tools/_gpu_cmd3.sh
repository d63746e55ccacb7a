set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r05x}
O=gpurun_out/$T
mkdir -p $O
TESTS=1 bash tools/gpu_r05.sh $T
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo "[$(date +%T)] default bench"
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log
bash tools/gpu_bench3.sh $T
