set -e
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05zc
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "rangefinder" > $O/rf.log 2>&1 || { tail -30 $O/rf.log; exit 1; }
tail -1 $O/rf.log
TESTS=1 BENCH=300 bash tools/gpu_r05.sh r05zc
