set -e
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05w
mkdir -p $O
MJH_LIB=asimov-mjlab_amd/mjlab_amd/variants/libmjh_head.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "diagonal_sliding or elliptic" > $O/head.log 2>&1 || { tail -5 $O/head.log; exit 1; }
tail -2 $O/head.log
