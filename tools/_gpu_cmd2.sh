set -e
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05zf
mkdir -p $O
V=asimov-mjlab_amd/mjlab_amd/variants
MJH_LIB=$V/libmjh_caccsw.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "single_step_parity or ball or builtin_sensor or force_torque or mocap" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
tail -1 $O/par.log
for R in 1 2; do for L in $V/libmjh_base.so $V/libmjh_caccsw.so; do for T in "4096 40 Mjlab-Velocity-Flat-Unitree-G1" "8192 40 Mjlab-Velocity-Flat-Unitree-Go1"; do MJH_LIB=$L timeout -k 10 120 python tools/kernel_bench.py $T >> $O/kb.log 2>&1; done; done; done
grep ms/launch $O/kb.log | cut -c1-150
