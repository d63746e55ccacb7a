set -e
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05ze
mkdir -p $O
V=asimov-mjlab_amd/mjlab_amd/variants
for R in 1 2; do for L in $V/libmjh_base.so $V/libmjh_newton.so $V/libmjh_lspar.so; do for T in "4096 40 Mjlab-Velocity-Flat-Unitree-G1" "8192 40 Mjlab-Velocity-Flat-Unitree-Go1"; do MJH_LIB=$L timeout -k 10 120 python tools/kernel_bench.py $T >> $O/kb.log 2>&1; done; done; done
grep ms/launch $O/kb.log | cut -c1-150
