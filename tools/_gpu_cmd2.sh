set -e
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05z
mkdir -p $O
for L in asimov-mjlab_amd/mjlab_amd/libmjh.so asimov-mjlab_amd/mjlab_amd/variants/libmjh_solv.so asimov-mjlab_amd/mjlab_amd/libmjh.so asimov-mjlab_amd/mjlab_amd/variants/libmjh_solv.so; do for T in "4096 40 Mjlab-Velocity-Flat-Unitree-G1" "8192 40 Mjlab-Velocity-Flat-Unitree-Go1"; do MJH_LIB=$L timeout -k 10 120 python tools/kernel_bench.py $T >> $O/kb.log 2>&1; done; done
grep ms/launch $O/kb.log
