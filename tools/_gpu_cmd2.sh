set -e
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_libab.sh r05u chain
MJH_LIB=asimov-mjlab_amd/mjlab_amd/variants/libmjh_chain.so timeout -k 10 120 python tools/kernel_bench.py 4096 40 Mjlab-Velocity-Flat-Unitree-G1 > gpurun_out/r05u/kb.log 2>&1
timeout -k 10 120 python tools/kernel_bench.py 4096 40 Mjlab-Velocity-Flat-Unitree-G1 >> gpurun_out/r05u/kb.log 2>&1
grep ms/launch gpurun_out/r05u/kb.log
