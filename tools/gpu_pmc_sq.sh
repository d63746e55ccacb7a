#!/bin/bash
# SQ (instruction mix / stall) counters of the physics step kernel, one rocprofv3
# --pmc pass per counter group, each under its own time limit.
# usage (repo root on the GPU box): bash tools/gpu_pmc_sq.sh <tag> [N]
set -e
TAG=${1:-sq}
N=${2:-4096}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
export MJH_BALANCE=1  # world ordering on, as in the bench
O=gpurun_out/$TAG
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
grep -o 'SQ_[A-Z0-9_]*' $O/counters_list.txt | sort -u > $O/sq_counters.txt || true
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
B="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
i=0
for G in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $O/p$i -o p -- python tools/kernel_bench.py $N 20 > $O/p$i.log 2>&1
done
python tools/pmc_summary.py "step_kernel" 20 $(find $O/p1 $O/p2 -name '*counter_collection.csv') > $O/sq_summary.json
cat $O/sq_summary.json
# the bench line's roofline_valu input (commit it under profiles/)
python tools/sq_to_roofline.py $O/sq_summary.json Mjlab-Velocity-Flat-Unitree-G1 $N "$TAG SQ_INSTS_VALU, kernel_bench G1 N=$N" $O/step_kernel_sq.json
find $O/p1 $O/p2 -name '*.csv' -delete
