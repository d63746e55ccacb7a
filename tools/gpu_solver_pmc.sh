#!/bin/bash
# Counter measurement of the constraint-solver launch of the split step build (north-star figure).
# usage (repo root on the box): bash tools/gpu_solver_pmc.sh <tag>
set -e
TAG=${1:-solver}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
L=asimov-mjlab_amd/mjlab_amd/variants/libmjh_split.so
MJH_LIB=$L MJH_BALANCE=1 timeout -k 10 120 python tools/kernel_bench.py 4096 40 > $O/kb_split.log 2>&1
cat $O/kb_split.log | grep ms/launch
MJH_LIB=$L MJH_BALANCE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python tools/kernel_bench.py 4096 40 > $O/st.log 2>&1
MJH_LIB=$L MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o f -- python tools/kernel_bench.py 4096 40 > $O/pf.log 2>&1
MJH_LIB=$L MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o w -- python tools/kernel_bench.py 4096 40 > $O/pw.log 2>&1
S=$(find $O/st -name '*kernel_stats.csv' | head -1)
F=$(find $O/pf -name '*counter_collection.csv' | head -1)
W=$(find $O/pw -name '*counter_collection.csv' | head -1)
cp $S $O/split_kernel_stats.csv
python tools/solver_roofline.py $S $F $W $O/kb_split.log 4096 35 "$TAG" > $O/solver_roofline.json
cat $O/solver_roofline.json
for P in pf pw; do
  C=$(find $O/$P -name '*counter_collection.csv' | head -1)
  { head -1 $C; grep 'step_kernel' $C || true; } > $O/${P}_step_rows.csv
done
find $O/st $O/pf $O/pw -name '*.csv' -delete
