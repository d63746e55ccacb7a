#!/bin/bash
# Final evidence on HEAD: three-config benches, SQ counters, PMC traffic of the step kernel.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03zd
mkdir -p $O
PROF=0 bash tools/gpu_bench3.sh r03zd_b3 > $O/b3.log 2>&1 || { tail -20 $O/b3.log; exit 1; }
grep '^{' $O/b3.log | cut -c1-200
bash tools/gpu_pmc_sq.sh r03zd_sq 4096 > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf -o f -- python tools/kernel_bench.py 4096 40 > $O/pmcf.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o w -- python tools/kernel_bench.py 4096 40 > $O/pmcw.log 2>&1
python tools/pmc_traffic.py $(find $O/pmcf -name '*counter_collection.csv') $(find $O/pmcw -name '*counter_collection.csv') 4096 > $O/step_kernel_traffic.json
cat $O/step_kernel_traffic.json
for P in pmcf pmcw; do
  F=$(find $O/$P -name '*counter_collection.csv' | head -1)
  { head -1 $F; grep 'step_kernel' $F || true; } > $O/${P}_step_kernel_rows.csv
done
find $O/pmcf $O/pmcw -name '*.csv' -delete
