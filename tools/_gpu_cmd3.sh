set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
echo "[$(date +%T)] pmc traffic"
MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf -o f -- python tools/kernel_bench.py 4096 40 > $O/pmcf.log 2>&1
MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o w -- python tools/kernel_bench.py 4096 40 > $O/pmcw.log 2>&1
python tools/pmc_traffic.py $(find $O/pmcf -name '*counter_collection.csv') $(find $O/pmcw -name '*counter_collection.csv') 4096 > $O/step_kernel_traffic.json
cat $O/step_kernel_traffic.json
find $O/pmcf $O/pmcw -name '*.csv' -delete
echo "[$(date +%T)] sq"
bash tools/gpu_pmc_sq.sh r05l
echo "[$(date +%T)] bench3"
bash tools/gpu_bench3.sh r05l
