set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-r05x}
O=gpurun_out/$T
mkdir -p $O
echo "[$(date +%T)] pmc traffic"
MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf -o f -- python tools/kernel_bench.py 4096 40 > $O/pmcf.log 2>&1
MJH_BALANCE=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o w -- python tools/kernel_bench.py 4096 40 > $O/pmcw.log 2>&1
python tools/pmc_traffic.py $(find $O/pmcf -name '*counter_collection.csv') $(find $O/pmcw -name '*counter_collection.csv') 4096 > $O/step_kernel_traffic.json
cat $O/step_kernel_traffic.json
find $O/pmcf $O/pmcw -name '*.csv' -delete
echo "[$(date +%T)] sq"
bash tools/gpu_pmc_sq.sh $T
echo "[$(date +%T)] phase"
timeout -k 10 200 python -u tools/phase_profile.py 4096 > $O/phase_4096.log 2>&1
head -12 $O/phase_4096.log
