set -e
cd "${GRAFT_REPO_ROOT:-.}"
TESTS=1 BENCH=300 bash tools/gpu_r05.sh r05p
grep "\[sensor " gpurun_out/r05p/gputests.log | head -40
