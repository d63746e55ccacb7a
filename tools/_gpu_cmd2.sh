set -e
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "single_step_parity or ball_joint or mocap or builtin_sensor" > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
tail -2 $O/par.log
timeout -k 10 200 python -u tools/phase_profile.py 4096 > $O/phase_4096.log 2>&1
grep -E "kinematics|total" $O/phase_4096.log
bash tools/gpu_ab.sh r05r asimov-mjlab_amd/mjlab_amd/variants/libmjh_base.so
