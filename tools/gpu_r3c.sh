# GPU box: 50-step trajectories (parity report) then the data-dependence matrix
set -o pipefail
mkdir -p gpurun_out
HDG_PARITY_REPORT=gpurun_out/parity_traj.json timeout -k 10 800 python -u -m pytest -x -v \
    --timeout 900 --timeout-method thread tests/test_trajectory_gpu.py > gpurun_out/traj.log 2>&1
rc=$?; tail -5 gpurun_out/traj.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/bench_data.sh
