# GPU box: trajectories + the parity suites with the achieved-error report
set -o pipefail
mkdir -p gpurun_out
HDG_PARITY_REPORT=gpurun_out/parity_traj.json timeout -k 10 600 python -u -m pytest -v \
    --timeout 900 --timeout-method thread tests/test_trajectory_gpu.py > gpurun_out/traj.log 2>&1
rc=$?; echo "traj rc=$rc"; tail -5 gpurun_out/traj.log
[ $rc -gt 1 ] && exit $rc
HDG_PARITY_REPORT=gpurun_out/parity_fwdbwd.json timeout -k 10 600 python -u -m pytest -q \
    --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_general_gpu.py > gpurun_out/par.log 2>&1
echo "parity rc=$?"; tail -3 gpurun_out/par.log
