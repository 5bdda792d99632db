# GPU box: the data-parallel checks (xGMI tails, one-rank-per-device and shared-device),
# bench.py --gpus 4 on the one GPU, and the driver's 1-GPU bench command.
set -o pipefail
mkdir -p gpurun_out/dp
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_xgmi_gpu.py tests/test_rccl_gpu.py > gpurun_out/dp/pytest_dp.log 2>&1 \
    || { tail -40 gpurun_out/dp/pytest_dp.log; exit 1; }
tail -3 gpurun_out/dp/pytest_dp.log
timeout -k 10 300 python bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu --e2e 0 \
    > gpurun_out/dp/bench_gpus4.log 2>&1 || { tail -40 gpurun_out/dp/bench_gpus4.log; exit 1; }
grep '^{' gpurun_out/dp/bench_gpus4.log | cut -c1-600
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
    > gpurun_out/dp/bench_driver_cmd.log 2>&1 || { tail -40 gpurun_out/dp/bench_driver_cmd.log; exit 1; }
grep '^{' gpurun_out/dp/bench_driver_cmd.log | cut -c1-700
