set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/mid_phases.py > gpurun_out/mid_phases.log 2>&1; echo "phases rc=$?"; grep -v amdgpu.ids gpurun_out/mid_phases.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu --e2e 0 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; grep -v amdgpu.ids gpurun_out/bench.log
