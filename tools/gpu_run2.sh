set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/mid_phases.py > gpurun_out/mid_phases.log 2>&1; echo "phases rc=$?"; cat gpurun_out/mid_phases.log | grep -v amdgpu.ids
