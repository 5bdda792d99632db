set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "${1:-}" > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|mismatch|  [a-zA-Z_/0-9]+:0: max" gpurun_out/pytest_gpu.log | head -40
