set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_general_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_general.log 2>&1; rc=$?; tail -2 gpurun_out/t_general.log; [ $rc -ne 0 ] && exit $rc
TESTS=none VARIANTS="2" BARGS="--path 2" bash tools/gpu_ab.sh orig head || exit 1
TESTS=none VARIANTS="2 4" BARGS="--ne 1024 --nc 512 --batch 32" bash tools/gpu_ab.sh orig head || exit 1
