# GPU box: model_4 parity tests on a candidate build (ab_<tag>.so), then interleaved
# bench lines of model_4 glide (hybrid) and, with STRESS=1, model_4 / model_2 stress
set -o pipefail
mkdir -p gpurun_out/m4ab
tag=$1
HDG_LIB_PATH=$(pwd)/hd-gnn_amd/csrc/ab_$tag.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_general_gpu.py tests/test_trajectory_gpu.py tests/test_fullsize_gpu.py \
    -k "${TK:-model4 or m4 or variant or ee_ or trajectory or max_}" > gpurun_out/m4ab/$tag.tests.log 2>&1 \
    || { tail -30 gpurun_out/m4ab/$tag.tests.log; exit 1; }
tail -1 gpurun_out/m4ab/$tag.tests.log
TESTS=none VARIANTS="${VARIANTS:-4}" STEPS=20 WARM=5 bash tools/gpu_ab.sh orig $tag || exit 1
if [ -n "$STRESS" ]; then
  TESTS=none VARIANTS="${SVARIANTS:-2 4}" STEPS=20 WARM=5 BARGS="--ne 1024 --nc 512 --batch 32" bash tools/gpu_ab.sh orig $tag || exit 1
fi
