# GPU box: general-path parity tests, then an A/B of libhdgnn.so ("orig") against
# hd-gnn_amd/csrc/ab_<tag>.so on the workloads given as BARGS lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_general_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_general.log 2>&1; rc=$?; tail -2 gpurun_out/t_general.log; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-head}
TESTS=none VARIANTS="${VARIANTS:-2}" BARGS="${BARGS1:---path 2}" bash tools/gpu_ab.sh orig $TAG || exit 1
[ -n "$BARGS2" ] && { TESTS=none VARIANTS="${VARIANTS2:-2 4}" BARGS="$BARGS2" bash tools/gpu_ab.sh orig $TAG || exit 1; }
exit 0
