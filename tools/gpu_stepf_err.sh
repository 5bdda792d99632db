# GPU box: the fused parity suite's achieved errors with the default build and with the
# HDG_STEPF=0 build (exact add + step masks instead of the clamped packed fma), so DESIGN 6
# can say which of the worst fused-gradient cases the mask form moves
set -o pipefail
mkdir -p gpurun_out/stepf
for tag in orig stepf0; do
  if [ $tag = orig ]; then LP=; else LP=$(pwd)/hd-gnn_amd/csrc/ab_$tag.so; fi
  HDG_LIB_PATH=$LP HDG_PARITY_REPORT=gpurun_out/stepf/$tag.json timeout -k 10 400 python -u -m pytest -x -q \
      --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/stepf/$tag.log 2>&1 \
      || { tail -20 gpurun_out/stepf/$tag.log; exit 1; }
  tail -1 gpurun_out/stepf/$tag.log
done
