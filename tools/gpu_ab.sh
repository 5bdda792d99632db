# GPU box: A/B of in-tree library builds hd-gnn_amd/csrc/ab_<tag>.so: per build the fused
# parity + fault tests (TESTS), then model_2 / model_4 glide bench lines; "orig" = libhdgnn.so.
# Variants load through HDG_LIB_PATH; the in-tree libhdgnn.so is never overwritten.
set -o pipefail
mkdir -p gpurun_out/ab
T=${TESTS:-tests/test_gpu_parity.py tests/test_fault_gpu.py}
lp() { if [ $1 = orig ]; then echo ""; else echo "$(pwd)/hd-gnn_amd/csrc/ab_$1.so"; fi; }
for tag in "$@"; do
  if [ "$T" != none ]; then
    HDG_LIB_PATH=$(lp $tag) timeout -k 10 400 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/$tag.tests.log 2>&1
    rc=$?; echo "$tag tests: $(tail -1 gpurun_out/ab/$tag.tests.log)"; [ $rc -ne 0 ] && exit $rc
  fi
done
for rep in 1 2; do
for tag in "$@"; do
  for v in ${VARIANTS:-2 4}; do
    HDG_LIB_PATH=$(lp $tag) timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps ${STEPS:-50} --warmup ${WARM:-10} --variant $v $BARGS > gpurun_out/ab/$tag.$v.log 2>&1 || exit 1
    grep -h '^{' gpurun_out/ab/$tag.$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d.get("steady_state") or {}; print(sys.argv[1], "model_%s" % sys.argv[2], d["value"], d["ms_per_step"], "steady", s.get("value"), s.get("ms_per_step"), d["kernels_ms"])' $tag $v
  done
done
done
