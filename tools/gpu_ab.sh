# GPU box: A/B of in-tree library builds hd-gnn_amd/csrc/ab_<tag>.so: per build the fused
# parity + fault tests (TESTS), then model_2 / model_4 glide bench lines; "orig" = libhdgnn.so
set -o pipefail
mkdir -p gpurun_out/ab
L=hd-gnn_amd/csrc/libhdgnn.so
cp $L gpurun_out/ab/orig.so
T=${TESTS:-tests/test_gpu_parity.py tests/test_fault_gpu.py}
for tag in "$@"; do
  if [ $tag = orig ]; then cp gpurun_out/ab/orig.so $L; else cp hd-gnn_amd/csrc/ab_$tag.so $L; fi
  if [ "$T" != none ]; then
    timeout -k 10 400 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/$tag.tests.log 2>&1
    rc=$?; echo "$tag tests: $(tail -1 gpurun_out/ab/$tag.tests.log)"; [ $rc -ne 0 ] && { cp gpurun_out/ab/orig.so $L; exit $rc; }
  fi
done
for rep in 1 2; do
for tag in "$@"; do
  if [ $tag = orig ]; then cp gpurun_out/ab/orig.so $L; else cp hd-gnn_amd/csrc/ab_$tag.so $L; fi
  for v in ${VARIANTS:-2 4}; do
    timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps 50 --warmup 10 --variant $v $BARGS > gpurun_out/ab/$tag.$v.log 2>&1 || { cp gpurun_out/ab/orig.so $L; exit 1; }
    grep -h '^{' gpurun_out/ab/$tag.$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], "model_%s" % sys.argv[2], d["value"], d["ms_per_step"], d["kernels_ms"])' $tag $v
  done
done
done
cp gpurun_out/ab/orig.so $L
