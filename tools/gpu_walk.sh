# GPU box: general-path + prep + fault tests, then the configs whose entity walks run on the
# general path (bench lines only).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_general_gpu.py tests/test_prep_gpu.py tests/test_fault_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/walk_tests.log 2>&1
rc=$?; tail -3 gpurun_out/walk_tests.log; [ $rc -eq 0 ] || exit $rc
for a in "--path 2" "--variant 4" "--variant 4 --path 2" "--variant 4 --ne 250 --nc 150" "--ne 1024 --nc 512 --batch 32" "--variant 4 --ne 1024 --nc 512 --batch 32"; do
  timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps 20 --warmup 3 $a > gpurun_out/b.log 2>&1 || exit 1
  echo "$a: $(grep -h '^{' gpurun_out/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("upload_prepare_ms"))')"
done
