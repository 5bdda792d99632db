# GPU box: quick A/B of the fused step: GPU parity tests of the fused path, phase stamps,
# bench (no CPU baseline).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fault_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/mid_phases.py > gpurun_out/ab_phases.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/ab_phases.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --e2e 0 ${BENCH_ARGS} > gpurun_out/ab_bench.log 2>&1 || exit $?
python - <<'PY'
import json
for l in open("gpurun_out/ab_bench.log"):
    if l.startswith("{"):
        d = json.loads(l); print("bench", d["value"], d["ms_per_step"], d["kernels_ms"], d["roofline"]["frac"])
PY
done
