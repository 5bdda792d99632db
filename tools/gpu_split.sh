# GPU box: fused-path parity (split + one-block), then bench both modes and phase stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?; tail -5 gpurun_out/split_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu --e2e 0 > gpurun_out/bench_split.log 2>&1 || exit $?
HDG_FUSED_SPLIT=0 timeout -k 10 300 python bench.py --no-cpu --e2e 0 > gpurun_out/bench_one.log 2>&1 || exit $?
timeout -k 10 120 python tools/mid_phases.py > gpurun_out/phases_split.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("bench_split", "bench_one"):
    for l in open("gpurun_out/%s.log" % f):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["value"], d["ms_per_step"], d["kernels_ms"])
PY
grep -v amdgpu gpurun_out/phases_split.log
timeout -k 10 60 hd-gnn_amd/csrc/mb_entity > gpurun_out/mbe.log 2>&1 && cat gpurun_out/mbe.log
