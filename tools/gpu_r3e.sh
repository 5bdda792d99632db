# GPU box: round-3 re-entry check -- every GPU test, model_2 / model_4 bench lines, phase stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/e_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu --e2e 0 > gpurun_out/e_m2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --e2e 0 --variant 4 > gpurun_out/e_m4.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("e_m2", "e_m4"):
    for l in open("gpurun_out/%s.log" % f):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["value"], d["ms_per_step"], d["roofline"].get("avg_launch_ms"))
PY
timeout -k 10 200 python tools/mid_phases.py > gpurun_out/e_ph.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/e_ph.log
