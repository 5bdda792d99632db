# GPU box: all GPU tests, then model_2 / model_4 glide bench lines and a model_4 kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/m4_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu --e2e 0 > gpurun_out/m2b.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --e2e 0 --variant 4 > gpurun_out/m4b.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("m2b", "m4b"):
    for l in open("gpurun_out/%s.log" % f):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["value"], d["ms_per_step"])
PY
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_m4c -o run -- \
    python3 $R/bench.py --variant 4 --steps 20 --warmup 3 --no-cpu --e2e 0 > $R/gpurun_out/prof_m4c.log 2>&1 || exit $?
head -8 $R/gpurun_out/prof_m4c/run_kernel_stats.csv | cut -c1-60,200-260
