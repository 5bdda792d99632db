# GPU box: general-path parity tests, then a rocprofv3 kernel-stats run of bench.py
# (BENCH_ARGS, default model_4 glide) and the bench line.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
BA=${BENCH_ARGS:---variant 4}
timeout -k 10 600 python -u -m pytest tests/test_general_gpu.py tests/test_fault_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gen_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gen_tests.log; [ $rc -ne 0 ] && exit $rc
R=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/gen_prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --e2e 0 $BA > $R/gpurun_out/gen_prof.log 2>&1) || exit $?
python3 - <<'PY'
import csv, glob, json, re
f = sorted(glob.glob("gpurun_out/gen_prof/**/*kernel_stats.csv", recursive=True))[0]
for r in list(csv.DictReader(open(f)))[:14]:
    n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("hdg::", "")
    print("%-28s %6s %9.2f us" % (n[:28], r["Calls"], float(r["AverageNs"]) / 1e3))
for l in open("gpurun_out/gen_prof.log"):
    if l.startswith("{"):
        d = json.loads(l); print("bench(traced)", d["value"], d["ms_per_step"])
PY
