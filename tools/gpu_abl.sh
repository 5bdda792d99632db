# GPU box: kernel times of bench.py (ABL_ARGS) under each library in gpurun_lib/ (HDG_LIB_PATH)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
for L in gpurun_lib/lib*.so; do
  n=$(basename $L .so)
  (cd /tmp && export TMPDIR=/tmp HDG_LIB_PATH=$R/$L && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/abl_$n -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --e2e 0 ${ABL_ARGS:---path 2} > $R/gpurun_out/abl_$n.log 2>&1) || exit $?
  python3 - $n <<'PY'
import csv, glob, re, sys
f = sorted(glob.glob("gpurun_out/abl_%s/**/*kernel_stats.csv" % sys.argv[1], recursive=True))[0]
out = []
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "").replace("hdg::", "").replace("void ", ""))
    if r["Calls"] in ("61", "41") or "first" in n or "ent_fwd" in n:
        out.append("%s %.1f" % (n[:20], float(r["AverageNs"]) / 1e3))
print(sys.argv[1], " | ".join(out[:9]))
PY
done
