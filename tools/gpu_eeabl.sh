# GPU box: kernel times of ablation builds of the library (gpurun_abl_<n>.so next to the
# repo root, built with -DEE_ABL=<n>) against the in-tree build, model_4 glide.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/abl
for lib in base $(ls gpurun_abl_*.so 2>/dev/null); do
  tag=$(basename $lib .so)
  if [ $lib = base ]; then unset HDG_LIB_PATH; else export HDG_LIB_PATH=$R/$lib; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/abl/$tag -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --e2e 0 ${BENCH_ARGS:---variant 4} > $R/gpurun_out/abl/$tag.log 2>&1) || exit $?
  python3 - $tag <<'PY'
import csv, glob, re, sys
f = sorted(glob.glob("gpurun_out/abl/%s/**/*kernel_stats.csv" % sys.argv[1], recursive=True))[0]
out = []
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("hdg::", "")
    out.append("%s %.1f" % (n.split("<")[0], float(r["AverageNs"]) / 1e3))
print(sys.argv[1], "|", ", ".join(out[:8]))
PY
done
