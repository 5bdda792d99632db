# GPU box: model_4 hybrid per-kernel split (rocprofv3 kernel trace) for each in-tree
# library build hd-gnn_amd/csrc/ab_<tag>.so given on the command line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/hd-gnn_amd/csrc/libhdgnn.so
mkdir -p $R/gpurun_out/m4split
cp $L $R/gpurun_out/m4split/orig.so
cd /tmp && export TMPDIR=/tmp
for tag in "$@"; do
  cp $R/hd-gnn_amd/csrc/ab_$tag.so $L
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/m4split/$tag -o run -- \
      python3 $R/bench.py --variant 4 --steps 50 --warmup 10 --no-cpu --e2e 0 > $R/gpurun_out/m4split/$tag.log 2>&1 || exit $?
  f=$(find $R/gpurun_out/m4split/$tag -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$tag" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(sys.argv[2], r["Name"][:40], r["Calls"], "%.2f us" % (float(r["AverageNs"]) / 1e3))
PY
done
cp $R/gpurun_out/m4split/orig.so $L
