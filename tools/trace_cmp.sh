#!/bin/bash
# GPU box: rocprofv3 kernel-trace averages for several bench.py variants (A/B of kernels
# whose eager event times are not trusted).  tools/trace_cmp.sh <outdir> "tag|ENV=..|args" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$1
shift
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$R/$OUT/$tag" -o run -- \
      python3 $R/bench.py --no-cpu --e2e 0 --steps 20 --warmup 3 $args > "$R/$OUT/$tag.log" 2>&1 || exit $?
  python3 - "$R/$OUT/$tag" "$tag" <<'PY'
import csv, glob, sys, re, json
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
line = [json.loads(l) for l in open(sys.argv[1] + ".log") if l.startswith("{")]
v = line[0]["value"] if line else None
print("== %s  %s commits/s, %s ms/step" % (sys.argv[2], v, line[0]["ms_per_step"] if line else None))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("hdg::", "").split("(")[0]
    if int(r["Calls"]) >= 20:
        print("  %-40s %6s %9.2f us" % (n[:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
