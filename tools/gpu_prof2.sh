# GPU box: kernel stats of bench.py for two configs (PROF_A, PROF_B argument strings)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
n=0
for a in "${PROF_A:---ne 1024 --nc 512 --batch 32}" "${PROF_B:---variant 4}"; do
  n=$((n+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/p2_$n -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --e2e 0 $a > $R/gpurun_out/p2_$n.log 2>&1) || exit $?
  python3 - $n "$a" <<'PY'
import csv, glob, re, sys
f = sorted(glob.glob("gpurun_out/p2_%s/**/*kernel_stats.csv" % sys.argv[1], recursive=True))[0]
print("==", sys.argv[2])
for r in list(csv.DictReader(open(f)))[:16]:
    n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("hdg::", "")
    print("%-34s %6s %9.2f us" % (n[:34], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
