set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_general_gpu.py -x -q --timeout 120 --timeout-method thread -k "model4 or variant or stress or garbage or count or replay or determ" > gpurun_out/m4tests.log 2>&1
rc=$?; tail -3 gpurun_out/m4tests.log; [ $rc -eq 0 ] || exit $rc
for a in "--variant 4" "--variant 4 --path 2" "--variant 4 --ne 250 --nc 150" "--variant 4 --ne 1024 --nc 512 --batch 32"; do
  timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps 20 --warmup 3 $a > gpurun_out/b.log 2>&1 || exit 1
  echo "$a: $(grep -h '^{' gpurun_out/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_m4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --variant 4 --steps 20 --warmup 3 --no-cpu --e2e 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_m4.log 2>&1
