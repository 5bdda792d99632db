set -o pipefail
mkdir -p gpurun_out/m4c
timeout -k 10 600 python -u -m pytest tests/test_general_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/m4c/pytest.log 2>&1; rc=$?
tail -4 gpurun_out/m4c/pytest.log; [ $rc -eq 0 ] || exit $rc
R=${GRAFT_REPO_ROOT}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/m4c/prof -o run -- \
    python3 $R/bench.py --variant 4 --steps 20 --warmup 3 --no-cpu --e2e 0 > $R/gpurun_out/m4c/bench.log 2>&1 || exit $?
grep -h '^{' $R/gpurun_out/m4c/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
grep -h "ee_nodeb" $R/gpurun_out/m4c/prof/run_kernel_stats.csv | cut -c1-40,100-200
