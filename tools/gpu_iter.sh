# quick GPU iteration: fused parity tests, bench, phase stamps (stops at the first failure)
set -o pipefail
mkdir -p gpurun_out
T=${1:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > gpurun_out/it_tests.log 2>&1; rc=$?
tail -3 gpurun_out/it_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu --e2e 0 > gpurun_out/it_bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/it_bench.log | python3 -c "import sys,json; l=[x for x in sys.stdin if x.startswith('{')]; d=json.loads(l[-1]); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 200 python tools/mid_phases.py > gpurun_out/it_ph.log 2>&1 || exit $?
cat gpurun_out/it_ph.log | grep -v amdgpu
