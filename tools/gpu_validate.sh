# GPU box: the whole GPU suite, smoke and the default bench line (gpu_final.sh without the config matrix).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; tail -3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/final_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/final_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/final_bench.log; [ $rc -eq 0 ] || exit $rc
