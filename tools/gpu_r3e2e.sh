# GPU box: graph2graph train/test tests, the default bench line (with the e2e training-loop
# leg), then the profile set's second half (tools/gpu_r3tail.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/model_tests.log 2>&1
rc=$?; tail -2 $R/gpurun_out/model_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python $R/bench.py > $R/gpurun_out/e2e_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $R/gpurun_out/e2e_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d.get('e2e'), d.get('upload_prepare_ms'))"; [ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu_r3tail.sh
