# GPU box: model_4 parity (general + fused hybrid) and the model_4 bench lines, then the
# per-kernel split of model_4 glide (entity-edge kernels).
set -o pipefail
mkdir -p gpurun_out/eef
timeout -k 10 600 python -u -m pytest tests/test_general_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/eef/tests.log 2>&1
rc=$?; tail -3 gpurun_out/eef/tests.log; [ $rc -eq 0 ] || exit $rc
for a in "m4_glide --variant 4" "m4_s5 --variant 4 --ne 250 --nc 150" "m4_general_glide --variant 4 --path 2"; do
  set -- $a; tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --e2e 0 --steps 20 --warmup 3 "$@" > gpurun_out/eef/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc $(grep -h '^{' gpurun_out/eef/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/eef/prof -o run -- \
    python3 $R/bench.py --variant 4 --steps 20 --warmup 3 --no-cpu --e2e 0 > $R/gpurun_out/eef/prof.log 2>&1
echo "prof rc=$?"
