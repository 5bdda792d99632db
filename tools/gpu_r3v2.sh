# GPU box: e2e parts, then the full GPU suite, smoke and the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python $R/tools/e2e_parts.py > $R/gpurun_out/e2e_parts.log 2>&1
rc=$?; tail -2 $R/gpurun_out/e2e_parts.log; [ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu_validate.sh
