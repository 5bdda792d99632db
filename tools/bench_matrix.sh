# GPU box: one bench.py line per workload of tools/configs.sh (+ model_2 glide with one block
# per commit) -> gpurun_out/matrix/<tag>.log; summarise locally with
#   python tools/bench_matrix.py gpurun_out/matrix profiles/<round>/bench_matrix
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
source "$R/tools/configs.sh"
mkdir -p gpurun_out/matrix
run() {   # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --e2e 0 --steps 20 --warmup 5 "$@" > gpurun_out/matrix/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -h '^{' gpurun_out/matrix/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms/step; steady", (d.get("steady_state") or {}).get("value"))' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
for t in ${*:-$ORDER}; do
  run $t ${CFG[$t]}
done
[ -z "$*" ] && HDG_FUSED_SPLIT=0 run glide_oneblock
exit 0
