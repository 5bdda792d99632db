# GPU box: bench.py over the BASELINE configs / variants / engine paths (one JSON line each)
# + a kernel trace of model_4 at glide (fused step kernel + entity-edge general kernels).
set -o pipefail
mkdir -p gpurun_out/matrix
run() {   # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --e2e 0 --steps 20 --warmup 3 "$@" > gpurun_out/matrix/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -h '^{' gpurun_out/matrix/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms/step")' 2>/dev/null)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run m2_fused_glide
run_env() { local v=$1; shift; HDG_FUSED_SPLIT=$v run "$@"; }
run_env 0 m2_fused_glide_oneblock
run m2_general_glide --path 2
run m1_glide --variant 1
run m3_glide --variant 3
run m4_glide --variant 4
run m4_general_glide --variant 4 --path 2
run m2_fused_s3 --ne 250 --nc 114
run m2_fused_s5 --ne 250 --nc 150
run m4_s5 --variant 4 --ne 250 --nc 150
run m4_general_s5 --variant 4 --ne 250 --nc 150 --path 2
run m2_stress --ne 1024 --nc 512 --batch 32
run m4_stress --variant 4 --ne 1024 --nc 512 --batch 32
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_general -o run -- \
    python3 $R/bench.py --variant 4 --steps 20 --warmup 3 --no-cpu --e2e 0 > $R/gpurun_out/matrix/prof_m4.log 2>&1
echo "prof rc=$?"
