# GPU box: round-3 profile set -- kernel trace + stats, FETCH / WRITE passes, SQ passes,
# FP32 FLOP passes (model_2 fused at glide), and a kernel trace of model_4 hybrid at glide.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/profile.sh r03 || exit $?
bash $R/tools/pmc_flops.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_m4 -o run -- \
    python3 $R/bench.py --variant 4 --steps 50 --warmup 10 --no-cpu --e2e 0 > $R/gpurun_out/prof_m4.log 2>&1 || exit $?
echo done
