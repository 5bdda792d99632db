# GPU box: the profile set's second half -- FP32 FLOP passes, model_4 hybrid trace, bench matrix
# (tools/probe/flops_cal is built on the CPU first: hipcc --offload-arch=gfx950 -O2 -o
# tools/probe/flops_cal tools/probe/flops_cal.hip)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/pmc_flops.sh > $R/gpurun_out/pmc_flops.log 2>&1 || { echo "flops rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_m4 -o run -- \
    python3 $R/bench.py --variant 4 --steps 50 --warmup 10 --no-cpu --e2e 0 > $R/gpurun_out/prof_m4.log 2>&1 || { echo "m4 rc=$?"; exit 1; }
cd $R
bash $R/tools/bench_matrix.sh > $R/gpurun_out/matrix.txt 2>&1 || { echo "matrix rc=$?"; exit 1; }
cat $R/gpurun_out/matrix.txt
