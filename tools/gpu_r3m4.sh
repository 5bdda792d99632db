# GPU box: model_4 hybrid kernel trace at glide and the config matrix (final HEAD)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_m4 -o run -- \
    python3 $R/bench.py --variant 4 --steps 50 --warmup 10 --no-cpu --e2e 0 > $R/gpurun_out/prof_m4.log 2>&1 || { echo "m4 rc=$?"; exit 1; }
cd $R
bash $R/tools/bench_matrix.sh > $R/gpurun_out/matrix.txt 2>&1 || { echo "matrix rc=$?"; exit 1; }
cat $R/gpurun_out/matrix.txt
