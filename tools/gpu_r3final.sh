# GPU box: round-3 final measurement set -- profiles (trace + PMC), the bench matrix
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_prof3.sh > $R/gpurun_out/prof3.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo prof ok
bash $R/tools/bench_matrix.sh > $R/gpurun_out/matrix.txt 2>&1 || { echo "matrix rc=$?"; exit 1; }
cat $R/gpurun_out/matrix.txt
