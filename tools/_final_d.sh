set -o pipefail
bash tools/bench_matrix.sh
