#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --steps 50 --warmup 10 --no-cpu --e2e 0 > $OUT/bench_traced.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --e2e 0 > $OUT/bench_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --e2e 0 > $OUT/bench_write.log 2>&1 || exit $?
bash $R/tools/pmc_sq.sh || exit $?
# summarise locally afterwards: python tools/prof_summary.py gpurun_out/prof_$TAG $TAG; python tools/valu_issue.py gpurun_out/pmc_sq gpurun_out/prof_$TAG $TAG 200
