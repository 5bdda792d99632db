#!/bin/bash
# model_4 hybrid at glide: per-kernel HBM traffic (FETCH_SIZE, WRITE_SIZE in separate
# --pmc passes) and the SQ counter passes (tools/pmc_sq_m4.sh).  Run on the GPU box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_m4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -f csv -d $OUT/$c -o run -- \
      python3 $R/bench.py --variant 4 --steps 10 --warmup 2 --no-cpu --e2e 0 > $OUT/$c.log 2>&1 || exit $?
done
bash $R/tools/pmc_sq_m4.sh > $OUT/sq.txt 2>&1 || exit $?
echo done
