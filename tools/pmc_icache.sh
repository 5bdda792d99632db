#!/bin/bash
# Instruction-cache behaviour of the step kernel (SQC counters, one --pmc pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_icache
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -f csv -d $OUT/a -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --e2e 0 --no-graph ${PMC_ARGS:-} > $OUT/a.log 2>&1 || exit $?
cd $R && python3 tools/pmc_table.py $OUT/a
