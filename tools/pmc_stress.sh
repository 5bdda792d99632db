#!/bin/bash
# SQ counters per kernel of the general path at the stress shape (model_2, 1024 x 512,
# B = 32): instruction mix, busy / wait cycles -- two --pmc passes, eager launches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_stress
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--ne 1024 --nc 512 --batch 32 --steps 3 --warmup 1 --no-cpu --e2e 0 --no-graph ${PMC_ARGS:-}"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -f csv -d $OUT/a -o run -- \
    python3 $R/bench.py $ARGS > $OUT/a.log 2>&1 || exit $?
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -f csv -d $OUT/b -o run -- \
    python3 $R/bench.py $ARGS > $OUT/b.log 2>&1 || exit $?
cd $R && python3 tools/pmc_table.py $OUT --json $OUT/table.json > $OUT/table.txt
