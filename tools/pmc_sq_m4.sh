#!/bin/bash
# SQ counters per kernel for model_4 hybrid at glide (two --pmc passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_sq_m4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -f csv -d $OUT/a -o run -- \
    python3 $R/bench.py --variant 4 --steps 5 --warmup 2 --no-cpu --e2e 0 --no-graph > $OUT/a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -f csv -d $OUT/b -o run -- \
    python3 $R/bench.py --variant 4 --steps 5 --warmup 2 --no-cpu --e2e 0 --no-graph > $OUT/b.log 2>&1 || exit $?
cd $R && python3 tools/pmc_table.py $OUT
