#!/bin/bash
# SQ counters of the pair-tile microbenchmark kernels (csrc/microbench): two --pmc passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_mb
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -f csv -d $OUT/a -o run -- \
    $R/hd-gnn_amd/csrc/microbench > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR -f csv -d $OUT/b -o run -- \
    $R/hd-gnn_amd/csrc/microbench > $OUT/b.log 2>&1 || exit $?
cd $R && python3 tools/pmc_table.py $OUT
