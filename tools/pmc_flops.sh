#!/bin/bash
# FP32 FLOP counters: the calibration probe (known instruction counts), then bench.py's
# kernels (one --pmc pass each, 8 SQ counters).  Run on the GPU box via gpurun.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_flops
mkdir -p $OUT
C="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc $C -f csv -d $OUT/cal -o run -- $R/tools/probe/flops_cal > $OUT/cal.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc $C -f csv -d $OUT/bench -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --e2e 0 --no-graph ${BENCH_ARGS} > $OUT/bench.log 2>&1 || exit $?
cd $R && python3 tools/pmc_table.py $OUT/cal && python3 tools/pmc_table.py $OUT/bench
