#!/bin/bash
# PMC calibration on the GPU box (via gpurun): kernels of known byte / instruction counts
# under the same counters the profiles use.   tools/calibrate.sh <round>
#   fetch_cal (tools/probe/fetch_cal.hip)  FETCH_SIZE / WRITE_SIZE per access width
#   flops_cal (tools/probe/flops_cal.hip)  FP32 FLOP counters per instruction form
# and the device's counter list.  Summarise with tools/roofline_profile.py --cal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1/cal
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 5 -s KILL 60 rocprofv3 --list-avail > "$OUT/counters.txt" 2>&1 || echo "list rc=$?"
timeout -k 5 -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- \
    "$R/tools/probe/fetch_cal" > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 5 -s KILL 60 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- \
    "$R/tools/probe/fetch_cal" > "$OUT/write.log" 2>&1 || exit $?
timeout -k 5 -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS \
    SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 \
    SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU -f csv -d "$OUT/flops" -o run -- \
    "$R/tools/probe/flops_cal" > "$OUT/flops.log" 2>&1 || exit $?
echo "calibration ok"
