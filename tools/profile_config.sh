#!/bin/bash
# rocprofv3 evidence for one bench.py workload (GPU box, via gpurun):
#   tools/profile_config.sh <round>/<tag> [bench.py args ...]
# writes gpurun_out/<round>/<tag>/: a kernel trace + stats of the bench command (HIP-graph
# replay, as the bench line runs), then one --pmc pass each (eager launches): FETCH_SIZE,
# WRITE_SIZE, SQ issue / wait counters, LDS bank conflicts, FP32 FLOP counters.  Summarise locally with
#   python tools/roofline_profile.py gpurun_out/<round>/<tag> profiles/<round>/<tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
echo "$*" > "$OUT/args.txt"
BENCH="$R/bench.py --no-cpu --e2e 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 $BENCH --steps 20 --warmup 5 > "$OUT/bench_trace.log" 2>&1 || exit $?
echo "$TAG trace ok"
pmc() {   # pmc <name> <counters...>
  local name=$1
  shift
  timeout -k 5 -s KILL 180 rocprofv3 --pmc "$@" -f csv -d "$OUT/$name" -o run -- \
      python3 $BENCH --steps 3 --warmup 1 --no-graph --no-steady > "$OUT/bench_$name.log" 2>&1 || exit $?
  echo "$TAG $name ok"
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pmc lds SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM_RD \
    SQ_INSTS_VMEM_WR SQ_INSTS_SALU
pmc flops SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_MFMA_MOPS_F32 \
    SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 \
    SQ_INSTS_VALU
exit 0
