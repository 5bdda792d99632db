# GPU box: per-phase counter attribution of k_commit_step.  For every library build
# hd-gnn_amd/csrc/stop_<n>.so (HDG_STOP_AFTER=n: blocks return at phase boundary n) and
# the full build, one --pmc pass (LDS / issue counters) and one kernel trace of
# tools/lds_phase.py.  Summarise locally with tools/lds_phases_sum.py gpurun_out/lds.
# The builds load through HDG_LIB_PATH; the in-tree libhdgnn.so is never overwritten.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lds
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for tag in "$@"; do
  if [ "$tag" = full ]; then unset HDG_LIB_PATH; else export HDG_LIB_PATH=$R/hd-gnn_amd/csrc/stop_$tag.so; fi
  timeout -k 5 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU -f csv -d "$OUT/pmc_$tag" -o run -- \
      python3 $R/tools/lds_phase.py > "$OUT/pmc_$tag.log" 2>&1 || { echo "pmc $tag failed"; exit 1; }
  timeout -k 5 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/tr_$tag" -o run -- \
      python3 $R/tools/lds_phase.py > "$OUT/tr_$tag.log" 2>&1 || { echo "trace $tag failed"; exit 1; }
  echo "$tag ok"
done
