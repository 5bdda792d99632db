# GPU box: k_commit_step's LDS bank-conflict counters per library build
# hd-gnn_amd/csrc/ab_<tag>.so ("orig" = libhdgnn.so): one --pmc pass of tools/lds_phase.py each.
# Variants load through HDG_LIB_PATH; the in-tree libhdgnn.so is never overwritten.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ldsab
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for tag in "$@"; do
  if [ $tag = orig ]; then unset HDG_LIB_PATH; else export HDG_LIB_PATH=$R/hd-gnn_amd/csrc/ab_$tag.so; fi
  timeout -k 5 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU -f csv -d "$OUT/pmc_$tag" -o run -- \
      python3 $R/tools/lds_phase.py > "$OUT/pmc_$tag.log" 2>&1 || { echo "pmc $tag failed"; exit 1; }
  python3 - "$OUT/pmc_$tag" $tag "$R/tools" <<'PY'
import sys
sys.path.insert(0, sys.argv[3])
from roofline_profile import pmc
c = pmc(sys.argv[1]).get("k_commit_step", {})
print(sys.argv[2], "ldsconf %.0f ldsactive %.0f ratio %.3f insts_lds %.0f valu %.0f" % (
    c.get("SQ_LDS_BANK_CONFLICT", 0), c.get("SQ_LDS_IDX_ACTIVE", 0),
    c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 1)),
    c.get("SQ_INSTS_LDS", 0), c.get("SQ_INSTS_VALU", 0)))
PY
done
