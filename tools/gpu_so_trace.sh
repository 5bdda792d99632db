# GPU box: rocprofv3 kernel-trace averages per library build hd-gnn_amd/csrc/ab_<tag>.so
# ("orig" = the current libhdgnn.so) with the same bench arguments ($BARGS).
# Variants load through HDG_LIB_PATH; the in-tree libhdgnn.so is never overwritten.
set -o pipefail
mkdir -p gpurun_out/sot
for tag in "$@"; do
  if [ $tag = orig ]; then unset HDG_LIB_PATH; else export HDG_LIB_PATH=$(pwd)/hd-gnn_amd/csrc/ab_$tag.so; fi
  bash tools/trace_cmp.sh gpurun_out/sot "$tag||$BARGS" || exit 1
done
