# GPU box: rocprofv3 kernel-trace averages per library build hd-gnn_amd/csrc/ab_<tag>.so
# ("orig" = the current libhdgnn.so) with the same bench arguments ($BARGS)
set -o pipefail
L=hd-gnn_amd/csrc/libhdgnn.so
mkdir -p gpurun_out/sot
cp $L gpurun_out/sot/orig.so
for tag in "$@"; do
  if [ $tag = orig ]; then cp gpurun_out/sot/orig.so $L; else cp hd-gnn_amd/csrc/ab_$tag.so $L; fi
  bash tools/trace_cmp.sh gpurun_out/sot "$tag||$BARGS" || { cp gpurun_out/sot/orig.so $L; exit 1; }
done
cp gpurun_out/sot/orig.so $L
