# Build library variants for counter attribution / A/B runs, in parallel (CPU, here):
#   tools/build_variants.sh <out_prefix> "<tag>:<hipcc -D flags>" ...
# -> hd-gnn_amd/csrc/<out_prefix>_<tag>.so; both sources compiled with the tag's flags
# (the wide.hip knobs, HDG_ABL_* / HDG_GAM_FROM_PROBS ..., and hdgnn.hip's HDG_STOP_AFTER ...)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/hd-gnn_amd/csrc
P=$1; shift
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include"
T=$(mktemp -d /tmp/hdgv.XXXX)
for spec in "$@"; do
  tag=${spec%%:*}; fl=${spec#*:}
  for src in hdgnn wide; do
    ( $HIPCC $fl -c -o $T/${src}_$tag.o $C/$src.hip ) &
    while [ $(jobs -r | wc -l) -ge ${JOBS:-6} ]; do sleep 1; done
  done
done
wait
for spec in "$@"; do
  tag=${spec%%:*}
  $HIPCC -shared -o $C/${P}_$tag.so $T/hdgnn_$tag.o $T/wide_$tag.o
done
rm -rf $T
