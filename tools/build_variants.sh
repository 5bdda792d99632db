# Build library variants for counter attribution / A/B runs, in parallel (CPU, here):
#   tools/build_variants.sh <out_prefix> "<tag>:<hipcc -D flags>" ...
# -> hd-gnn_amd/csrc/<out_prefix>_<tag>.so; wide.hip compiled once.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/hd-gnn_amd/csrc
P=$1; shift
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include"
T=$(mktemp -d /tmp/hdgv.XXXX)
$HIPCC -c -o $T/wide.o $C/wide.hip &
pids=""
for spec in "$@"; do
  tag=${spec%%:*}; fl=${spec#*:}
  ( $HIPCC $fl -c -o $T/h_$tag.o $C/hdgnn.hip ) &
  pids="$pids $!"
  while [ $(jobs -r | wc -l) -ge ${JOBS:-6} ]; do sleep 1; done
done
wait
for spec in "$@"; do
  tag=${spec%%:*}
  $HIPCC -shared -o $C/${P}_$tag.so $T/h_$tag.o $T/wide.o
done
rm -rf $T
