#!/bin/bash
# Register / spill / LDS usage of the fused step kernel instantiations (device-only compile):
#   bash tools/kres.sh [pattern]     default: the glide split training kernel <5, true, false, true>
P=${1:-k_commit_stepILi5ELb1ELb0ELb1E}
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include --cuda-device-only \
    -c $R/hd-gnn_amd/csrc/hdgnn.hip -o /tmp/kres_hd.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v P="$P" '/Function Name:/ {show = index($0, P) > 0} show && /VGPRs:|Spill|ScratchSize|Occupancy|SGPRs:/ {sub(/.*remark: /, ""); print}'
