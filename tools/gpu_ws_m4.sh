# GPU box: wave stamps of model_4 glide (hybrid) entity-edge kernels (WSTAMP builds ws_<id>.so)
set -o pipefail
mkdir -p gpurun_out/wsm4
for k in 7 5 6 13; do
  HDG_LIB_PATH=$(pwd)/hd-gnn_amd/csrc/ws_$k.so timeout -k 10 120 python tools/wstamp.py 5 --ne 200 --nc 74 \
      --batch 100 --variant 4 --path 1 > gpurun_out/wsm4/ws_$k.log 2>&1 || { tail -5 gpurun_out/wsm4/ws_$k.log; exit 1; }
  echo "== kernel id $k"; grep -v amdgpu.ids gpurun_out/wsm4/ws_$k.log
done
