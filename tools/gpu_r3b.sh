set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe/valu_rate > gpurun_out/vr.log 2>&1 && \
timeout -k 10 120 ./hd-gnn_amd/csrc/microbench > gpurun_out/mb.log 2>&1
echo rc=$?
