# GPU box: full bench line (with the CPU baseline) + rocprofv3 evidence for profiles/<tag>.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_full.log | tail -3
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh $TAG; rc=$?; echo "profile rc=$rc"; exit $rc
