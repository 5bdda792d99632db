# GPU box: general-path + model_4 parity with the in-tree build, then A/B of ab_base / ab_xcd
# (model_4 hybrid and general at glide, two runs each, plus model_2 general)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_general_gpu.py tests/test_trajectory_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
L=hd-gnn_amd/csrc/libhdgnn.so
cp $L gpurun_out/ab/orig.so
for rep in 1 2; do
for tag in base xcd; do
  cp hd-gnn_amd/csrc/ab_$tag.so $L
  for pa in "--variant 4 --path 1" "--variant 4 --path 2" "--variant 2 --path 2"; do
    timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps 50 --warmup 10 $pa > gpurun_out/ab/run.log 2>&1 || { cp gpurun_out/ab/orig.so $L; exit 1; }
    grep -h '^{' gpurun_out/ab/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"])' $tag "$pa"
  done
done
done
cp gpurun_out/ab/orig.so $L
