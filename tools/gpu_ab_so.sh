# GPU box: A/B the in-tree library builds hd-gnn_amd/csrc/ab_<tag>.so (bench line per
# build: model_2 fused and model_4 hybrid at glide), plus the VALU rate probe
set -o pipefail
mkdir -p gpurun_out/ab
L=hd-gnn_amd/csrc/libhdgnn.so
cp $L gpurun_out/ab/orig.so
timeout -k 10 120 ./tools/probe/valu_rate > gpurun_out/valu_rate.txt 2>&1 || exit $?
for rep in 1 2; do
for tag in "$@"; do
  cp hd-gnn_amd/csrc/ab_$tag.so $L
  for v in 2 4; do
    timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps 50 --warmup 10 --variant $v > gpurun_out/ab/$tag.$v.log 2>&1 || exit $?
    grep -h '^{' gpurun_out/ab/$tag.$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], "model_%s" % sys.argv[2], d["value"], d["ms_per_step"], d["kernels_ms"])' $tag $v
  done
done
done
cp gpurun_out/ab/orig.so $L
