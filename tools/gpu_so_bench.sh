# GPU box: one bench line per library build hd-gnn_amd/csrc/ab_<tag>.so ("orig" = the
# current libhdgnn.so), interleaved, no tests (timing probes whose outputs may be void).
# Variants load through HDG_LIB_PATH; the in-tree libhdgnn.so is never overwritten.
set -o pipefail
O=gpurun_out/sob; mkdir -p $O
for rep in 1 2; do
  for tag in "$@"; do
    if [ $tag = orig ]; then LP=; else LP=$(pwd)/hd-gnn_amd/csrc/ab_$tag.so; fi
    HDG_LIB_PATH=$LP timeout -k 10 200 python bench.py --no-cpu --e2e 0 --no-steady --steps ${STEPS:-20} --warmup ${WARM:-5} $BARGS > $O/$tag.$rep.log 2>&1 || exit 1
    grep -h '^{' $O/$tag.$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' $tag
  done
done
