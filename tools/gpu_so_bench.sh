# GPU box: one bench line per library build hd-gnn_amd/csrc/ab_<tag>.so ("orig" = the
# current libhdgnn.so), interleaved, no tests (timing probes whose outputs may be void)
set -o pipefail
O=gpurun_out/sob; mkdir -p $O
L=hd-gnn_amd/csrc/libhdgnn.so
cp $L $O/orig.so
for rep in 1 2; do
  for tag in "$@"; do
    if [ $tag = orig ]; then cp $O/orig.so $L; else cp hd-gnn_amd/csrc/ab_$tag.so $L; fi
    timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps ${STEPS:-20} --warmup 5 $BARGS > $O/$tag.$rep.log 2>&1 || { cp $O/orig.so $L; exit 1; }
    grep -h '^{' $O/$tag.$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' $tag
  done
done
cp $O/orig.so $L
