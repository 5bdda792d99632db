# GPU box: phase stamps (tools/mid_phases.py) of k_commit_step per library build
# hd-gnn_amd/csrc/ab_<tag>.so ("orig" = libhdgnn.so), two runs each, interleaved
set -o pipefail
mkdir -p gpurun_out/ph
L=hd-gnn_amd/csrc/libhdgnn.so
cp $L gpurun_out/ph/orig.so
for rep in 1 2; do
for tag in "$@"; do
  if [ $tag = orig ]; then cp gpurun_out/ph/orig.so $L; else cp hd-gnn_amd/csrc/ab_$tag.so $L; fi
  timeout -k 10 200 python tools/mid_phases.py > gpurun_out/ph/$tag.$rep.log 2>&1 || { cp gpurun_out/ph/orig.so $L; exit 1; }
  echo "$tag $rep: $(grep -E 'phase (5|9|13)->' gpurun_out/ph/$tag.$rep.log | awk '{print $4}' | tr '\n' ' ') total $(grep 'total' gpurun_out/ph/$tag.$rep.log | awk '{print $4}')"
done
done
cp gpurun_out/ph/orig.so $L
rm -f gpurun_out/ph/orig.so
