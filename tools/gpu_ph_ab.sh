# GPU box: phase stamps (tools/mid_phases.py) of k_commit_step per library build
# hd-gnn_amd/csrc/ab_<tag>.so ("orig" = libhdgnn.so), two runs each, interleaved.
# Variants load through HDG_LIB_PATH; the in-tree libhdgnn.so is never overwritten.
set -o pipefail
mkdir -p gpurun_out/ph
for rep in 1 2; do
for tag in "$@"; do
  if [ $tag = orig ]; then LP=; else LP=$(pwd)/hd-gnn_amd/csrc/ab_$tag.so; fi
  HDG_LIB_PATH=$LP timeout -k 10 200 python tools/mid_phases.py > gpurun_out/ph/$tag.$rep.log 2>&1 || exit 1
  echo "$tag $rep: $(grep -E 'phase (5|9|13)->' gpurun_out/ph/$tag.$rep.log | awk '{print $4}' | tr '\n' ' ') total $(grep 'total' gpurun_out/ph/$tag.$rep.log | awk '{print $4}')"
done
done
