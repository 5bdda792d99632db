# GPU box: data-dependence matrix of the step throughput at glide (Ne=200, Nc=74, B=100).
# Entity density {0.05, 0.2, 0.5} x hunk (label) density {0.1, 0.3} x attributes
# {int10: integers 0..9, real: Ne distinct signed reals} for model_2 fused, model_2 general
# and model_4 hybrid.  One bench.py line per cell -> gpurun_out/data/<tag>.log, and a
# table gpurun_out/data/summary.txt (copied to profiles/rNN/data_matrix.txt).
set -o pipefail
mkdir -p gpurun_out/data
S=gpurun_out/data/summary.txt
echo "# path edensity hdensity xkind commits/s ms/step kernel_ms" > $S
for path in m2_fused m2_general m4_hybrid; do
  case $path in
    m2_fused) pa="--variant 2 --path 1";;
    m2_general) pa="--variant 2 --path 2";;
    m4_hybrid) pa="--variant 4 --path 1";;
  esac
  for ed in 0.05 0.2 0.5; do
    for hd in 0.1 0.3; do
      for xk in int10 real; do
        tag=${path}_e${ed}_h${hd}_${xk}
        timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps 20 --warmup 4 $pa \
            --edensity $ed --hdensity $hd --xkind $xk > gpurun_out/data/$tag.log 2>&1
        rc=$?
        if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -3 gpurun_out/data/$tag.log; exit $rc; fi
        grep -h '^{' gpurun_out/data/$tag.log | python3 -c '
import json, sys
d = json.loads(sys.stdin.read())
k = d["kernels_ms"]; kk = list(k)[0]
print(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], d["value"], d["ms_per_step"], kk, k[kk])' \
            $path $ed $hd $xk >> $S
        tail -1 $S
      done
    done
  done
done
