#!/bin/bash
# GPU box: general-path hunk sums, two-pass dense sweeps vs sorted thresholds vs one-sweep
# tiles, over Nc (one bench line each, model_2, --path 2, HIP-graph replay) -> the defaults
# HDG_HUNK_SORTED_MIN_NC / HDG_HUNK_TILED_MIN_NC.
#   tools/hunk_crossover.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/hunk}
mkdir -p "$OUT"
line() { grep -h '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f commits/s %.4f ms/step" % (d["value"], d["ms_per_step"]))'; }
for cfg in "200 74 100" "250 150 100" "250 200 100" "250 256 64" "250 384 32" "1024 512 32" "512 768 16" "512 1024 8" "512 2048 2"; do
  set -- $cfg
  for h in dense sorted tiled; do
    tag=${1}x${2}_$h
    timeout -k 10 200 python bench.py --path 2 --ne $1 --nc $2 --batch $3 --hunk $h --steps 20 \
        --warmup 3 --no-cpu --e2e 0 > "$OUT/$tag.log" 2>&1 || exit $?
    echo "$tag $(line $OUT/$tag.log)"
  done
done
