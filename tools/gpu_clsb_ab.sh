# GPU box: balanced-piece kw_ee_clsb candidates (ab_<tag>.so, tags as arguments): the model_4
# parity tests per candidate, then interleaved model_4 glide (hybrid and general) and model_4
# stress bench lines against the in-tree libhdgnn.so ("orig").  TESTS=none: benches only.
set -o pipefail
mkdir -p gpurun_out/clsb
lp() { if [ $1 = orig ]; then echo ""; else echo "$(pwd)/hd-gnn_amd/csrc/ab_$1.so"; fi; }
for tag in "$@"; do
  [ "$TESTS" = none ] && break
  HDG_LIB_PATH=$(lp $tag) timeout -k 10 500 python -u -m pytest -x -q --timeout 200 \
      --timeout-method thread tests/test_general_gpu.py tests/test_fullsize_gpu.py \
      -k "${TK:-4}" > gpurun_out/clsb/$tag.tests.log 2>&1 \
      || { tail -30 gpurun_out/clsb/$tag.tests.log; exit 1; }
  echo "$tag tests: $(tail -1 gpurun_out/clsb/$tag.tests.log)"
done
if [ -n "$M2" ]; then   # M2=1: model_2 general-path lines too
  CFGS=("glide:--variant 4" "general:--variant 4 --path 2" "stress:--variant 4 --ne 1024 --nc 512 --batch 32"
        "m2gen:--variant 2 --path 2" "m2stress:--variant 2 --ne 1024 --nc 512 --batch 32")
else
  CFGS=("glide:--variant 4" "general:--variant 4 --path 2" "stress:--variant 4 --ne 1024 --nc 512 --batch 32")
fi
for rep in 1 2; do
  for tag in orig "$@"; do
    for cfg in "${CFGS[@]}"; do
      name=${cfg%%:*}; args=${cfg#*:}
      HDG_LIB_PATH=$(lp $tag) timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps 20 --warmup 5 $args \
          > gpurun_out/clsb/$tag.$name.log 2>&1 || { tail -5 gpurun_out/clsb/$tag.$name.log; exit 1; }
      grep -h '^{' gpurun_out/clsb/$tag.$name.log | python3 -c '
import json, sys
d = json.loads(sys.stdin.read()); s = d.get("steady_state") or {}; k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], "steady", s.get("value"), s.get("ms_per_step"),
      "clsb", k.get("kw_ee_clsb"), "eefwd", k.get("kw_ee_fwd"), "scan", k.get("kw_scan"))' $tag $name
    done
  done
done
