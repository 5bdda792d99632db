# GPU box: interleaved bench lines of env-knob variants ("tag|ENV=.. ENV=.."), $BARGS added
set -o pipefail
O=gpurun_out/envab; mkdir -p $O
for rep in 1 2 3; do
  for spec in "$@"; do
    tag=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 200 python bench.py --no-cpu --e2e 0 --steps ${STEPS:-20} --warmup 5 $BARGS > $O/$tag.$rep.log 2>&1 || exit 1
    grep -h '^{' $O/$tag.$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' $tag
  done
done
