# GPU box, end of round 6, part $1:
#   a: the whole gpu test suite (parity report), smoke, the driver's bench command, the
#      default bench line (e2e loop + CPU baseline)
#   b: the bench matrix of every workload, bench.py --gpus 2 / 4 on the one device, phases
set -o pipefail
mkdir -p gpurun_out/final
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/final/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/final/$name.log" | tail -${TAILN:-3} | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ "$1" = a ]; then
  HDG_PARITY_REPORT=gpurun_out/final/parity_report.json step pytest_gpu 1000 \
      python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread
  step smoke 300 python __graft_entry__.py smoke
  step bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step bench_default 600 python bench.py
else
  bash tools/bench_matrix.sh || exit $?
  step bench_gpus2 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --e2e 0
  step bench_gpus4 300 python bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu --e2e 0
  step phases 200 python tools/mid_phases.py
fi
