# GPU box: the whole gpu test suite, smoke, the bench line (+ e2e loop), phase stamps.
# Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-4}
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
HDG_PARITY_REPORT=gpurun_out/parity_report.json step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench 600 python bench.py --e2e 50
step phases 200 python tools/mid_phases.py
