# GPU box: parity tests, per-phase stamps, bench.  Stops at the first crash-like exit
# (abort / segfault / timeout); an ordinary test failure (rc 1) still lets the rest run.
set -o pipefail
mkdir -p gpurun_out
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-25}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step phases 300 python tools/mid_phases.py
step bench 300 python bench.py --steps 50 --warmup 10 --no-cpu --e2e 0
