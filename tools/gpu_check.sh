# GPU box: new tests first (verbose), then the full GPU suite, smoke and a short bench.
set -o pipefail
mkdir -p gpurun_out
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -n "$FIRST" ]; then
  step first 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread $FIRST
fi
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench 600 python bench.py ${BENCH_ARGS:---no-cpu --e2e 0}
