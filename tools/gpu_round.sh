# GPU box: parity tests, smoke, full bench line (with the CPU baseline), rocprofv3 evidence.
# Stops at the first crash-like exit (abort / segfault / timeout).
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
step() {   # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-8}
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step smoke 300 python __graft_entry__.py smoke
step bench_full 900 python bench.py
bash tools/profile.sh $TAG; rc=$?; echo "profile rc=$rc"; exit $rc
