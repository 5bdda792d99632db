# final-HEAD validation (round 4, late): GPU suite, smoke, driver-command and default bench lines, bench matrix
set -o pipefail
mkdir -p gpurun_out/val
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/val/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids "gpurun_out/val/$name.log" | tail -2 | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
HDG_PARITY_REPORT=gpurun_out/val/parity_report.json step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python __graft_entry__.py smoke
step bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 400 python bench.py
bash tools/bench_matrix.sh
