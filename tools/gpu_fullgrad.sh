# GPU box: the full-size gradient / Adam checks against the oracle
set -o pipefail
mkdir -p gpurun_out/fg
export PYTHONUNBUFFERED=1 HDG_PARITY_REPORT=gpurun_out/fg/parity_fullsize.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_parity.py::test_full_size_properties tests/test_fullsize_gpu.py \
    > gpurun_out/fg/pytest_fullsize.log 2>&1 || { tail -60 gpurun_out/fg/pytest_fullsize.log; exit 1; }
tail -12 gpurun_out/fg/pytest_fullsize.log
