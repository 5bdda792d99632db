# GPU box: parity tests (general path first, then the rest); stops after a crash-like exit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_general_gpu.py -q -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_general.log 2>&1
rc=$?; echo "general rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_general.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q --deselect tests/test_general_gpu.py > gpurun_out/pytest_gpu.log 2>&1
rc2=$?; echo "rest rc=$rc2"; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -15
exit $(( rc > rc2 ? rc : rc2 ))
