# GPU box: per-phase stamps of k_commit_step + SQ instruction-mix counters.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/mid_phases.py > gpurun_out/phases.log 2>&1; rc=$?
echo "phases rc=$rc"; grep -v amdgpu.ids gpurun_out/phases.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_sq.sh > gpurun_out/pmc_sq.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -30 gpurun_out/pmc_sq.log; exit $rc
