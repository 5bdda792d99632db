# GPU box: prepared tables of the current build vs a reference build (copy the older
# libhdgnn.so to hd-gnn_amd/csrc/libhdgnn_old.so first),
# bytewise; then the GPU parity tests and a kernel trace of the stress prepare.
set -o pipefail
mkdir -p gpurun_out/prep
timeout -k 10 300 env HDG_LIB_PATH=$PWD/hd-gnn_amd/csrc/libhdgnn_old.so python tools/prep_dump.py gpurun_out/prep/old.npz > gpurun_out/prep/old.log 2>&1 || { echo old failed; tail gpurun_out/prep/old.log; exit 1; }
timeout -k 10 300 python tools/prep_dump.py gpurun_out/prep/new.npz > gpurun_out/prep/new.log 2>&1 || { echo new failed; tail gpurun_out/prep/new.log; exit 1; }
python - <<'PY' || exit 1
import numpy as np
a = np.load("gpurun_out/prep/old.npz"); b = np.load("gpurun_out/prep/new.npz")
bad = 0
for k in a.files:
    d = np.flatnonzero(a[k] != b[k])
    print(k, a[k].size, "words differ:", d.size, d[:8])
    bad += d.size
print("PREP_BYTEWISE", "OK" if bad == 0 else "MISMATCH")
raise SystemExit(0 if bad == 0 else 1)
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/prep/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/prep/pytest.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prep/prof_m2 -o run -- \
    python3 $R/bench.py --ne 1024 --nc 512 --batch 32 --steps 10 --warmup 2 --no-cpu --e2e 0 > $R/gpurun_out/prep/m2_stress.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prep/prof_glide -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --e2e 0 > $R/gpurun_out/prep/glide.log 2>&1 || exit $?
grep -h prep $R/gpurun_out/prep/prof_m2/run_kernel_stats.csv $R/gpurun_out/prep/prof_glide/run_kernel_stats.csv
