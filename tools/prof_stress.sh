set -o pipefail
R=${GRAFT_REPO_ROOT}
mkdir -p $R/gpurun_out/prof_stress
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_stress/m2 -o run -- \
    python3 $R/bench.py --ne 1024 --nc 512 --batch 32 --steps 20 --warmup 3 --no-cpu --e2e 0 > $R/gpurun_out/prof_stress/m2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_stress/m4 -o run -- \
    python3 $R/bench.py --variant 4 --ne 1024 --nc 512 --batch 32 --steps 20 --warmup 3 --no-cpu --e2e 0 > $R/gpurun_out/prof_stress/m4.log 2>&1 || exit $?
echo done
