set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu --e2e 0 > gpurun_out/b0.log 2>&1 && \
timeout -k 10 200 python tools/mid_phases.py > gpurun_out/ph0.log 2>&1
echo rc=$?
