# GPU box: end-of-round evidence -- gpu_full.sh (suite, smoke, bench lines, phases), then
# the split-mode soak (tools/soak.py) at glide for model_2 / model_4 and at stress.
set -o pipefail
bash tools/gpu_full.sh || exit $?
rm -f gpurun_out/soak.json
timeout -k 10 300 python tools/soak.py --variant 2 --steps 20000 > gpurun_out/soak_m2.log 2>&1 || { tail -5 gpurun_out/soak_m2.log; exit 1; }
timeout -k 10 300 python tools/soak.py --variant 4 --steps 5000 > gpurun_out/soak_m4.log 2>&1 || { tail -5 gpurun_out/soak_m4.log; exit 1; }
timeout -k 10 300 python tools/soak.py --variant 2 --ne 1024 --nc 512 --batch 32 --steps 1000 > gpurun_out/soak_stress.log 2>&1 || { tail -5 gpurun_out/soak_stress.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/soak.json'):
    d = json.loads(l); r = d['runs']
    print('soak v%d %dx%d B%d %d steps: no_fault %s bitwise_equal %s split %s loss %.6f %.4f ms/step' % (d['variant'], d['ne'], d['nc'], d['batch'], d['steps'], d['no_fault'], d['bitwise_equal'], r[0]['split'], r[0]['loss'], r[0]['ms_per_step']))
"
