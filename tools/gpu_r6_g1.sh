set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 120 ./tools/flagbench/sessionbench > gpurun_out/r6/sessionbench.txt 2>&1 || { cat gpurun_out/r6/sessionbench.txt; exit 1; }
cat gpurun_out/r6/sessionbench.txt
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads=c2 --no-host-input > gpurun_out/r6/base_c4.json 2> gpurun_out/r6/base_c4.err || { tail -20 gpurun_out/r6/base_c4.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r6/base_c4.json').read().strip().splitlines()[-1])
print('C4', d['value'], d.get('ms_per_step_p50'), d.get('kernels_ms_per_step'))
print('C2', d['c2']['value'], d['c2'].get('ms_per_step_p50'))
"
