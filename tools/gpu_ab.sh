#!/bin/bash
# A/B of voxel_subdivision on C4 and C5 (bench lines only), after the GPU tests.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for s in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --subdiv $s > gpurun_out/ab_c4_$s.json 2> gpurun_out/ab_c4_$s.err || { tail -20 gpurun_out/ab_c4_$s.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_c4_$s.json')); print('c4 subdiv $s', d['value'], d['ms_per_step'], d.get('kernels_ms_per_step'), d.get('match_work_per_query'))"
done
for s in 1 2; do
  timeout -k 10 400 python bench.py --workload c5 --steps 10 --warmup 5 --no-cpu-baseline --subdiv $s > gpurun_out/ab_c5_$s.json 2> gpurun_out/ab_c5_$s.err || { tail -20 gpurun_out/ab_c5_$s.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_c5_$s.json')); print('c5 subdiv $s', d['value'], d['ms_per_step'], d.get('kernels_ms_per_step'), d.get('match_work_per_query'))"
done
