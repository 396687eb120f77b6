#!/bin/bash
# GPU tests, then C4 (match diag) and C5 bench A/B: form_amd/ab/libfmx_prev.so vs this build.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
REPS=${REPS:-2} bash tools/gpu_abn.sh prev || exit 1
for rep in 1 2; do
  for tag in prev new; do
    if [ $tag = prev ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so; else unset FMX_LIB; fi
    timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_$tag$rep.json 2> gpurun_out/c5_$tag$rep.err || { tail -20 gpurun_out/c5_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/c5_$tag$rep.json')); print('c5 $tag', d['value'], d['ms_per_step'], {k: v for k, v in d.get('kernels_ms_per_step', {}).items() if v}, d.get('match_work_per_query'))"
  done
done
