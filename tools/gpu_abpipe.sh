#!/bin/bash
# GPU tests, then A/B of the default (pipelined) bench line: form_amd/ab/libfmx_prev.so vs this build.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for tag in prev new; do
    if [ $tag = prev ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so; else unset FMX_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-ablation > gpurun_out/abp_$tag$rep.json 2> gpurun_out/abp_$tag$rep.err || { tail -20 gpurun_out/abp_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abp_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], d['gpu_busy_frac'], d.get('sequential_extraction'), {k: v for k, v in d['kernels_ms_per_step'].items() if v})"
  done
done
