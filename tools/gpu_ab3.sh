#!/bin/bash
# prev build vs new build (host LM) vs new build (device LM), interleaved, one box.
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
FMX_DEVICE_LM=1 timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider -k register > gpurun_out/pytest_devlm.log 2>&1 || { tail -30 gpurun_out/pytest_devlm.log; exit 1; }
tail -1 gpurun_out/pytest_devlm.log
for rep in $(seq 1 ${REPS:-2}); do
  for tag in prev host dev; do
    unset FMX_LIB FMX_DEVICE_LM
    [ $tag = prev ] && export FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so
    [ $tag = dev ] && export FMX_DEVICE_LM=1
    timeout -k 10 400 python bench.py --steps ${STEPS:-30} --warmup 10 --no-cpu-baseline > gpurun_out/ab3_$tag$rep.json 2> gpurun_out/ab3_$tag$rep.err || { tail -20 gpurun_out/ab3_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab3_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], {k: v for k, v in d['kernels_ms_per_step'].items() if v}, d['counters']['linearizations'])"
  done
done
