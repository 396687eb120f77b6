#!/bin/bash
# A/B two builds on one box: form_amd/ab/libfmx_prev.so vs form_amd/libfmx.so,
# interleaved (prev, new, prev, new) so clock drift shows up.  WORKLOAD=c4|c5.
mkdir -p gpurun_out
W=${WORKLOAD:-c4}
S=${STEPS:-30}
for rep in $(seq 1 ${REPS:-2}); do
  for tag in prev new; do
    if [ $tag = prev ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so; else unset FMX_LIB; fi
    timeout -k 10 400 python bench.py --workload $W --steps $S --warmup 10 --no-cpu-baseline > gpurun_out/ab_$tag$rep.json 2> gpurun_out/ab_$tag$rep.err || { tail -20 gpurun_out/ab_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], {k: v for k, v in d['kernels_ms_per_step'].items() if v})"
  done
done
