#!/bin/bash
# A/B of a HIP runtime environment setting on the default C4 bench line:
# ENVSET (e.g. "HIP_FORCE_DEV_KERNARG=1") vs unset, interleaved.
mkdir -p gpurun_out
for rep in 1 2; do
  for tag in off on; do
    if [ $tag = on ]; then E="$ENVSET"; else E=""; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-ablation > gpurun_out/env_$tag$rep.json 2> gpurun_out/env_$tag$rep.err || { tail -20 gpurun_out/env_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/env_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], d.get('sequential_extraction'), {k: v for k, v in d['kernels_ms_per_step'].items() if v})"
  done
done
