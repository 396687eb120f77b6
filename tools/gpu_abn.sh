#!/bin/bash
# A/B of N builds on one box, interleaved REPS times: "base" = form_amd/libfmx.so, others
# form_amd/ab/libfmx_<tag>.so.  Usage: bash tools/gpu_abn.sh tag1 tag2 ...   (C4 steady state;
# WORKLOAD=c5 for the C5 line, ABARGS for extra bench flags, e.g. "--c5-dist wholemap");
# a tag "env:NAME=VALUE" runs the base library with that environment setting instead)
mkdir -p gpurun_out
S=${STEPS:-30}
for rep in $(seq 1 ${REPS:-2}); do
  for tag in base "$@"; do
    E=""
    if [ $tag = base ]; then unset FMX_LIB; elif [ "${tag#env:}" != "$tag" ]; then unset FMX_LIB; E="${tag#env:}"; else export FMX_LIB=$PWD/form_amd/ab/libfmx_$tag.so; fi
    tag=${tag//[:=]/_}
    env $E FMX_MATCH_DIAG=1 timeout -k 10 300 python bench.py --workload ${WORKLOAD:-c4} --steps $S --warmup 10 --no-cpu-baseline --no-c5 --no-ablation --streams "" $ABARGS > gpurun_out/ab_$tag$rep.json 2> gpurun_out/ab_$tag$rep.err || { tail -20 gpurun_out/ab_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], {k: v for k, v in d['kernels_ms_per_step'].items() if v}, d.get('match_work_per_query'))"
    grep "match diag: [0-9]" gpurun_out/ab_$tag$rep.err | sed 's/^/   /'
  done
done
