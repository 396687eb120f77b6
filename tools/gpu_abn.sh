#!/bin/bash
# Best-of-N A/B of named variants on one box.  VARIANTS="name:ENV=val,ENV2=val ..."
# ("prev" in a name selects form_amd/ab/libfmx_prev.so).  Prints each run and the
# best (max scans/s) per variant: host jitter is additive, so the best run is the
# stable statistic.
mkdir -p gpurun_out
V=${VARIANTS:-"prev: new:"}
for rep in $(seq 1 ${REPS:-3}); do
  for spec in $V; do
    name=${spec%%:*}; envs=${spec#*:}
    for v in $(env | grep -o "^FMX_[A-Z_]*"); do unset $v; done
    case $name in prev*) export FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so;; esac
    [ -f form_amd/ab/libfmx_$name.so ] && export FMX_LIB=$PWD/form_amd/ab/libfmx_$name.so
    for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 400 python bench.py --workload ${WORKLOAD:-c4} --steps ${STEPS:-30} --warmup 10 --no-cpu-baseline > gpurun_out/abn_$name$rep.json 2> gpurun_out/abn_$name$rep.err || { tail -20 gpurun_out/abn_$name$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abn_$name$rep.json')); print('$name', d['value'], d['ms_per_step'], {k: v for k, v in d['kernels_ms_per_step'].items() if v})"
  done
done
python - <<'PY'
import glob, json, re, collections
best = collections.defaultdict(float)
for f in glob.glob('gpurun_out/abn_*.json'):
    name = re.match(r'gpurun_out/abn_(.*)(\d)\.json', f).group(1)
    best[name] = max(best[name], json.load(open(f))['value'])
print('BEST', dict(best))
PY
