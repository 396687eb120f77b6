#!/bin/bash
# Regrouped warm-launch search (FMX_REGROUP): GPU match parity with the default build,
# then C4 (and C2) A/B of variant builds interleaved on one box.  Outputs gpurun_out/rg/.
set -o pipefail
D=gpurun_out/rg
mkdir -p $D
for lib in ${PLIBS:-new}; do
  if [ $lib = new ]; then unset FMX_LIB; else export FMX_LIB=$PWD/form_amd/ab/libfmx_$lib.so; fi
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mapbuild.py > $D/parity_$lib.log 2>&1 || { tail -30 $D/parity_$lib.log; exit 1; }
  echo "parity $lib: $(tail -1 $D/parity_$lib.log)"
done
for rep in $(seq 1 ${REPS:-2}); do
  for tag in ${TAGS:-rg0 new rg3 rg7}; do
    if [ $tag = new ]; then unset FMX_LIB; else export FMX_LIB=$PWD/form_amd/ab/libfmx_$tag.so; fi
    for w in ${WLS:-c4}; do
      timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 10 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams= > $D/$tag.$w.$rep.json 2> $D/$tag.$w.$rep.err || { tail -20 $D/$tag.$w.$rep.err; exit 1; }
      python -c "
import json; d=json.loads(open('$D/$tag.$w.$rep.json').read().strip().splitlines()[-1])
k=d.get('kernels_ms_per_step',{}); m=sum(v for n,v in k.items() if 'match' in n)
print('$tag $w', d['value'], 'p50', d.get('ms_per_step_p50'), 'match_ms', round(m,4), 'mw', json.dumps(d.get('match_work_per_query'))[:200])"
    done
  done
done
echo RG-DONE
