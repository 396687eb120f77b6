#!/bin/bash
# Round 6: interleaved env-variant A/B on the headline stream (VARIANTS ';'-separated env
# assignments, empty = default), WORKLOADS, REPS.
set -o pipefail
D=gpurun_out/r6env
mkdir -p $D
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for W in ${WORKLOADS:-c4}; do
  for rep in $(seq 1 ${REPS:-2}); do
    i=0
    for v in "${VS[@]}"; do
      i=$((i+1))
      timeout -k 10 300 env $v python bench.py --workload $W --steps ${STEPS:-60} --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads= --no-host-input > $D/e_${W}_$i$rep.json 2> $D/e_${W}_$i$rep.err || { tail -20 $D/e_${W}_$i$rep.err; exit 1; }
      python -c "import json; d=json.loads(open('$D/e_${W}_$i$rep.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$W %-32s' % '${v:-default}', d['value'], 'p50', d.get('ms_per_step_p50'), {x: k[x] for x in ('match','pair_sort','window','extract_rows','fit') if x in k})"
    done
  done
done
echo ENV-DONE
