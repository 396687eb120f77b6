#!/bin/bash
# Round 6: A/B of form_amd/ab/libfmx_prev.so vs form_amd/libfmx.so on the C4 line with the
# concurrent-streams block (2 and 4 contexts on one GPU), interleaved.  gpurun_out/r6st/.
set -o pipefail
D=gpurun_out/r6st
mkdir -p $D
for rep in $(seq 1 ${REPS:-2}); do
  for tag in prev new; do
    if [ $tag = prev ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so; else unset FMX_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams 2,4 > $D/$tag$rep.json 2> $D/$tag$rep.err || { tail -20 $D/$tag$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$D/$tag$rep.json').read().strip().splitlines()[-1]); c=d['concurrent_streams']; print('$tag', d['value'], 'p50', d['ms_per_step_p50'], 'streams2', c['2']['scans_per_s'], 'streams4', c['4']['scans_per_s'])"
  done
done
echo STREAMS-DONE
