#!/bin/bash
# Round 6: host phase times of the C4 line (FMX_HOST_TIMING + the FMX_LM_PROF build,
# form_amd/ab/libfmx_lmprof.so; both print at exit).  gpurun_out/ht6/.
set -o pipefail
D=gpurun_out/ht6
mkdir -p $D
for W in ${WORKLOADS:-c4}; do
  FMX_HOST_TIMING=1 FMX_LIB=$PWD/form_amd/ab/libfmx_lmprof.so timeout -k 10 300 python bench.py --workload $W --steps 100 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams= > $D/$W.json 2> $D/$W.err || { tail -20 $D/$W.err; exit 1; }
  python -c "import json; d=json.loads(open('$D/$W.json').read().strip().splitlines()[-1]); print('$W', d['value'], d['ms_per_step_p50'])"
  grep -E "^host|^lm" $D/$W.err
done
