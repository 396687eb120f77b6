#!/bin/bash
# Round-5 host-input A/B: the headline (C4) bench with its host_input block, per variant
# (VARIANTS: ';'-separated env assignments, empty = default), $REPS reps interleaved;
# prints the host/device ratios (means and medians).
set -o pipefail
D=gpurun_out/r5host
mkdir -p $D
export TMPDIR=/tmp
N=${REPS:-1}
IFS=';' read -ra VS <<< "${VARIANTS:-;FMX_STAGE_ROWS=0}"
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads="
for rep in $(seq 1 $N); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    timeout -k 10 300 env $v $B > $D/h${i}_$rep.json 2> $D/h${i}_$rep.err || { tail -20 $D/h${i}_$rep.err; exit 1; }
    python - $D/h${i}_$rep.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h = d['host_input']; s = d.get('sequential_extraction') or {}
print('%-20s dev %7.1f seq %7.1f | pg_seq %7.1f pg_pipe %7.1f pin_seq %7.1f pin_pipe %7.1f | vs_dev %s | p50 %s' % (
    sys.argv[2] or 'default', d['value'], s.get('scans_per_s', 0), h['pageable_sequential']['scans_per_s'],
    h['pageable_pipelined']['scans_per_s'], h['pinned_sequential']['scans_per_s'], h['pinned_pipelined']['scans_per_s'],
    h['vs_device'], h['vs_device_p50']))
PY
  done
done
