#!/bin/bash
# Round-5 A/B of environment variants on one box, interleaved: each variant's C4 line with
# the C2 sub-line, $REPS reps (default 2).  VARIANTS: ';'-separated env assignments, an
# empty entry = the default build ("" ; "FMX_MOMENTS=1" ; ...).  Then (HOSTTIME=1) the
# default's FMX_HOST_TIMING breakdown for C4 and C2.
set -o pipefail
D=gpurun_out/r5ab
mkdir -p $D
export TMPDIR=/tmp
N=${REPS:-2}
IFS=';' read -ra VS <<< "${VARIANTS:-;FMX_LIN_ROWS=1}"
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads c2 --no-host-input"
for rep in $(seq 1 $N); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    timeout -k 10 300 env $v $B > $D/v${i}_$rep.json 2> $D/v${i}_$rep.err || { tail -20 $D/v${i}_$rep.err; exit 1; }
    python - $D/v${i}_$rep.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d['kernels_ms_per_step']; c2 = d['c2']; k2 = c2['kernels_ms_per_step']
f = lambda kk, n: kk.get(n, 0.0)
print('%-22s C4 %7.1f /s p50 %.3f match %.3f win %.3f mom %.3f rt %4.1f busy %.2f | C2 %6.1f /s p50 %.3f match %.3f win %.3f mom %.3f rt %4.1f' % (
    sys.argv[2] or 'default', d['value'], d['ms_per_step_p50'], f(k, 'match'), f(k, 'window'), f(k, 'moments'),
    d['host_round_trips_per_scan'], d['main_stream_busy_frac'], c2['value'], c2['ms_per_step_p50'], f(k2, 'match'),
    f(k2, 'window'), f(k2, 'moments'), c2['host_round_trips_per_scan']))
PY
  done
done
if [ -n "$HOSTTIME" ]; then  # every variant; LMPROF=1: with the FMX_LM_PROF build (form_amd/ab/libfmx_lmprof.so)
  [ -n "$LMPROF" ] && export FMX_LIB=$PWD/form_amd/ab/libfmx_lmprof.so
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    for w in ${HT_WORKLOADS:-c4 c2}; do
      env $v FMX_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload $w --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads= --no-host-input > $D/ht_${w}_$i.json 2> $D/ht_${w}_$i.err || { tail -20 $D/ht_${w}_$i.err; exit 1; }
      echo "== $w ${v:-default}: $(python -c "import json; d=json.loads(open('$D/ht_${w}_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step_p50'])")"
      grep "^host\|^lm " $D/ht_${w}_$i.err
    done
  done
fi
