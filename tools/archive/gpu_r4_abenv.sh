#!/bin/bash
# Round 4 A/B of an environment switch: the whole GPU suite at the default, then C4 + C2
# interleaved, default vs "$1" set (e.g. FMX_NO_SPEC_LIN=1), $2 reps (default 3).
set -o pipefail
ENVSET=$1; N=${2:-3}
mkdir -p gpurun_out/r4ab
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4ab/tests_env.log 2>&1 || { tail -30 gpurun_out/r4ab/tests_env.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/r4ab/tests_env.log
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads c2 --no-host-input"
for rep in $(seq 1 $N); do
  for tag in env default; do
    if [ $tag = env ]; then E="env $ENVSET"; else E=""; fi
    timeout -k 10 300 $E $B > gpurun_out/r4ab/env_$tag$rep.json 2> gpurun_out/r4ab/env_$tag$rep.err || { tail -20 gpurun_out/r4ab/env_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4ab/env_$tag$rep.json')); k=d['kernels_ms_per_step']; k2=d['c2']['kernels_ms_per_step']; print('%-8s C4 %7.1f ms %.3f p50 %.3f match %.4f win %.4f rt %.1f | C2 %6.1f ms %.3f p50 %.3f match %.4f win %.4f' % ('$tag', d['value'], d['ms_per_step'], d['ms_per_step_p50'], k['match'], k['window'], d['host_round_trips_per_scan'], d['c2']['value'], d['c2']['ms_per_step'], d['c2']['ms_per_step_p50'], k2['match'], k2['window']))"
  done
done
