#!/bin/bash
# Round 6: the GPU suite at the current build (steps bounded, stops at a crash), then an
# interleaved A/B of form_amd/ab/libfmx_prev.so vs form_amd/libfmx.so (WORKLOADS, REPS).
set -o pipefail
D=gpurun_out/r6chk
mkdir -p $D
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  bash tools/gpu_tests.sh $D/tests "tests -m gpu ${TESTARGS}" || exit 1
  grep -q " passed" $D/tests/step1.log && ! grep -q " failed" $D/tests/step1.log || { grep -E "FAILED|Error" $D/tests/step1.log | head -20; exit 1; }
fi
for W in ${WORKLOADS:-c4 c2}; do
  for rep in $(seq 1 ${REPS:-2}); do
    for tag in prev new; do
      if [ $tag = prev ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so; else unset FMX_LIB; fi
      timeout -k 10 300 python bench.py --workload $W --steps ${STEPS:-60} --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads= --no-host-input > $D/ab_${W}_$tag$rep.json 2> $D/ab_${W}_$tag$rep.err || { tail -20 $D/ab_${W}_$tag$rep.err; exit 1; }
      python -c "import json; d=json.loads(open('$D/ab_${W}_$tag$rep.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$W $tag', d['value'], 'p50', d.get('ms_per_step_p50'), {x: k[x] for x in ('match','pair_sort','window') if x in k})"
    done
  done
done
echo CHECK-DONE
