#!/bin/bash
# Round 4 A/B: the parity tests through the default build, then C4 + C2 interleaved,
# default (libfmx.so) vs the variant form_amd/ab/libfmx_$1.so, $2 reps (default 3).
set -o pipefail
V=$1; N=${2:-3}
mkdir -p gpurun_out/r4ab
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_map.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py > gpurun_out/r4ab/tests_$V.log 2>&1 || { tail -30 gpurun_out/r4ab/tests_$V.log; exit 1; }
tail -1 gpurun_out/r4ab/tests_$V.log
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads c2 --no-host-input"
for rep in $(seq 1 $N); do
  for tag in $V default; do
    unset FMX_LIB
    if [ $tag != default ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_$tag.so; fi
    timeout -k 10 300 $B > gpurun_out/r4ab/${V}_$tag$rep.json 2> gpurun_out/r4ab/${V}_$tag$rep.err || { tail -20 gpurun_out/r4ab/${V}_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4ab/${V}_$tag$rep.json')); k=d['kernels_ms_per_step']; k2=d['c2']['kernels_ms_per_step']; print('%-8s C4 %7.1f match %.4f pair %.4f win %.4f | C2 %6.1f match %.4f pair %.4f win %.4f' % ('$tag', d['value'], k['match'], k['pair_sort'], k['window'], d['c2']['value'], k2['match'], k2['pair_sort'], k2['window']))"
  done
done
