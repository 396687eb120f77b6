#!/bin/bash
# (the A side: make -C form_amd/csrc BUILD=build_nocert OUT=../ab/libfmx_nocert.so EXTRA=-DFMX_WARM_CERT=0)
# The warm certificate as the default build: the whole GPU suite, then an interleaved
# A/B against the build without it (libfmx_nocert, FMX_WARM_CERT=0), C4 + C2.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4/certdef_tests.log 2>&1 || { tail -40 gpurun_out/r4/certdef_tests.log; exit 1; }
tail -1 gpurun_out/r4/certdef_tests.log
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads c2 --no-host-input"
for rep in 1 2 3; do
  for tag in nocert cert; do
    unset FMX_LIB
    if [ $tag = nocert ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_nocert.so; fi
    timeout -k 10 300 $B > gpurun_out/r4/cd_$tag$rep.json 2> gpurun_out/r4/cd_$tag$rep.err || { tail -20 gpurun_out/r4/cd_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4/cd_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], d['kernels_ms_per_step'].get('match'), 'c2', d['c2']['value'], d['c2']['kernels_ms_per_step'].get('match'))"
  done
done
