#!/bin/bash
# C5 A/B of builds: TAGS (default "g4 g2") — "g4" = this build (form_amd/libfmx.so), any
# other tag = form_amd/ab/libfmx_<tag>.so — after the large-query-set parity tests on
# form_amd/ab/libfmx_$TEST_TAG.so.
mkdir -p gpurun_out
FMX_LIB=$PWD/form_amd/ab/libfmx_${TEST_TAG:-g2}.so timeout -k 10 400 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_parity.py -k "c5 or large or C5" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_g2.log 2>&1 || { tail -40 gpurun_out/pytest_g2.log; exit 1; }
tail -1 gpurun_out/pytest_g2.log
for rep in 1 2; do
  for tag in ${TAGS:-g4 g2}; do
    if [ $tag = g4 ]; then unset FMX_LIB; else export FMX_LIB=$PWD/form_amd/ab/libfmx_$tag.so; fi
    timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_$tag$rep.json 2> gpurun_out/c5_$tag$rep.err || { tail -20 gpurun_out/c5_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/c5_$tag$rep.json')); print('c5 $tag', d['value'], d['ms_per_step'], {k: v for k, v in d.get('kernels_ms_per_step', {}).items() if v}, d.get('match_work_per_query'))"
  done
done
