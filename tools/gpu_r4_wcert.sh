#!/bin/bash
# The warm-certificate build (FMX_WARM_CERT: certified warm queries skip the search):
# the match parity tests through it, then an interleaved A/B against the default build.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
FMX_LIB=$PWD/form_amd/ab/libfmx_wcert.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_map.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py > gpurun_out/r4/wcert_tests.log 2>&1 || { tail -30 gpurun_out/r4/wcert_tests.log; exit 1; }
tail -2 gpurun_out/r4/wcert_tests.log
for rep in 1 2; do
  for tag in base wcert; do
    if [ $tag = wcert ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_wcert.so; else unset FMX_LIB; fi
    FMX_MATCH_DIAG=1 timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams "" --no-ablation --no-c5 --sub-workloads c2 --no-host-input > gpurun_out/r4/ab_$tag$rep.json 2> gpurun_out/r4/ab_$tag$rep.err || { tail -20 gpurun_out/r4/ab_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4/ab_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], {k: v for k, v in d['kernels_ms_per_step'].items() if v}, 'c2', d['c2']['value'], d['c2']['kernels_ms_per_step'].get('match'))"
    grep "warm certificate\|span" gpurun_out/r4/ab_$tag$rep.err | head -4
  done
done
export FMX_LIB=$PWD/form_amd/ab/libfmx_wcert.so
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_wcert -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams "" --no-ablation --no-c5 --sub-workloads c2 --no-host-input > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_wcert.json 2> $GRAFT_REPO_ROOT/gpurun_out/r4/prof_wcert.err || exit 1
cd $GRAFT_REPO_ROOT
find gpurun_out/r4/prof_wcert -name "*kernel_stats.csv" | head -1 | xargs -I{} python -c "import csv,sys; r=list(csv.DictReader(open('{}'))); [print(x['Name'][:60], x['Calls'], x['AverageNs']) for x in r if 'match' in x['Name']]"
