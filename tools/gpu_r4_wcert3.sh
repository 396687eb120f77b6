#!/bin/bash
# Warm certificate, final A/B: default build vs FMX_WARM_CERT one launch (certified
# queries skip the search) vs the split (FMX_CERT_SPLIT: certify, then 64 lanes per
# listed query); parity of the one-launch mode first.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
FMX_LIB=$PWD/form_amd/ab/libfmx_wcert.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_map.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py > gpurun_out/r4/wcert3_tests.log 2>&1 || { tail -30 gpurun_out/r4/wcert3_tests.log; exit 1; }
tail -1 gpurun_out/r4/wcert3_tests.log
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads c2 --no-host-input"
for rep in 1 2 3; do
  for tag in base one split; do
    unset FMX_LIB FMX_CERT_SPLIT FMX_LIST_GRID
    if [ $tag != base ]; then export FMX_LIB=$PWD/form_amd/ab/libfmx_wcert.so; fi
    if [ $tag = split ]; then export FMX_CERT_SPLIT=1 FMX_LIST_GRID=1024; fi
    timeout -k 10 300 $B > gpurun_out/r4/w3_$tag$rep.json 2> gpurun_out/r4/w3_$tag$rep.err || { tail -20 gpurun_out/r4/w3_$tag$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4/w3_$tag$rep.json')); print('$tag', d['value'], d['ms_per_step'], d['kernels_ms_per_step'].get('match'), 'c2', d['c2']['value'], d['c2']['kernels_ms_per_step'].get('match'))"
  done
done
unset FMX_LIB FMX_CERT_SPLIT FMX_LIST_GRID
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_base -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads c2 --no-host-input > /tmp/prof_base.json 2> /tmp/prof_base.err || exit 1
cd $GRAFT_REPO_ROOT
f=$(find /tmp/prof_base -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/r4/base_kernel_stats.csv
python -c "import csv; r=list(csv.DictReader(open('$f'))); [print(x['Name'][:70], x['Calls'], x['AverageNs']) for x in r if 'fmx' in x['Name']]"
