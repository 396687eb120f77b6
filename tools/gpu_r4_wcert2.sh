#!/bin/bash
# Warm-certificate list-launch sizing: adaptive grid (debug print) vs fixed grids, C4 + C2,
# and the kernels' average durations (rocprofv3 stats, csv only).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
export FMX_LIB=$PWD/form_amd/ab/libfmx_wcert.so
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads c2 --no-host-input"
FMX_LIST_DEBUG=1 timeout -k 10 300 $B > gpurun_out/r4/g_adapt.json 2> gpurun_out/r4/g_adapt.err || { tail -20 gpurun_out/r4/g_adapt.err; exit 1; }
grep list_grid gpurun_out/r4/g_adapt.err | sort | uniq -c | sort -rn | head -12
for grid in 0 256 512 1024; do
  if [ $grid = 0 ]; then unset FMX_LIST_GRID; else export FMX_LIST_GRID=$grid; fi
  timeout -k 10 300 $B > gpurun_out/r4/g_$grid.json 2> gpurun_out/r4/g_$grid.err || { tail -20 gpurun_out/r4/g_$grid.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4/g_$grid.json')); print('grid $grid', d['value'], d['kernels_ms_per_step'].get('match'), 'c2', d['c2']['value'], d['c2']['kernels_ms_per_step'].get('match'))"
done
unset FMX_LIST_GRID
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_wcert -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline --streams "" --no-ablation --no-c5 --sub-workloads c2 --no-host-input > /tmp/prof_wcert.json 2> /tmp/prof_wcert.err || exit 1
cd $GRAFT_REPO_ROOT
f=$(find /tmp/prof_wcert -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/r4/wcert_kernel_stats.csv
python -c "import csv; r=list(csv.DictReader(open('$f'))); [print(x['Name'][:70], x['Calls'], x['AverageNs']) for x in r if 'match' in x['Name']]"
