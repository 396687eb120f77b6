#!/bin/bash
# C4 kernel stats (map build kernels vs round 4's)
export TMPDIR=/tmp
D=gpurun_out/diag_build
rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads= --no-host-input > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
find $D/prof -name "*kernel_trace.csv" -delete
python tools/stats_fmx.py $(find $D/prof -name "*kernel_stats.csv" | head -1) > $D/stats.csv
head -24 $D/stats.csv
timeout -k 10 300 python bench.py --workload c5 --c5-dist local --steps 3 --warmup 1 --no-cpu-baseline > $D/c5.json 2> $D/c5.err || { tail -5 $D/c5.err; exit 1; }
python -c "import json; d=json.loads(open('$D/c5.json').read().strip().splitlines()[-1]); print('c5 build', json.dumps(d.get('map_build'))[:300])"
