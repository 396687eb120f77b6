#!/bin/bash
# C4 only: rocprofv3 kernel trace + stats of the bench, the context stream's critical
# path (tools/critical_path.py) and the fmx kernel stats.  Outputs: gpurun_out/cpath/.
set -o pipefail
D=gpurun_out/cpath
rm -rf $D && mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --streams "" --sub-workloads= --no-host-input --no-c5 --no-ablation > $D/bench_prof.json 2> $D/prof.err || { tail -20 $D/prof.err; exit 1; }
python tools/critical_path.py $(find $D/prof -name "*kernel_trace.csv" | head -1) 40 $D/critical_path_c4.json 40 > /dev/null || exit 1
python tools/trace_gaps.py $(find $D/prof -name "*kernel_trace.csv" | head -1) > $D/trace_gaps.txt 2>&1 || true
find $D/prof -name "*kernel_trace.csv" -delete
python tools/stats_fmx.py $(find $D/prof -name "*kernel_stats.csv" | head -1) > $D/kernel_stats_fmx.csv
head -8 $D/kernel_stats_fmx.csv
cat $D/critical_path_c4.json
python -c "import json; d=json.loads(open('$D/bench_prof.json').read().strip().splitlines()[-1]); print('bench under tracer', d['value'], d['roofline']['avg_launch_us'], d['kernels_ms_per_step'])"
