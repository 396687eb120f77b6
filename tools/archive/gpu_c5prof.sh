#!/bin/bash
# C5 bench + rocprofv3 kernel stats (stats CSV only kept)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload c5 --steps 10 --warmup 5 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
rm -rf gpurun_out/prof_c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python bench.py --workload c5 --steps 10 --warmup 5 > /dev/null 2> gpurun_out/prof_c5.err || { tail -5 gpurun_out/prof_c5.err; exit 1; }
find gpurun_out/prof_c5 -name "*kernel_trace.csv" -delete
