#!/bin/bash
# Kernel timeline of a short C4 run (kernel_trace.csv kept, trimmed) for gap analysis.
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python bench.py --steps ${STEPS:-20} --warmup 5 --profile-steps 0 --no-cpu-baseline --no-ablation --no-c5 --streams "" > gpurun_out/trace_bench.json 2> gpurun_out/trace.err || { tail -20 gpurun_out/trace.err; exit 1; }
f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py "$f" ${STEPS:-20} > gpurun_out/trace_gaps.txt
true
find gpurun_out/trace -name "*kernel_trace.csv" -delete
cat gpurun_out/trace_gaps.txt | head -60
