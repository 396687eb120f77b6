#!/bin/bash
# A/B by kernel trace: median per-step span of the C4 steady-state stream for the
# default build ("base") and form_amd/ab/libfmx_<tag>.so builds.  Usage: bash tools/gpu_ab_trace.sh tag...
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${STEPS:-60}
for rep in $(seq 1 ${REPS:-1}); do
  for tag in base "$@"; do
    if [ $tag = base ]; then unset FMX_LIB; else export FMX_LIB=$PWD/form_amd/ab/libfmx_$tag.so; fi
    rm -rf gpurun_out/trace_$tag
    timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_$tag -o run --output-format csv -- python bench.py --steps $S --warmup 5 --profile-steps 0 --no-cpu-baseline --no-ablation --no-c5 > gpurun_out/trace_$tag.json 2> gpurun_out/trace_$tag.err || { tail -20 gpurun_out/trace_$tag.err; exit 1; }
    f=$(find gpurun_out/trace_$tag -name "*kernel_trace.csv" | head -1)
    python tools/trace_gaps.py "$f" $S > gpurun_out/trace_gaps_$tag$rep.txt
    find gpurun_out/trace_$tag -name "*kernel_trace.csv" -delete
    echo "$tag: $(tail -1 gpurun_out/trace_gaps_$tag$rep.txt) | bench $(python -c "import json; print(json.load(open('gpurun_out/trace_$tag.json'))['value'])")"
  done
done
