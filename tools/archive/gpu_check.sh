#!/bin/bash
# GPU round trip: parity tests, bench, rocprofv3 kernel stats (stats CSV only kept).
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 30 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --kernel-include-regex "fmx::" -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/prof.err || { tail -20 gpurun_out/prof.err; exit 1; }
  find gpurun_out/prof -name "*kernel_trace.csv" -delete
  find gpurun_out/prof -name "*stats.csv" | head -5
  cut -d, -f1-8 $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) | head -25
fi
