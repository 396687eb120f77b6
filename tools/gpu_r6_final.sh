#!/bin/bash
# Round 6, final sources: the GPU suite, then (only if it passed) the profiling part of
# the end-of-round script (kernel stats, critical paths, smoke).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_gpu_suite_final.log 2>&1
tail -3 gpurun_out/r6_gpu_suite_final.log
grep -q " passed" gpurun_out/r6_gpu_suite_final.log && ! grep -q "failed" gpurun_out/r6_gpu_suite_final.log || exit 1
PART=prof bash tools/gpu_r6_end.sh > gpurun_out/end6_prof2.log 2>&1
tail -12 gpurun_out/end6_prof2.log
