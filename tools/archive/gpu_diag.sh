#!/bin/bash
# Latency diagnostics of the smoothing-mode step: window-kernel phase stamps
# (FMX_WIN_TIMING), host phase timers (FMX_HOST_TIMING), kernel trace gaps.
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --profile-steps 0 --no-cpu-baseline --no-ablation"
FMX_WIN_TIMING=1 timeout -k 10 300 $B > gpurun_out/wt.json 2> gpurun_out/wt.err || { tail -20 gpurun_out/wt.err; exit 1; }
FMX_HOST_TIMING=1 timeout -k 10 300 $B > gpurun_out/ht.json 2> gpurun_out/ht.err || { tail -20 gpurun_out/ht.err; exit 1; }
grep -v amdgpu.ids gpurun_out/wt.err
grep -v amdgpu.ids gpurun_out/ht.err
python -c "import json; d=json.load(open('gpurun_out/ht.json')); print('ht', d['value'])"
bash tools/gpu_trace.sh
