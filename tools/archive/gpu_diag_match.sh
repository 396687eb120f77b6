#!/bin/bash
# Match-kernel diagnostics on the C4 steady-state stream (block-duration spread,
# per-query candidate tail).  Usage: bash tools/gpu_diag_match.sh [bench args]
mkdir -p gpurun_out
FMX_MATCH_DIAG=1 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-c5 --no-ablation "$@" > gpurun_out/diag.json 2> gpurun_out/diag.err || { tail -30 gpurun_out/diag.err; exit 1; }
grep "match diag" gpurun_out/diag.err
python -c "import json; d=json.load(open('gpurun_out/diag.json')); print(d['value'], d['kernels_ms_per_step'], d.get('match_work_per_query'))"
