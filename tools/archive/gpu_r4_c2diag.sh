#!/bin/bash
# C2 host-time diagnosis: host phase timers (FMX_HOST_TIMING) + LM phase timers (the
# FMX_LM_PROF build), then a rocprofv3 kernel trace -> the context stream's share.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
B="--steps 40 --warmup 10 --no-cpu-baseline --streams '' --no-ablation --no-c5 --sub-workloads '' --no-host-input"
for wl in c2 c4; do
  FMX_HOST_TIMING=1 FMX_LIB=$PWD/form_amd/ab/libfmx_lmprof.so timeout -k 10 300 python bench.py --workload $wl --steps 40 --warmup 10 --no-cpu-baseline --streams "" --no-ablation --no-c5 --sub-workloads "" --no-host-input > gpurun_out/r4/diag_$wl.json 2> gpurun_out/r4/diag_$wl.err || { tail -20 gpurun_out/r4/diag_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4/diag_$wl.json')); print('$wl', d['value'], d['ms_per_step'], d['counters'], d['kernels_ms_per_step'])"
  grep -E "^host|^lm" gpurun_out/r4/diag_$wl.err
done
rm -rf gpurun_out/r4/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4/prof_c2 -o run --output-format csv -- python bench.py --workload c2 --steps 40 --warmup 10 --no-cpu-baseline --streams "" --no-ablation --no-c5 --sub-workloads "" --no-host-input > gpurun_out/r4/c2_trace_bench.json 2> gpurun_out/r4/c2_trace.err || { tail -20 gpurun_out/r4/c2_trace.err; exit 1; }
python tools/critical_path.py $(find gpurun_out/r4/prof_c2 -name "*kernel_trace.csv" | head -1) 40 gpurun_out/r4/critical_path_c2.json 40 && cat gpurun_out/r4/critical_path_c2.json
python tools/trace_gaps.py $(find gpurun_out/r4/prof_c2 -name "*kernel_trace.csv" | head -1) > gpurun_out/r4/c2_trace_gaps.txt 2>&1 || true
find gpurun_out/r4/prof_c2 -name "*kernel_trace.csv" -delete
# warm-certificate diagnostic (FMX_CERT_DIAG build): C4 and C2, the profiled pass's matches
for wl in c4 c2; do
  FMX_MATCH_DIAG=1 FMX_LIB=$PWD/form_amd/ab/libfmx_cert.so timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --streams "" --no-ablation --no-c5 --sub-workloads "" --no-host-input > gpurun_out/r4/cert_$wl.json 2> gpurun_out/r4/cert_$wl.err || { tail -20 gpurun_out/r4/cert_$wl.err; exit 1; }
  echo "cert $wl"; grep "match diag" gpurun_out/r4/cert_$wl.err
done
