#!/bin/bash
# Host-side time per call site (FMX_HOST_TIMING, printed at exit), C4 and C2 streams.
set -o pipefail
mkdir -p gpurun_out/r4
for w in c4 c2; do
  FMX_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload $w --steps 40 --warmup 10 --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads= --no-host-input > gpurun_out/r4/ht_$w.json 2> gpurun_out/r4/ht_$w.err || { tail -20 gpurun_out/r4/ht_$w.err; exit 1; }
  echo "== $w"; grep "^host" gpurun_out/r4/ht_$w.err
done
