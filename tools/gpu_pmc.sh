#!/bin/bash
# PMC passes (one counter group per run; no trace domains combined with --pmc).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
RX='k_match|k_extract_rows|k_normals|k_closest|k_fit|k_linearize|k_map_|k_insert|k_win_linearize|k_pair_scatter'
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc/p$i
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" -d gpurun_out/pmc/p$i -o run --output-format csv -- python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-c5 --no-ablation > gpurun_out/pmc/p$i.json 2> gpurun_out/pmc/p$i.err || { tail -20 gpurun_out/pmc/p$i.err; exit 1; }
done
python tools/pmc_traffic.py c4 gpurun_out/pmc/traffic.json gpurun_out/pmc/p1 gpurun_out/pmc/p2 gpurun_out/pmc/p3 > /dev/null
find gpurun_out/pmc -name "*counter_collection.csv" -delete
cat gpurun_out/pmc/traffic.json | head -80
