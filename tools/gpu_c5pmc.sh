#!/bin/bash
# C5: bench line, rocprofv3 kernel stats, PMC HBM traffic per kernel (separate passes)
mkdir -p gpurun_out/pmc_c5
export TMPDIR=/tmp
bash tools/gpu_c5prof.sh || exit 1
python tools/stats_fmx.py $(find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -1) > gpurun_out/c5_kernel_stats_fmx.csv
RX='k_match|k_linearize|k_map_|k_pair_scatter'
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_c5/p$i
  timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" -d gpurun_out/pmc_c5/p$i -o run --output-format csv -- python bench.py --workload c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_c5/p$i.json 2> gpurun_out/pmc_c5/p$i.err || { tail -20 gpurun_out/pmc_c5/p$i.err; exit 1; }
done
python tools/pmc_traffic.py c5 gpurun_out/pmc_c5/traffic.json gpurun_out/pmc_c5/p1 gpurun_out/pmc_c5/p2 gpurun_out/pmc_c5/p3 > /dev/null
find gpurun_out/pmc_c5 -name "*counter_collection.csv" -delete
cat gpurun_out/c5.json
cat gpurun_out/c5_kernel_stats_fmx.csv
python -c "
import json; d=json.load(open('gpurun_out/pmc_c5/traffic.json'))
for k,v in d['kernels'].items(): print(k, v.get('hbm_bytes_per_launch'), v.get('l2_hit_rate'), v['launches'])"
