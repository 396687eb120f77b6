#!/bin/bash
# C5, per query distribution (local = the 240 m scan, wholemap = 2M distinct features
# over the whole map): rocprofv3 kernel stats, then PMC HBM traffic per kernel (one
# counter group per run, as MI355X_MICROARCH.md §rocprofv3 prescribes).
# Outputs: gpurun_out/pmc_c5_<dist>/traffic.json (+ pmc_c5_local/traffic_build.json), gpurun_out/c5_<dist>_kernel_stats_fmx.csv
set -o pipefail
export TMPDIR=/tmp
RX='k_match|k_linearize|k_map_|k_pair_scatter'
for dist in local wholemap; do
  D=gpurun_out/pmc_c5_$dist
  rm -rf $D gpurun_out/prof_c5_$dist
  mkdir -p $D
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$dist -o run --output-format csv -- python bench.py --workload c5 --c5-dist $dist --steps 10 --warmup 2 > $D/bench.json 2> $D/prof.err || { tail -20 $D/prof.err; exit 1; }
  find gpurun_out/prof_c5_$dist -name "*kernel_trace.csv" -delete
  python tools/stats_fmx.py $(find gpurun_out/prof_c5_$dist -name "*kernel_stats.csv" | head -1) > gpurun_out/c5_${dist}_kernel_stats_fmx.csv
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" -d $D/p$i -o run --output-format csv -- python bench.py --workload c5 --c5-dist $dist --steps 4 --warmup 2 > $D/p$i.json 2> $D/p$i.err || { tail -20 $D/p$i.err; exit 1; }
  done
  W=c5; [ $dist = wholemap ] && W=c5_wholemap  # the workload key bench.py looks up
  python tools/pmc_traffic.py $W $D/traffic.json $D/p1 $D/p2 $D/p3 > /dev/null
  # the map build's own summary (bench.py's c5_map_build roofline: workload key c5_build)
  [ $dist = local ] && python tools/pmc_traffic.py c5_build $D/traffic_build.json $D/p1 $D/p2 $D/p3 > /dev/null
  find $D -name "*counter_collection.csv" -delete
  cat gpurun_out/c5_${dist}_kernel_stats_fmx.csv | head -6
  python -c "
import json; d=json.load(open('$D/traffic.json'))
for k,v in d['kernels'].items(): print('$dist', k, v.get('hbm_bytes_per_launch'), v.get('l2_hit_rate'), v['launches'])"
done
