#!/bin/bash
# Round 4: PMC HBM traffic per kernel for the scan configs (C4, C2, C3), one counter
# group per run (MI355X_MICROARCH.md §rocprofv3), and the C4 match's SQ wave-state.
# Outputs: gpurun_out/pmc_r4/traffic_<w>.json, gpurun_out/pmc_r4/sq_c4.json
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/pmc_r4
rm -rf $D && mkdir -p $D
RX='k_match|k_extract_rows|k_normals|k_closest|k_fit|k_linearize|k_map_|k_insert|k_win_linearize|k_pair_scatter|k_unpack'
for w in c4 c2 c3; do
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" -d $D/$w/p$i -o run --output-format csv -- python bench.py --workload $w --steps 10 --warmup 5 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams= > $D/$w.p$i.json 2> $D/$w.p$i.err || { tail -20 $D/$w.p$i.err; exit 1; }
  done
  python tools/pmc_traffic.py $w $D/traffic_$w.json $D/$w/p1 $D/$w/p2 $D/$w/p3 > /dev/null || exit 1
  find $D/$w -name "*counter_collection.csv" -delete
  python -c "
import json; d=json.load(open('$D/traffic_$w.json'))
for k,v in d['kernels'].items(): print('$w', k, v.get('hbm_bytes_per_launch'), round(v.get('l2_hit_rate') or 0, 3), v['launches'])"
done
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex "k_match" -d $D/sq -o run --output-format csv -- python bench.py --workload c4 --steps 10 --warmup 5 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams= > $D/sq.out 2> $D/sq.err || { tail -20 $D/sq.err; exit 1; }
python tools/pmc_traffic.py c4 $D/sq_c4.json $D/sq > /dev/null || exit 1
find $D/sq -name "*counter_collection.csv" -delete
echo done
