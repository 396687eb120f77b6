#!/bin/bash
# Round-5 end-of-round evidence at HEAD, in two parts (one gpurun
# call each, ~10-15 min):
#   PART=scan : PMC HBM traffic per kernel for C4 / C2 / C3 (one counter group per run),
#               the C4 match's SQ wave-state, and the context-stream critical path + fmx
#               kernel stats of C4 and C2 (rocprofv3 --kernel-trace --stats)
#   PART=c5   : tools/gpu_c5pmc.sh (C5 local / wholemap traffic + the map build's) and the
#               whole-map fused match's SQ wave-state
# Every summary is stamped with the hashes of the sources it measured (tools/provenance.py).
# Outputs under gpurun_out/ev5/.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/ev5
mkdir -p $D
B="--steps 10 --warmup 5 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams="
RX='k_match|k_extract_rows|k_normals|k_closest|k_fit|k_linearize|k_map_|k_insert|k_win_|k_pair_scatter|k_unpack'
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
if [ "${PART:-scan}" = scan ]; then
  [ "${PMC:-1}" = 1 ] && for w in ${WORKLOADS:-c4 c2 c3}; do
    i=0
    for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      rm -rf $D/$w/p$i
      timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" -d $D/$w/p$i -o run --output-format csv -- python bench.py --workload $w $B > $D/$w.p$i.json 2> $D/$w.p$i.err || { tail -20 $D/$w.p$i.err; exit 1; }
    done
    python tools/pmc_traffic.py $w $D/traffic_$w.json $D/$w/p1 $D/$w/p2 $D/$w/p3 > /dev/null || exit 1
    find $D/$w -name "*counter_collection.csv" -delete
    python -c "
import json; d=json.load(open('$D/traffic_$w.json'))
for k,v in d['kernels'].items(): print('$w', k, v.get('hbm_bytes_per_launch'), round(v.get('l2_hit_rate') or 0, 3), v['launches'])"
  done
  if [ "${PMC:-1}" = 1 ]; then
    rm -rf $D/sq_c4
    timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex "k_match" -d $D/sq_c4 -o run --output-format csv -- python bench.py --workload c4 $B > $D/sq_c4.out 2> $D/sq_c4.err || { tail -20 $D/sq_c4.err; exit 1; }
    python tools/pmc_traffic.py c4 $D/sq_wavestate_c4.json $D/sq_c4 > /dev/null || exit 1
    find $D/sq_c4 -name "*counter_collection.csv" -delete
  fi
  for w in ${CPATH:-c4 c2}; do
    rm -rf $D/prof_$w
    # --steps 40 (+ a 40-scan profile pass after them: skip 40)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$w -o run --output-format csv -- python bench.py --workload $w --steps 40 --warmup 10 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams= > $D/bench_prof_$w.json 2> $D/prof_$w.err || { tail -20 $D/prof_$w.err; exit 1; }
    T=$(find $D/prof_$w -name "*kernel_trace.csv" | head -1)
    python tools/critical_path.py $T 40 $D/critical_path_$w.json 40 > /dev/null || exit 1
    python tools/trace_gaps.py $T > $D/trace_gaps_$w.txt 2>&1 || true
    find $D/prof_$w -name "*kernel_trace.csv" -delete
    python tools/stats_fmx.py $(find $D/prof_$w -name "*kernel_stats.csv" | head -1) > $D/${w}_kernel_stats_fmx.csv
    head -8 $D/${w}_kernel_stats_fmx.csv
    python -c "import json; d=json.load(open('$D/critical_path_$w.json')); print('$w', {k: d[k] for k in d if not isinstance(d[k], (list, dict))})"
  done
else
  bash tools/gpu_c5pmc.sh || exit 1
  for dist in local wholemap; do
    cp gpurun_out/pmc_c5_$dist/traffic.json $D/traffic_c5_$dist.json
    cp gpurun_out/c5_${dist}_kernel_stats_fmx.csv $D/c5_${dist}_kernel_stats_fmx.csv
  done
  cp gpurun_out/pmc_c5_local/traffic_build.json $D/traffic_c5_build.json
  WORKLOADS=c5_wholemap bash tools/gpu_sqpmc.sh || exit 1
  cp gpurun_out/sq/c5_wholemap.json $D/sq_wavestate_c5_wholemap.json
fi
echo EVIDENCE-DONE
