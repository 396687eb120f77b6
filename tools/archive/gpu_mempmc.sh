#!/bin/bash
# Memory-pipeline counters of the match kernels (C5 fused match + linearization on both
# query sets, C4 match): address translation (UTCL1), L1 / L2 request latency, TA / TD
# busy, instruction mix — one rocprofv3 --pmc pass per counter group, each within the
# per-block slot limits (MI355X_MICROARCH.md §rocprofv3 PMC slots).
# Output: gpurun_out/mem/<workload>.json (tools/pmc_traffic.py format) + a summary.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/mem
rm -rf $D && mkdir -p $D
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
P2="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum"
P3="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA"
run() {  # name, bench args
  local n=$1; shift
  local i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex "k_match" -d $D/$n/p$i -o run --output-format csv -- python bench.py "$@" > $D/$n.p$i.out 2> $D/$n.p$i.err || { tail -20 $D/$n.p$i.err; exit 1; }
  done
  python tools/pmc_traffic.py $n $D/$n.json $D/$n/p1 $D/$n/p2 $D/$n/p3 > /dev/null || exit 1
  find $D/$n -name "*counter_collection.csv" -delete
  python - $D/$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    c = v["counters_per_launch"]
    print(d["workload"], k, v["launches"], {n: round(x, 1) for n, x in sorted(c.items())})
PY
}
run c5_local --workload c5 --c5-dist local --steps 4 --warmup 2 --no-cpu-baseline
run c5_wholemap --workload c5 --c5-dist wholemap --steps 4 --warmup 2 --no-cpu-baseline
run c4 --workload c4 --steps 10 --warmup 5 --no-cpu-baseline --no-c5 --no-ablation --streams ""
