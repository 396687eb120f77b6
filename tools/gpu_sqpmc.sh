#!/bin/bash
# Where the match kernels' wave time goes: SQ wave-state counters (issue vs parked on
# memory vs issue stalls) for the C4 match and the C5 fused match + linearization, one
# rocprofv3 --pmc pass each (8 SQ counters, MI355X_MICROARCH.md §rocprofv3 PMC slots).
# Outputs: gpurun_out/sq/<workload>.json (tools/pmc_traffic.py format), counters.txt.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/sq
rm -rf $D && mkdir -p $D
timeout -k 10 120 rocprofv3 -L > $D/counters.txt 2>&1 || { tail -5 $D/counters.txt; exit 1; }
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
run() {  # name, bench args
  local n=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex "k_match" -d $D/$n -o run --output-format csv -- python bench.py "$@" > $D/$n.out 2> $D/$n.err || { tail -20 $D/$n.err; exit 1; }
  python tools/pmc_traffic.py $n $D/$n.json $D/$n > /dev/null || exit 1
  find $D/$n -name "*counter_collection.csv" -delete
  python - $D/$n.json <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    c = v["counters_per_launch"]
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(d["workload"], k, "launches", v["launches"], "waves/launch %.0f" % c.get("SQ_WAVES", 0),
          "wave-cycles/wave %.0f" % (wc / max(c.get("SQ_WAVES", 1), 1)),
          " ".join("%s %.3f" % (n[3:], c.get(n, 0) / wc) for n in
                   ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA")),
          "busy-cycles %.0f" % c.get("SQ_BUSY_CYCLES", 0))
EOF
}
# WORKLOADS: which runs (default all three)
for w in ${WORKLOADS:-c5_local c5_wholemap c4}; do
  case $w in
    c5_local) run c5_local --workload c5 --c5-dist local --steps 4 --warmup 2 --no-cpu-baseline ;;
    c5_wholemap) run c5_wholemap --workload c5 --c5-dist wholemap --steps 4 --warmup 2 --no-cpu-baseline ;;
    c4) run c4 --workload c4 --steps 10 --warmup 5 --no-cpu-baseline --no-c5 --no-ablation --streams "" ;;
  esac
done
