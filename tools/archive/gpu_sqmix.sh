#!/bin/bash
# VALU instruction mix of the match kernels (C4 match, C5 fused match + linearization):
# two rocprofv3 --pmc passes of 8 SQ counters each (MI355X_MICROARCH.md PMC slot limits).
# Output: gpurun_out/sqmix/<workload>.json (tools/pmc_traffic.py format) + a per-wave summary.
# WORKLOADS: which runs (default c4 c5_local).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/sqmix
rm -rf $D && mkdir -p $D
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
P2="SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
run() {  # name, bench args
  local n=$1; shift
  local i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex "k_match" -d $D/$n/p$i -o run --output-format csv -- python bench.py "$@" > $D/$n.p$i.out 2> $D/$n.p$i.err || { tail -20 $D/$n.p$i.err; exit 1; }
  done
  python tools/pmc_traffic.py $n $D/$n.json $D/$n/p1 $D/$n/p2 > /dev/null || exit 1
  find $D/$n -name "*counter_collection.csv" -delete
  python - $D/$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    c = v["counters_per_launch"]
    w = max(c.get("SQ_WAVES", 1), 1)
    print(d["workload"], k, "launches", v["launches"], "per wave:",
          " ".join("%s %.0f" % (n.replace("SQ_INSTS_", ""), x / w) for n, x in sorted(c.items()) if n != "SQ_WAVES"))
PY
}
for w in ${WORKLOADS:-c4 c5_local}; do
  case $w in
    c5_local) run c5_local --workload c5 --c5-dist local --steps 4 --warmup 2 --no-cpu-baseline ;;
    c4) run c4 --workload c4 --steps 10 --warmup 5 --no-cpu-baseline --no-c5 --no-ablation --streams "" ;;
  esac
done
