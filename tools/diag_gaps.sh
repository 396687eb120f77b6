#!/bin/bash
# Kernel-trace timeline of UNPROFILED C4 / C2 scans (--profile-steps 0: no per-kernel HIP
# events in the run), printed for a few steps in the middle of the timed region.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/gaps
mkdir -p $D
for w in ${WL:-c4}; do
  rm -rf $D/$w
  timeout -k 10 300 rocprofv3 --kernel-trace -d $D/$w -o run --output-format csv -- python bench.py --workload $w --steps 20 --warmup 5 --profile-steps 0 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams= > $D/$w.json 2> $D/$w.err || { tail -20 $D/$w.err; exit 1; }
  T=$(find $D/$w -name "*kernel_trace.csv" | head -1)
  for b in 4 7 10; do python tools/trace_gaps.py $T $b > $D/${w}_step$b.txt || exit 1; done
  python - $T > $D/${w}_trace_small.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60].replace(",", ";"), r.get("Stream_Id", "")) for r in rows)
ev = ev[-4000:]
print("start,end,name,stream")
for e in ev: print(*e, sep=",")
PY
  find $D/$w -name "*.csv" -delete
done
echo GAPS-DONE
