#!/bin/bash
# Round 6: the driver's default bench command (no flags) with its wall time, and the line's
# headline figures.  REPS runs back to back on one box.  Outputs under gpurun_out/end6/.
set -o pipefail
D=gpurun_out/end6
mkdir -p $D
for r in $(seq 1 ${REPS:-1}); do
  T0=$(date +%s.%N)
  timeout -k 10 900 python bench.py > $D/bench_d$r.json 2> $D/bench_d$r.err || { tail -20 $D/bench_d$r.err; exit 1; }
  T1=$(date +%s.%N)
  python - $D/bench_d$r.json "$T0" "$T1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("wall_s", round(float(sys.argv[3]) - float(sys.argv[2]), 1), "C4", d["value"], "p50", d["ms_per_step_p50"], "steps", d["steps"],
      "roof", r["kernel"], r["frac"], r["avg_launch_us"])
print("c2", d["c2"]["value"], d["c2"]["ms_per_step_p50"], "c3", d["c3"]["value"], d["c3"]["ms_per_step_p50"])
print("kernels", json.dumps(d["kernels_ms_per_step"]))
print("host", json.dumps(d["host_input"]["vs_device"]), "c5", d["sharded_c5"]["value"], d["sharded_c5_wholemap"]["value"])
PY
done
echo BENCH-DONE
