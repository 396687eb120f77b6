#!/bin/bash
# The driver's default bench command once more on this box (headline spread across
# boxes); the line to gpurun_out/reps/bench_$TAG.json and its key fields to stdout.
set -o pipefail
D=gpurun_out/reps
mkdir -p $D
T=${TAG:-x}
timeout -k 10 900 python bench.py > $D/bench_$T.json 2> $D/bench_$T.err || { tail -20 $D/bench_$T.err; exit 1; }
python - $D/bench_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C4", d["value"], "p50", d.get("ms_per_step_p50"), "busy", d.get("main_stream_busy_frac"), "frac", d["roofline"].get("frac"),
      "seq", (d.get("host_input") or {}).get("vs_device"))
for k in ("c2", "c3"):
    s = d.get(k) or {}
    print(k, s.get("value"), "p50", s.get("ms_per_step_p50"), "busy", s.get("main_stream_busy_frac"))
for k in ("sharded_c5", "sharded_c5_wholemap"):
    s = d.get(k) or {}
    print(k, s.get("value"))
PY
