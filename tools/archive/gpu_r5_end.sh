#!/bin/bash
# Round-5 end measurements.  PART=bench: the default bench line (the driver's command) and
# the host-input A/B of the piecewise extraction (FMX_STAGE_ROWS=0 = the whole scan first).
# PART=prof: rocprofv3 kernel stats of the same default bench command, and the C4 / C2
# critical paths at HEAD.  Outputs under gpurun_out/end5/.
set -o pipefail
D=gpurun_out/end5
mkdir -p $D
export TMPDIR=/tmp
if [ "${PART:-bench}" = bench ]; then
  timeout -k 10 900 python bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
  python - $D/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C4", d["value"], "p50", d.get("ms_per_step_p50"), "busy", d.get("main_stream_busy_frac"), "roof", {k: d["roofline"].get(k) for k in ("kernel", "frac", "hbm_frac", "avg_launch_us")})
print("host_input", json.dumps(d.get("host_input", {}).get("vs_device")), json.dumps(d.get("host_input", {}).get("vs_device_p50")))
for k in ("c2", "c3"):
    s = d.get(k) or {}
    print(k, s.get("value"), "p50", s.get("ms_per_step_p50"), "busy", s.get("main_stream_busy_frac"))
for k in ("sharded_c5", "sharded_c5_wholemap"):
    s = d.get(k) or {}
    r = s.get("roofline") or {}
    print(k, s.get("value"), "frac", r.get("frac"), "hbm_frac", r.get("hbm_frac"), "traffic", r.get("traffic"), "alg", r.get("alg_bytes_per_launch"))
b = d.get("c5_map_build") or {}
print("c5_map_build", b.get("ms_per_build"), json.dumps(b.get("roofline"))[:300])
print("cpu_baseline", json.dumps(d.get("cpu_baseline"))[:300])
PY
  for v in "" "FMX_STAGE_ROWS=0"; do
    timeout -k 10 300 env $v python bench.py --no-cpu-baseline --streams= --no-ablation --no-c5 --sub-workloads= > $D/host_${v:-default}.json 2> $D/host_${v:-default}.err || { tail -20 $D/host_${v:-default}.err; exit 1; }
    python -c "import json; d=json.loads(open('$D/host_${v:-default}.json').read().strip().splitlines()[-1]); h=d['host_input']; print('${v:-default}', d['value'], h['vs_device'], h['vs_device_p50'])"
  done
else
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py > $D/bench_prof.json 2> $D/prof.err || { tail -20 $D/prof.err; exit 1; }
  find $D/prof -name "*kernel_trace.csv" -delete
  python tools/stats_fmx.py $(find $D/prof -name "*kernel_stats.csv" | head -1) > $D/kernel_stats_fmx.csv
  head -12 $D/kernel_stats_fmx.csv
  CPATH="c4 c2" PMC=0 PART=scan bash tools/gpu_r5_evidence.sh || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
  tail -3 $D/smoke.log
fi
echo END-DONE
