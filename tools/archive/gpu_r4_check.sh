#!/bin/bash
# Round 4 check: the new GPU tests, then the default bench line (all blocks).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -x -v --timeout 500 --timeout-method thread -p no:cacheprovider tests/test_gpu_map.py tests/test_gpu_parity.py::test_warm_matches_c4_icp_sequence tests/test_gpu_c5.py > gpurun_out/r4/t_check.log 2>&1 || { tail -40 gpurun_out/r4/t_check.log; exit 1; }
tail -2 gpurun_out/r4/t_check.log
timeout -k 10 560 python -u bench.py > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err || { tail -30 gpurun_out/r4/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r4/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "seq", d.get("sequential_extraction"))
print("host_input", json.dumps(d.get("host_input")))
for k in ("c2", "c3", "sharded_c5", "sharded_c5_wholemap"):
    if k in d:
        x = d[k]
        print(k, x["value"], x.get("ms_per_step"), json.dumps(x.get("roofline")), x.get("cpu_baseline", {}).get("value"), x.get("ate"))
PY
