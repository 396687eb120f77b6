#!/bin/bash
# Round-5 C5 A/B of builds, both query sets + the map build: TAGS ("base" = form_amd/libfmx.so,
# any other tag = form_amd/ab/libfmx_<tag>.so), REPS reps interleaved.  First the C5 parity
# tests on every variant build (TEST=0 skips them).
set -o pipefail
D=gpurun_out/r5c5
mkdir -p $D
export TMPDIR=/tmp
TAGS=${TAGS:-base}
lib() { if [ $1 = base ]; then unset FMX_LIB; else export FMX_LIB=$PWD/form_amd/ab/libfmx_$1.so; fi; }
if [ "${TEST:-1}" = 1 ]; then
  for tag in $TAGS; do
    [ $tag = base ] && continue
    lib $tag
    timeout -k 10 400 python -u -m pytest tests/test_gpu_c5.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest_$tag.log 2>&1 || { tail -40 $D/pytest_$tag.log; exit 1; }
    echo "$tag: $(tail -1 $D/pytest_$tag.log)"
  done
fi
for rep in $(seq 1 ${REPS:-2}); do
  for tag in $TAGS; do
    lib $tag
    timeout -k 10 300 python bench.py --workload c5 --c5-dist both --steps 10 --warmup 2 --no-cpu-baseline > $D/$tag$rep.json 2> $D/$tag$rep.err || { tail -20 $D/$tag$rep.err; exit 1; }
    python - $D/$tag$rep.json $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d.get("wholemap", {}); b = d.get("map_build") or {}
f = lambda x: (x.get("kernels_ms_per_step") or {}).get("match_linearize", 0.0)
print("%-6s local %7.1f /s (%.3f ms, it %.1f) | wholemap %7.1f /s (%.3f ms, it %.1f) work %s | build %.2f ms" % (
    sys.argv[2], d["value"], f(d), d["icp_iters_per_registration"], w.get("value", 0), f(w),
    w.get("icp_iters_per_registration", 0), w.get("match_work_per_query"), b.get("ms_per_build", 0)))
PY
  done
done
