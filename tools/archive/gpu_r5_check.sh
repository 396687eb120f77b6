#!/bin/bash
# Round-5 working check: the GPU suite (or the tests named in $TESTS), then a short
# default-config bench line.  Outputs under gpurun_out/r5/.  Stops at the first failure.
set -o pipefail
D=gpurun_out/r5
mkdir -p $D
export TMPDIR=/tmp
T=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
grep -h "warm certificate" $D/gpu_tests.log | head -5
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline --streams "" --no-host-input --no-c5 --no-ablation > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
  head -c 1500 $D/bench.json; echo
fi
