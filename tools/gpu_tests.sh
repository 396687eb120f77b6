#!/bin/bash
# GPU test steps under per-step time limits; stops at the first step that times out,
# aborts or crashes (exit status other than 0 = pass / 1 = test failures).
# usage: tools/gpu_tests.sh OUTDIR "pytest args 1" ["pytest args 2" ...]
D=$1; shift
mkdir -p $D
export TMPDIR=/tmp
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider $args > $D/step$i.log 2>&1
  rc=$?
  echo "step $i ($args): exit $rc"; tail -3 $D/step$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
