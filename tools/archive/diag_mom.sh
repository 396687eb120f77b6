#!/bin/bash
# moments-path diagnostic: one registration-stream test with the step trace (FMX_MOMENTS=1),
# then the same test's ICP / LM iteration log in both modes
export TMPDIR=/tmp FMX_SEGV_TRACE=1
FMX_MOMENTS=1 FMX_TRACE=1 timeout -s ABRT -k 10 100 python -u -m pytest tests/test_gpu_configs.py -k c3_full_window -x -q --timeout 90 --timeout-method thread -p no:cacheprovider -s > gpurun_out/diag_mom.log 2>&1
r=$?
echo "rc $r"
grep -n "fmx: native\|(+0x\|Fatal\|terminate\|what()\|passed\|failed\|Error" gpurun_out/diag_mom.log | tail -30
[ $r -ne 0 ] && exit 1
for m in FMX_MOMENTS FMX_LIN_ROWS; do
  env $m=1 FMX_SPEC_LOG=1 timeout -k 10 100 python -u -m pytest tests/test_gpu_configs.py -k c3_full_window -x -q --timeout 90 --timeout-method thread -p no:cacheprovider -s > gpurun_out/diag_$m.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/diag_$m.log; exit 1; }
  echo "$m: icp lines $(grep -c '^icp it' gpurun_out/diag_$m.log), next $(grep -c 'final next' gpurun_out/diag_$m.log), $(tail -1 gpurun_out/diag_$m.log)"
done
exit 0
