#!/bin/bash
# Round-5 GPU batch: (1) the whole GPU suite at the default path, (2) the registration
# stream tests again with the moments path (FMX_MOMENTS=1), (3) an A/B of VARIANTS
# (tools/gpu_r5_abenv.sh).  Stops at the first failing step.
set -o pipefail
D=gpurun_out/r5b
mkdir -p $D
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > $D/tests_default.log 2>&1 || { tail -40 $D/tests_default.log; exit 1; }
  tail -1 $D/tests_default.log
  FMX_MOMENTS=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_window.py tests/test_gpu_pipeline.py tests/test_gpu_concurrent.py tests/test_gpu_evalio.py tests/test_golden.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests_moments.log 2>&1 || { tail -40 $D/tests_moments.log; exit 1; }
  tail -1 $D/tests_moments.log
fi
[ -n "$VARIANTS" ] && bash tools/gpu_r5_abenv.sh
exit 0
