#!/bin/bash
# Round 5: the moments path (FMX_MOMENTS=1) — its registration-stream tests, a short bench
# with the step trace, then the A/B of VARIANTS (tools/gpu_r5_abenv.sh).
set -o pipefail
D=gpurun_out/r5b
mkdir -p $D
export TMPDIR=/tmp
FMX_MOMENTS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_window.py tests/test_gpu_pipeline.py tests/test_gpu_concurrent.py tests/test_gpu_evalio.py tests/test_golden.py tests/test_gpu_moments.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/tests_moments.log 2>&1 || { grep -v "^  File" $D/tests_moments.log | tail -30; exit 1; }
tail -1 $D/tests_moments.log
[ -n "$VARIANTS" ] && bash tools/gpu_r5_abenv.sh
exit 0
