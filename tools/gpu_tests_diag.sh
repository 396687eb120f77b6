#!/bin/bash
# Full GPU parity suite, then the match diagnostics bench line.  Usage: bash tools/gpu_tests_diag.sh [pytest -k expr]
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_gpu.log | tail -40; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
bash tools/gpu_diag_match.sh
