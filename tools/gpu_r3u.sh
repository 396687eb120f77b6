# multi-lane match: ring-1 passes in the query's octant frame (base) vs the fixed
# shift order with the same code (nooct) and the last commit (head): C4 parity and
# stream tests, C4 A/B (match span in the diag lines).
set -o pipefail
tools/gpu_tests.sh gpurun_out/r3u "tests/test_gpu_parity.py" "tests/test_gpu_configs.py" "tests/test_gpu_pipeline.py" "tests/test_gpu_window.py" "tests/test_gpu_map.py" || exit $?
grep -q " failed" gpurun_out/r3u/step*.log && { echo "tests failed"; exit 1; }
REPS=2 bash tools/gpu_abn.sh nooct head > gpurun_out/r3u/ab_c4.txt 2>&1 || { tail -20 gpurun_out/r3u/ab_c4.txt; exit 1; }
echo "== c4"; cat gpurun_out/r3u/ab_c4.txt
