# 8 x 8 x 8 dense sub-cells (libfmx_f8): parity tests on that build, then the C4 A/B
# against the 4 x 4 x 4 default.  Stops at the first failure.
set -o pipefail
export FMX_LIB=$PWD/form_amd/ab/libfmx_f8.so
tools/gpu_tests.sh gpurun_out/r3h "tests/test_gpu_map.py tests/test_gpu_window.py -k match" "tests/test_gpu_parity.py -k match" "tests/test_gpu_window.py -k c4_full" || exit $?
unset FMX_LIB
grep -q " failed" gpurun_out/r3h/step*.log && { echo "tests failed"; exit 1; }
REPS=3 STEPS=30 bash tools/gpu_abn.sh f8 > gpurun_out/r3h/ab_c4.txt 2>&1 || { tail -20 gpurun_out/r3h/ab_c4.txt; exit 1; }
cat gpurun_out/r3h/ab_c4.txt
