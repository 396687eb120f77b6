tools/gpu_tests.sh gpurun_out/r3b "tests/test_gpu_evalio.py tests/test_gpu_configs.py" "tests/test_gpu_c5.py tests/test_bench_cli.py" "-m gpu --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_c5.py --deselect tests/test_gpu_evalio.py tests" || exit $?
REPS=2 STEPS=30 bash tools/gpu_abn.sh prev c128 c320 > gpurun_out/r3b/ab.txt 2>&1; tail -40 gpurun_out/r3b/ab.txt
