# fused C5 path: tests, then C5 A/B (prev = round-2 HEAD lib vs this build), then the new C5 lines
tools/gpu_tests.sh gpurun_out/r3c "tests/test_gpu_c5.py" "-m gpu --deselect tests/test_gpu_c5.py tests" || exit $?
WORKLOAD=c5 STEPS=10 REPS=2 bash tools/gpu_ablib.sh > gpurun_out/r3c/ab_c5.txt 2>&1; tail -8 gpurun_out/r3c/ab_c5.txt
timeout -k 10 600 python bench.py --workload c5 --steps 10 --warmup 2 > gpurun_out/r3c/c5.json 2> gpurun_out/r3c/c5.err || { tail -20 gpurun_out/r3c/c5.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r3c/c5.json'))
for k in (d, d['wholemap']): print(k['config']['query_distribution'], k['value'], k['ms_per_step'], k['icp_iters_per_registration'], k['pose_error'], k.get('kernels_ms_per_step'), k.get('match_work_per_query'), k['roofline'])"
