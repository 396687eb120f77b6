# heavy-query queue + fused fixes: tests, C4 A/B (prev = round-2 lib, c0 = no deferral,
# c128 / c320 = other caps), C5 A/B, the C5 lines.  Stops at the first failing step.
set -o pipefail
tools/gpu_tests.sh gpurun_out/r3d "tests/test_gpu_c5.py" "-m gpu --deselect tests/test_gpu_c5.py tests" || exit $?
grep -q " failed" gpurun_out/r3d/step*.log && { echo "tests failed: no benches"; exit 1; }
REPS=2 STEPS=30 bash tools/gpu_abn.sh prev c0 c128 c320 > gpurun_out/r3d/ab_c4.txt 2>&1 || { tail -20 gpurun_out/r3d/ab_c4.txt; exit 1; }
cat gpurun_out/r3d/ab_c4.txt
WORKLOAD=c5 STEPS=10 REPS=2 bash tools/gpu_ablib.sh > gpurun_out/r3d/ab_c5.txt 2>&1 || { tail -20 gpurun_out/r3d/ab_c5.txt; exit 1; }
tail -4 gpurun_out/r3d/ab_c5.txt
timeout -k 10 600 python bench.py --workload c5 --steps 10 --warmup 2 > gpurun_out/r3d/c5.json 2> gpurun_out/r3d/c5.err || { tail -20 gpurun_out/r3d/c5.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r3d/c5.json'))
for k in (d, d['wholemap']): print(k['config']['query_distribution'], k['value'], k['ms_per_step'], k['icp_iters_per_registration'], k['pose_error'], k.get('kernels_ms_per_step'), k.get('match_work_per_query'), k['roofline'])"
