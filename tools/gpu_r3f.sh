# own-brick probe cache (C5 path): tests, then C5 A/B (head = last commit, base = this
# build at 7 waves, ob6 = 6 waves) on both query sets; comm overhead; C4 k_match
# variants (d3 = 3 record loads in flight, sc1 / sc3 = small-cell size).  Stops at the first failure.
set -o pipefail
tools/gpu_tests.sh gpurun_out/r3f "tests/test_gpu_c5.py tests/test_gpu_concurrent.py" "tests/test_gpu_parity.py -k large" || exit $?
grep -q " failed" gpurun_out/r3f/step*.log && { echo "tests failed"; exit 1; }
WORKLOAD=c5 ABARGS="--c5-dist local" REPS=2 STEPS=20 bash tools/gpu_abn.sh head ob6 > gpurun_out/r3f/ab_local.txt 2>&1 || { tail -20 gpurun_out/r3f/ab_local.txt; exit 1; }
grep -v "match diag" gpurun_out/r3f/ab_local.txt
WORKLOAD=c5 ABARGS="--c5-dist wholemap" REPS=2 STEPS=20 bash tools/gpu_abn.sh head ob6 > gpurun_out/r3f/ab_whole.txt 2>&1 || { tail -20 gpurun_out/r3f/ab_whole.txt; exit 1; }
grep -v "match diag" gpurun_out/r3f/ab_whole.txt
for comm in "" "--c5-comm"; do
  timeout -k 10 300 python bench.py --workload c5 --c5-dist local --steps 20 --warmup 3 $comm > gpurun_out/r3f/comm$comm.json 2> gpurun_out/r3f/comm.err || { tail -20 gpurun_out/r3f/comm.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3f/comm$comm.json')); print('comm' if '$comm' else 'none', d['value'], d['ms_per_step'], d['config']['rccl_communicator'], d['kernels_ms_per_step'])"
done
REPS=2 STEPS=30 bash tools/gpu_abn.sh d3 sc1 sc3 > gpurun_out/r3f/ab_c4.txt 2>&1 || { tail -20 gpurun_out/r3f/ab_c4.txt; exit 1; }
cat gpurun_out/r3f/ab_c4.txt
