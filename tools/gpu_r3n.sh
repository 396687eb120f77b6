# per-lane ring-1 work list in the one-lane-per-query match (base) vs the wave-wide
# shift passes (nocomp): match parity, C5 A/B on both query sets, SQ wave state.
set -o pipefail
tools/gpu_tests.sh gpurun_out/r3n "tests/test_gpu_c5.py" "tests/test_gpu_parity.py" "tests/test_gpu_configs.py -k match" || exit $?
grep -q " failed" gpurun_out/r3n/step*.log && { echo "tests failed"; exit 1; }
for d in local wholemap; do
  WORKLOAD=c5 ABARGS="--c5-dist $d" REPS=2 STEPS=20 bash tools/gpu_abn.sh nocomp > gpurun_out/r3n/ab_$d.txt 2>&1 || { tail -20 gpurun_out/r3n/ab_$d.txt; exit 1; }
  echo "== $d"; grep -v "match diag" gpurun_out/r3n/ab_$d.txt
done
bash tools/gpu_sqpmc.sh 2>&1 | tail -3
