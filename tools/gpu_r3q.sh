# confirmation: the C5 one-lane match changes of this step (base) vs the last commit (head):
# match parity, C5 A/B on both sets, C4 A/B.
set -o pipefail
tools/gpu_tests.sh gpurun_out/r3q "tests/test_gpu_c5.py" "tests/test_gpu_parity.py" "tests/test_gpu_configs.py -k match" || exit $?
grep -q " failed" gpurun_out/r3q/step*.log && { echo "tests failed"; exit 1; }
for d in local wholemap; do
  WORKLOAD=c5 ABARGS="--c5-dist $d" REPS=2 STEPS=20 bash tools/gpu_abn.sh head > gpurun_out/r3q/ab_$d.txt 2>&1 || { tail -20 gpurun_out/r3q/ab_$d.txt; exit 1; }
  echo "== $d"; grep -v "match diag" gpurun_out/r3q/ab_$d.txt
done
REPS=2 bash tools/gpu_abn.sh head > gpurun_out/r3q/ab_c4.txt 2>&1 || { tail -20 gpurun_out/r3q/ab_c4.txt; exit 1; }
echo "== c4"; cat gpurun_out/r3q/ab_c4.txt
