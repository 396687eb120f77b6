# ring-1 walk in nearest-first octant order (base) vs the index-order walk of the last
# commit (head): match parity, walk statistics (FMX_DIAG_WALK build), C5 A/B.
set -o pipefail
tools/gpu_tests.sh gpurun_out/r3t "tests/test_gpu_c5.py" "tests/test_gpu_parity.py -k large" || exit $?
grep -q " failed" gpurun_out/r3t/step*.log && { echo "tests failed"; exit 1; }
for d in local wholemap; do
  FMX_LIB=$PWD/form_amd/ab/libfmx_walk.so FMX_MATCH_DIAG=1 timeout -k 10 300 python bench.py --workload c5 --c5-dist $d --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r3t/walk_$d.json 2> gpurun_out/r3t/walk_$d.err || { tail -20 gpurun_out/r3t/walk_$d.err; exit 1; }
  echo "== $d"; grep "list walk" gpurun_out/r3t/walk_$d.err
  WORKLOAD=c5 ABARGS="--c5-dist $d" REPS=2 STEPS=20 bash tools/gpu_abn.sh head > gpurun_out/r3t/ab_$d.txt 2>&1 || { tail -20 gpurun_out/r3t/ab_$d.txt; exit 1; }
  grep -v "match diag" gpurun_out/r3t/ab_$d.txt
done
