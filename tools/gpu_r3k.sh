# window chunk-size A/B (w128, w64 vs the 256-row default), hardware-queue count A/B for
# the concurrent-streams figure, and the critical-path trace.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/r3k
export TMPDIR=/tmp
REPS=2 STEPS=30 bash tools/gpu_abn.sh w128 w64 > gpurun_out/r3k/ab_win.txt 2>&1 || { tail -20 gpurun_out/r3k/ab_win.txt; exit 1; }
grep -v "match diag" gpurun_out/r3k/ab_win.txt
for rep in 1 2; do
  for q in 4 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --no-cpu-baseline --no-ablation --no-c5 > gpurun_out/r3k/hwq$q.$rep.json 2> gpurun_out/r3k/hwq.err || { tail -20 gpurun_out/r3k/hwq.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r3k/hwq$q.$rep.json')); print('hwq $q', d['value'], d['ms_per_step'], d['concurrent_streams'], d['sequential_extraction'])" || exit 1
  done
done
rm -rf gpurun_out/r3k/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --streams "" --no-c5 > gpurun_out/r3k/bench_prof.json 2> gpurun_out/r3k/prof.err || { tail -20 gpurun_out/r3k/prof.err; exit 1; }
python tools/critical_path.py $(find gpurun_out/r3k/prof -name "*kernel_trace.csv" | head -1) 40 gpurun_out/r3k/critical_path_c4.json 40 || exit 1
find gpurun_out/r3k/prof -name "*kernel_trace.csv" -delete
