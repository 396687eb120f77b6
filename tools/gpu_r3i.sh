# match diagnostics: where the slowest C4 blocks spend (probes, walk segments, grid position)
set -o pipefail
mkdir -p gpurun_out/r3i
REPS=1 STEPS=30 bash tools/gpu_abn.sh f8 > gpurun_out/r3i/ab_c4.txt 2>&1 || { tail -20 gpurun_out/r3i/ab_c4.txt; exit 1; }
cat gpurun_out/r3i/ab_c4.txt
grep -h "match diag" gpurun_out/ab_base1.err gpurun_out/ab_f81.err
