# PMC HBM traffic (C4, both C5 query sets).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/r3g
bash tools/gpu_pmc.sh > gpurun_out/r3g/pmc_c4.txt 2>&1 || { tail -20 gpurun_out/r3g/pmc_c4.txt; exit 1; }
head -30 gpurun_out/r3g/pmc_c4.txt
bash tools/gpu_c5pmc.sh > gpurun_out/r3g/pmc_c5.txt 2>&1 || { tail -20 gpurun_out/r3g/pmc_c5.txt; exit 1; }
tail -14 gpurun_out/r3g/pmc_c5.txt
