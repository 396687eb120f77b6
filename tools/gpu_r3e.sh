# C5 parity (both query sets), PMC traffic for C4 and both C5 query sets, the exchange
# step's overhead (1-rank communicator vs none).  Stops at the first failing step.
set -o pipefail
tools/gpu_tests.sh gpurun_out/r3e "tests/test_gpu_c5.py" || exit $?
grep -q " failed" gpurun_out/r3e/step1.log && { echo "tests failed"; exit 1; }
bash tools/gpu_pmc.sh > gpurun_out/r3e/pmc_c4.txt 2>&1 || { tail -20 gpurun_out/r3e/pmc_c4.txt; exit 1; }
bash tools/gpu_c5pmc.sh > gpurun_out/r3e/pmc_c5.txt 2>&1 || { tail -20 gpurun_out/r3e/pmc_c5.txt; exit 1; }
tail -12 gpurun_out/r3e/pmc_c5.txt
for rep in 1 2; do
  for comm in "" "--c5-comm"; do
    timeout -k 10 300 python bench.py --workload c5 --c5-dist local --steps 20 --warmup 3 $comm > gpurun_out/r3e/comm$rep$comm.json 2> gpurun_out/r3e/comm.err || { tail -20 gpurun_out/r3e/comm.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r3e/comm$rep$comm.json')); print('comm' if '$comm' else 'none', d['value'], d['ms_per_step'], d['config']['rccl_communicator'], d['kernels_ms_per_step'])"
  done
done
