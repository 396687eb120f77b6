#!/bin/bash
# Round 4: host-resident scan input (pipeline tests + tools/host_input_probe.py variants)
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_pipeline.py > gpurun_out/r4/t2.log 2>&1 || { tail -40 gpurun_out/r4/t2.log; exit 1; }
tail -2 gpurun_out/r4/t2.log
timeout -k 10 400 python -u tools/host_input_probe.py > gpurun_out/r4/probe_all.json 2> gpurun_out/r4/probe.err || { tail -20 gpurun_out/r4/probe.err; exit 1; }
cat gpurun_out/r4/probe_all.json
for v in "FMX_STAGE_THREADS=0" "FMX_STAGE_THREADS=7" "FMX_STAGE_DMAS=1" "FMX_STAGE_DMAS=8 FMX_STAGE_CHUNK_KB=128" "FMX_HOST_PAGEABLE=1"; do
  env $v timeout -k 10 400 python -u tools/host_input_probe.py --modes device_sequential,host_sequential,host_pipelined > gpurun_out/r4/probe_v.json 2> gpurun_out/r4/probe.err || { tail -20 gpurun_out/r4/probe.err; exit 1; }
  cat gpurun_out/r4/probe_v.json
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_seam.py > gpurun_out/r4/t3.log 2>&1 || { tail -30 gpurun_out/r4/t3.log; exit 1; }
tail -2 gpurun_out/r4/t3.log
