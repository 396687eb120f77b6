#!/bin/bash
# Round 4: host-resident scan input variants (tools/host_input_probe.py, C4 steady state)
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
M=device_sequential,host_sequential,pinned_sequential,host_pipelined
for v in "FMX_STAGE_THREADS=3" "FMX_STAGE_THREADS=0" "FMX_STAGE_THREADS=7" "FMX_STAGE_PACK=0" "FMX_STAGE_DMAS=1" "FMX_STAGE_DMAS=8 FMX_STAGE_CHUNK_KB=128" "FMX_HOST_PAGEABLE=1"; do
  env $v timeout -k 10 300 python -u tools/host_input_probe.py --modes $M --reps 2 > gpurun_out/r4/probe_v.json 2> gpurun_out/r4/probe.err || { tail -20 gpurun_out/r4/probe.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4/probe_v.json')); print('$v', d['scans_per_s'], d['env'], 'copies', d['pageable_h2d_us'], d['pinned_h2d_us'], d['memcpy_to_pinned_us'])"
done
