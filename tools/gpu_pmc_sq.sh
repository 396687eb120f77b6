#!/bin/bash
# SQ stall breakdown for one kernel (KRX regex, default k_match): wave cycles split
# into parked (waitcnt / barrier), issue-stalled and active; instruction mix.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsq
KRX=${KRX:-k_match}
rm -rf gpurun_out/pmcsq/p
timeout -k 10 300 rocprofv3 --pmc ${CTRS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS} --kernel-include-regex "$KRX" -d gpurun_out/pmcsq/p -o run --output-format csv -- python bench.py --steps 5 --warmup 3 --profile-steps 0 --no-cpu-baseline > gpurun_out/pmcsq/b.json 2> gpurun_out/pmcsq/b.err || { tail -20 gpurun_out/pmcsq/b.err; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmcsq/p/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'][:60]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
for k, d in acc.items():
    launches = max(v for (kk, c), v in n.items() if kk == k)
    print(k, 'launches', launches)
    for c, v in sorted(d.items()): print('  %-22s %14.0f per launch' % (c, v / launches))
PY
find gpurun_out/pmcsq -name "*counter_collection.csv" -delete
