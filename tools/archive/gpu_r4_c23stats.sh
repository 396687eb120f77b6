#!/bin/bash
# rocprofv3 kernel stats of the C2 and C3 streams alone (fmx kernels), round 4.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/c23
rm -rf $D && mkdir -p $D
for w in c2 c3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/$w -o run --output-format csv -- python bench.py --workload $w --no-cpu-baseline --streams "" --sub-workloads= --no-host-input --no-c5 --no-ablation > $D/$w.json 2> $D/$w.err || { tail -20 $D/$w.err; exit 1; }
  python tools/critical_path.py $(find $D/$w -name "*kernel_trace.csv" | head -1) 40 $D/critical_path_$w.json 40 > /dev/null || exit 1
  find $D/$w -name "*kernel_trace.csv" -delete
  python tools/stats_fmx.py $(find $D/$w -name "*kernel_stats.csv" | head -1) > $D/${w}_kernel_stats_fmx.csv
  echo "== $w"; head -8 $D/${w}_kernel_stats_fmx.csv; cat $D/critical_path_$w.json
done
