#!/bin/bash
# End-of-round style check at HEAD: full GPU parity suite, smoke(), the default bench line,
# rocprofv3 kernel stats of the same bench command (+ the main-stream critical path from
# its kernel trace).  Outputs under gpurun_out/end/.  Stops at the first failing step.
set -o pipefail
D=gpurun_out/end
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
head -c 800 $D/bench.json; echo
rm -rf $D/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --streams "" --sub-workloads= --no-host-input --no-c5 --no-ablation > $D/bench_prof.json 2> $D/prof.err || { tail -20 $D/prof.err; exit 1; }
python tools/critical_path.py $(find $D/prof -name "*kernel_trace.csv" | head -1) 40 $D/critical_path_c4.json 40 > /dev/null || exit 1
find $D/prof -name "*kernel_trace.csv" -delete
python tools/stats_fmx.py $(find $D/prof -name "*kernel_stats.csv" | head -1) > $D/kernel_stats_fmx.csv
head -20 $D/kernel_stats_fmx.csv
cat $D/critical_path_c4.json
