# end-of-round style check (tests, smoke, C4 bench + rocprof + critical path), then the
# C2 and C3 bench lines.  Stops at the first failure.
set -o pipefail
bash tools/gpu_endcheck.sh || exit 1
for w in c2 c3; do
  timeout -k 10 600 python bench.py --workload $w --no-c5 --streams "" > gpurun_out/end/bench_$w.json 2> gpurun_out/end/bench_$w.err || { tail -20 gpurun_out/end/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/end/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d['cpu_baseline']['value'], d['ate'], d['counters'].get('icp_iters'))"
done
