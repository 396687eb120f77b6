mkdir -p gpurun_out
FMX_HOST_TIMING=1 timeout -k 10 300 python bench.py --steps 60 --warmup 10 --profile-steps 0 --no-cpu-baseline --no-ablation > gpurun_out/ht.json 2> gpurun_out/ht.err || { tail -20 gpurun_out/ht.err; exit 1; }
grep host gpurun_out/ht.err
python -c "import json; d=json.load(open('gpurun_out/ht.json')); print(d['value'], d['ms_per_step'], d['counters'])"
bash tools/gpu_trace.sh
