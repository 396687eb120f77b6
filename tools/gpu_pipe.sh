#!/bin/bash
# Pipelined-extraction check: the new GPU tests, the full GPU suite, then an A/B of the
# bench (HEAD build form_amd/ab/libfmx_prev.so without pipelining vs this build with).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pipe.log 2>&1 || { tail -40 gpurun_out/pytest_pipe.log; exit 1; }
tail -3 gpurun_out/pytest_pipe.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  FMX_LIB=$PWD/form_amd/ab/libfmx_prev.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-pipeline > gpurun_out/pipe_prev$rep.json 2> gpurun_out/pipe_prev$rep.err || { tail -20 gpurun_out/pipe_prev$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pipe_prev$rep.json')); print('prev', d['value'], d['ms_per_step'], d['gpu_busy_frac'])"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 > gpurun_out/pipe_new$rep.json 2> gpurun_out/pipe_new$rep.err || { tail -20 gpurun_out/pipe_new$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pipe_new$rep.json')); print('new', d['value'], d['ms_per_step'], d['gpu_busy_frac'], d.get('sequential_extraction'), {k: v for k, v in d['kernels_ms_per_step'].items() if v})"
done
