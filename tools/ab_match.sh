set -e
mkdir -p gpurun_out/ab
for r in 1 2; do for v in off f15 f30; do
  if [ $v = f15 ]; then L=form_amd/libfmx.so; else L=form_amd/ab/libfmx_$v.so; fi
  FMX_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --steps 60 > gpurun_out/ab/$v.$r.log 2>&1
  tail -1 gpurun_out/ab/$v.$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['roofline']['avg_launch_us'], d['kernels_ms_per_step']['match'], d['match_work_per_query'], d['ate']['max_pose_diff_m'])"
done; done
