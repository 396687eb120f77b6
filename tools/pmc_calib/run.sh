#!/bin/bash
# Build + run pmc_calib under two PMC passes (FETCH_SIZE, WRITE_SIZE); prints measured /
# known bytes per kernel.  Run on the GPU box: bash tools/pmc_calib/run.sh
set -e
export TMPDIR=/tmp
D=gpurun_out/pmc_calib
mkdir -p $D
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/pmc_calib/pmc_calib.hip -o $D/pmc_calib
timeout -k 10 120 $D/pmc_calib > $D/known.txt
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $D/$c
  timeout -s KILL 120 rocprofv3 --pmc $c -d $D/$c -o run --output-format csv -- $D/pmc_calib > /dev/null
done
python3 tools/pmc_calib/summarize.py $D | tee $D/calibration.txt
find $D -name "*counter_collection.csv" -delete
rm -f $D/pmc_calib
