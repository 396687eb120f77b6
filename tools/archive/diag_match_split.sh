#!/bin/bash
# Match-kernel block timing of the C4 stream, warm and cold launches apart (needs the
# diagnostics of profiles/r5_match_regroup_tail.patch applied: FMX_MATCH_DIAG_WARM, FMX_DIAG_TAIL)
# (FMX_MATCH_DIAG + FMX_MATCH_DIAG_WARM); outputs under gpurun_out/mdiag/.
set -o pipefail
D=gpurun_out/mdiag
mkdir -p $D
for wv in 1 0; do
  FMX_MATCH_DIAG=1 FMX_MATCH_DIAG_WARM=$wv timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-c5 --no-ablation --sub-workloads= --no-host-input --streams= "$@" > $D/w$wv.json 2> $D/w$wv.err || { tail -30 $D/w$wv.err; exit 1; }
  echo "== warm=$wv"; grep "match diag" $D/w$wv.err
done
echo MDIAG-DONE
