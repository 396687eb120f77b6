#!/bin/bash
# Round 6, final sources: long-stream parity against the oracle (tools/long_stream.py:
# window-store and pool compaction, many marginalizations), C4 pipelined and C2.
set -o pipefail
D=gpurun_out/long6
mkdir -p $D
timeout -k 10 500 python -u tools/long_stream.py --scans 300 --config c4 --pipeline > $D/c4.txt 2>&1 || { tail -20 $D/c4.txt; exit 1; }
tail -4 $D/c4.txt
timeout -k 10 500 python -u tools/long_stream.py --scans 300 --config c2 --pipeline > $D/c2.txt 2>&1 || { tail -20 $D/c2.txt; exit 1; }
tail -4 $D/c2.txt
