#!/bin/bash
# Quick A/B of the default build vs prev (HEAD) and optional diag variants: bash tools/gpu_ab_quick.sh [tags]
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2} STEPS=${STEPS:-40} bash tools/gpu_abn.sh "$@" 2>&1 | grep -v '^   match diag: block' 
