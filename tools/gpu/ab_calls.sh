#!/bin/bash
# Config-4 call-time A/B of library builds in ab/*.so: R alternating rounds,
# each run a median over N calls (tools/cfg4_calls.py, timing only):
#   bash tools/gpu/ab_calls.sh [rounds] [calls]
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in $(seq 1 ${1:-4}); do
  for lib in $R/ab/*.so; do
    NOISE_AMD_LIB=$lib timeout -k 10 200 python $R/tools/cfg4_calls.py ${2:-30} 2>/dev/null || exit 1
  done
done
