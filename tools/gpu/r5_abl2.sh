#!/bin/bash
# round 5: unit-kernel phase stamps and grid A/B (timing only, tools/cfg4_calls.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  NOISE_GPU_LONG=segments timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/segments /' || exit 1
  timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/units /' || exit 1
  for lib in ab/*.so; do
    NOISE_AMD_LIB=$lib timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null || exit 1
  done
done
