#!/bin/bash
# round 5: GPU suite on the current tree; rocprofv3 trace + PMC for configs 3
# and 5 (profiles/round5); Poly1305 / keystream pass span A/B on config 4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r5_call9_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5_call9_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/profile_cfg.sh 3 10 || exit 1
bash tools/gpu/profile_cfg.sh 5 5 || exit 1
cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/base /' || exit 1
  for lib in ab/*.so; do
    NOISE_AMD_LIB=$lib timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null || exit 1
  done
done
