#!/bin/bash
# round 5: unit kernel (load ordering) vs segments, and its phase stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_abl3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_abl3_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  NOISE_GPU_LONG=segments timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/segments /' || exit 1
  timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/units /' || exit 1
done
NOISE_AMD_LIB=ab/st8k.so timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null || exit 1
