#!/bin/bash
# round 4: plain (L2-allocating) record stores vs nt, configs 2 and 4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
NOISE_AMD_LIB=ab/b_plain.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_records_mixed.py -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/r4_plain_tests.log 2>&1 || { tail -30 gpurun_out/r4_plain_tests.log; exit 1; }
tail -1 gpurun_out/r4_plain_tests.log
echo "== config 2"; bash tools/gpu/ab_libs.sh 2 || exit 1; bash tools/gpu/ab_libs.sh 2 || exit 1
echo "== config 4"; bash tools/gpu/ab_libs.sh 4
