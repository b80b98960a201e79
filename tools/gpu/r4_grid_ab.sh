#!/bin/bash
# round 4: decrypt-pass grid caps (config 4), same box, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
NOISE_AMD_LIB=ab/c_x3072p2048.so timeout -k 10 300 python -u -m pytest tests/test_gpu_records_mixed.py \
    "tests/test_gpu_full_size.py::test_config4_full_size_zipf" -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r4_grid_tests.log 2>&1 || { tail -30 gpurun_out/r4_grid_tests.log; exit 1; }
tail -1 gpurun_out/r4_grid_tests.log
bash tools/gpu/ab_libs.sh 4
