#!/bin/bash
# round 3: config-4 records path -- records GPU tests + full-size config 4,
# then a same-box A/B of the ab/*.so builds on config 4 (alternating runs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py "tests/test_gpu_full_size.py::test_config4_full_size_zipf" \
    -x -q --timeout 400 --timeout-method thread > gpurun_out/r3_cfg4_tests.log 2>&1 || { tail -40 gpurun_out/r3_cfg4_tests.log; exit 1; }
tail -2 gpurun_out/r3_cfg4_tests.log
bash tools/gpu/ab_libs.sh 4
