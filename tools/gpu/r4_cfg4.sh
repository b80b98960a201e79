#!/bin/bash
# round 4: records-path parity (mixed batches, full-size config 4, the
# multirank oracle check), then config-4 A/B of ab/*.so (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py \
    "tests/test_gpu_multirank.py::test_bench_two_ranks_oracle_exact" tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r4_cfg4_tests.log 2>&1 || { tail -40 gpurun_out/r4_cfg4_tests.log; exit 1; }
tail -2 gpurun_out/r4_cfg4_tests.log
bash tools/gpu/ab_libs.sh 4
