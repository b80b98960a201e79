#!/bin/bash
# round 4 A/B 2: chunked verify-first decrypt (1/2/4/8 chunks) vs round 3 on
# config 4, after the records parity tests; then a kernel trace of config 4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py \
    "tests/test_gpu_multirank.py::test_bench_two_ranks_oracle_exact" tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r4_cfg4_tests.log 2>&1 || { tail -40 gpurun_out/r4_cfg4_tests.log; exit 1; }
tail -2 gpurun_out/r4_cfg4_tests.log
echo "== config 4"; bash tools/gpu/ab_libs.sh 4 || exit 1
bash tools/gpu/trace_cfg.sh 4
