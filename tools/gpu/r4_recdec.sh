#!/bin/bash
# round 4: whole-record decrypt of long records (k_rec_dec).  Parity on the
# in-tree library (records, full-size config 4, 2-rank oracle-checked config
# 4, the parity suite), then the config-4 A/B: a_pipe (the three-pass segment
# pipeline), b_w1 / c_w2 / d_w4 (k_rec_dec with 1 / 2 / 4 waves per record).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py \
    "tests/test_gpu_full_size.py::test_config4_full_size_zipf" \
    "tests/test_gpu_multirank.py::test_bench_two_ranks_oracle_exact[cfg4]" \
    tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r4_recdec_tests.log 2>&1 || { tail -40 gpurun_out/r4_recdec_tests.log; exit 1; }
tail -2 gpurun_out/r4_recdec_tests.log
echo "== config 4"
bash tools/gpu/ab_libs.sh 4
