#!/bin/bash
# round 4 A/B 1: the verify-first segmented decrypt (XOR pass at 128 / 256-B
# spans) against round 3 on config 4; the 128-B span uniform kernels
# (3 waves per SIMD) against 256 on config 2.  Parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py \
    "tests/test_gpu_multirank.py::test_bench_two_ranks_oracle_exact" tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r4_cfg4_tests.log 2>&1 || { tail -40 gpurun_out/r4_cfg4_tests.log; exit 1; }
tail -2 gpurun_out/r4_cfg4_tests.log
NOISE_AMD_LIB=$PWD/ab/d_u128.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tile_shapes.py \
    "tests/test_gpu_parity.py::test_config2_full_size_round_trip" -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r4_u128_tests.log 2>&1 || { tail -40 gpurun_out/r4_u128_tests.log; exit 1; }
tail -2 gpurun_out/r4_u128_tests.log
echo "== config 4"; bash tools/gpu/ab_libs.sh 4
echo "== config 2"; bash tools/gpu/ab_libs.sh 2
