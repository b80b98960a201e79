#!/bin/bash
# round 4: SPAN-aware LDS swizzle (conflict-free ds_write_b128 at 128-B spans).
# Parity of the records path on the in-tree library, then same-box A/Bs:
# config 4 (a_head: previous swizzle, b_swz: new) and config 2 (+ c_u128:
# the uniform kernels at 128-B spans, 3 waves/SIMD, with the new swizzle).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_records_mixed.py \
    "tests/test_gpu_full_size.py::test_config4_full_size_zipf" -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r4_swz_tests.log 2>&1 || { tail -40 gpurun_out/r4_swz_tests.log; exit 1; }
tail -2 gpurun_out/r4_swz_tests.log
echo "== config 4"
mkdir -p ab_c2 && mv ab/c_u128.so ab_c2/ || exit 1
bash tools/gpu/ab_libs.sh 4 || exit 1
mv ab_c2/c_u128.so ab/ || exit 1
echo "== config 2"
NOISE_AMD_LIB=ab/c_u128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "uniform or config2" \
    --timeout 200 --timeout-method thread > gpurun_out/r4_u128_tests.log 2>&1 || { tail -30 gpurun_out/r4_u128_tests.log; exit 1; }
tail -1 gpurun_out/r4_u128_tests.log
bash tools/gpu/ab_libs.sh 2
