#!/bin/bash
# round 4: decrypt small classes on a third companion stream; parity on the
# in-tree library, then config 4 A/B (a_aux2: the previous layout)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py \
    "tests/test_gpu_full_size.py::test_config4_full_size_zipf" \
    "tests/test_gpu_multirank.py::test_bench_two_ranks_oracle_exact[cfg4]" \
    tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_aux3_tests.log 2>&1 || { tail -40 gpurun_out/r4_aux3_tests.log; exit 1; }
tail -1 gpurun_out/r4_aux3_tests.log
bash tools/gpu/ab_libs.sh 4 || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 noise-cpp_amd/bin/transport_test bench pipeline 100 65536 16384 8 || exit 1
done
