#!/bin/bash
# round 4 A/B 3: after the sized records calls / runtime chunk count: parity
# (records, transport, multirank), small-batch latency, Pipeline 1 / 16 KiB,
# config 4 against round 3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py \
    "tests/test_gpu_multirank.py::test_bench_two_ranks_oracle_exact" tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r4_ab3_tests.log 2>&1 || { tail -40 gpurun_out/r4_ab3_tests.log; exit 1; }
tail -2 gpurun_out/r4_ab3_tests.log
timeout -k 10 200 python3 tools/bench_small_records.py || exit 1
B=noise-cpp_amd/bin/transport_test
for rep in 1 2 3; do
  timeout -k 10 200 $B bench pipeline 1000 1048576 1024 8 || exit 1
  timeout -k 10 200 $B bench pipeline 100 65536 16384 8 || exit 1
done
echo "== config 4"; bash tools/gpu/ab_libs.sh 4
