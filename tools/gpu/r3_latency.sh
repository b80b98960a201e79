#!/bin/bash
# round 3: single-record latency -- phase timing of the launch kernel, the
# resident-mode GPU tests, config-1 in both modes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 tools/ubench/one_timing > gpurun_out/one_timing.txt 2>&1 && timeout -k 10 60 tools/ubench/one_timing_fence > gpurun_out/one_timing_fence.txt 2>&1 || { cat gpurun_out/one_timing*.txt; exit 1; }
cat gpurun_out/one_timing.txt gpurun_out/one_timing_fence.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "resident or single or golden or kats or config1 or cipherstate or handshake_vectors" > gpurun_out/r3_lat_tests.log 2>&1 \
    || { tail -30 gpurun_out/r3_lat_tests.log; exit 1; }
tail -2 gpurun_out/r3_lat_tests.log
for m in launch resident; do
  timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 $m > gpurun_out/c1_$m.json 2>&1 || { cat gpurun_out/c1_$m.json; exit 1; }
  cat gpurun_out/c1_$m.json
done
