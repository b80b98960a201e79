#!/bin/bash
# round 3: resident latency path v2 (device-memory request image, speculation)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 100 --timeout-method thread \
    -k "resident or single or golden or kats or config1 or cipherstate or handshake_vectors" > gpurun_out/r3_res2_tests.log 2>&1 \
    || { tail -40 gpurun_out/r3_res2_tests.log; exit 1; }
tail -3 gpurun_out/r3_res2_tests.log
for k in fine host; do
  NOISE_GPU_RESIDENT_REQ=$k timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 resident > gpurun_out/c1_res_$k.json 2>&1 || { cat gpurun_out/c1_res_$k.json; exit 1; }
  echo "$k: $(cat gpurun_out/c1_res_$k.json)"
done
timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 launch > gpurun_out/c1_launch.json 2>&1 && cat gpurun_out/c1_launch.json
