#!/bin/bash
# round 3: resident latency workgroup -- tests, then config-1 both modes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 \
    --timeout-method thread -s > gpurun_out/r3_parity.log 2>&1 || { tail -40 gpurun_out/r3_parity.log; exit 1; }
tail -5 gpurun_out/r3_parity.log
for m in launch resident; do
  timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 $m > gpurun_out/c1_$m.json 2>&1 || exit 1
  cat gpurun_out/c1_$m.json
done
