#!/bin/bash
# round 3: single-record latency after the wait-loop change (no stream query
# in the first 100 us): the resident / launch GPU tests, then config1_bench
# resident and launch, three runs each, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread \
    -k "resident or single or golden or kats or config1 or cipherstate" > gpurun_out/r3_res4_tests.log 2>&1 \
    || { tail -30 gpurun_out/r3_res4_tests.log; exit 1; }
tail -2 gpurun_out/r3_res4_tests.log
for rep in 1 2 3; do
  timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 resident > gpurun_out/c1_res_$rep.json 2>&1 || { cat gpurun_out/c1_res_$rep.json; exit 1; }
  echo "resident: $(cat gpurun_out/c1_res_$rep.json)"
  timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 > gpurun_out/c1_launch_$rep.json 2>&1 || { cat gpurun_out/c1_launch_$rep.json; exit 1; }
  echo "launch: $(cat gpurun_out/c1_launch_$rep.json)"
done
