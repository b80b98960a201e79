#!/bin/bash
# round 3: Pipeline launcher thread A/B (same box), depth 3 / 4, three
# repetitions each; the transport GPU tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "transport" -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_tr_tests.log 2>&1 || { tail -30 gpurun_out/r3_tr_tests.log; exit 1; }
tail -2 gpurun_out/r3_tr_tests.log
B=noise-cpp_amd/bin/transport_test
for rep in 1 2 3; do
  for len in 1024 256; do
    for cfg in "3 0" "4 0" "4 1"; do
      timeout -k 10 200 $B bench pipeline 1000 1048576 $len 8 $cfg || exit 1
    done
  done
done
for cfg in "4 0" "4 1"; do timeout -k 10 200 $B bench pipeline 100 65536 16384 8 $cfg || exit 1; done
