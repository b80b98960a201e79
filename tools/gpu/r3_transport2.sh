#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "transport" -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_tr_tests.log 2>&1 || { tail -30 gpurun_out/r3_tr_tests.log; exit 1; }
tail -2 gpurun_out/r3_tr_tests.log
B=noise-cpp_amd/bin/transport_test
for t in 8 16; do timeout -k 10 200 $B bench pipeline 1000 1048576 256 $t || exit 1; done
timeout -k 10 200 $B bench pipeline 1000 1048576 1024 8 || exit 1
timeout -k 10 200 $B bench pipeline 100 65536 16384 8 || exit 1
