#!/bin/bash
# latency path: the host-entry GPU tests, then config 1
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "host or cipherstate or handshake or kats or loopback or transport" > gpurun_out/pytest_single.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_single.log; exit 1; }
tail -3 gpurun_out/pytest_single.log
timeout -k 10 120 python bench.py --config 1 > gpurun_out/cfg1.json 2> gpurun_out/cfg1.err || { echo "cfg1 failed"; tail -20 gpurun_out/cfg1.err; exit 1; }
cat gpurun_out/cfg1.json
