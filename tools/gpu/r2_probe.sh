#!/bin/bash
# round 2 first call: GPU tests, default bench, VALU issue-rate microbench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 120 tools/ubench/issue_bench > gpurun_out/issue_bench.txt 2>&1 || { echo "issue bench failed"; exit 1; }
cat gpurun_out/issue_bench.txt
