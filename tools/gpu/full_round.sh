#!/bin/bash
# tests -> bench -> rocprofv3 trace/stats -> PMC passes (each step time-limited,
# chained so the first failure ends the call).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -m pytest $R/tests -m gpu -x -q > $R/gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -2 $R/gpurun_out/pytest_gpu.log
timeout -k 10 300 python $R/bench.py > $R/gpurun_out/bench.json 2> $R/gpurun_out/bench.err || { echo "bench failed"; tail -20 $R/gpurun_out/bench.err; exit 1; }
cat $R/gpurun_out/bench.json
bash $R/tools/gpu/profile.sh || exit 1
