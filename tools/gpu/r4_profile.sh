#!/bin/bash
# round 4: rocprofv3 kernel trace + PMC passes for configs 2 and 4, then the
# default bench line (config 2 with the CPU baseline and the config-1 leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu/profile_cfg.sh 2 20 || exit 1
bash tools/gpu/profile_cfg.sh 4 10 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r4_bench_default.json 2> gpurun_out/r4_bench_default.err || { tail -20 gpurun_out/r4_bench_default.err; exit 1; }
cat gpurun_out/r4_bench_default.json
