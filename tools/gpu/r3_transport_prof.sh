#!/bin/bash
# round 3: Pipeline phase breakdown at 256 B / 1 KiB, then a rocprofv3
# kernel-trace stats pass of the default bench (profiles/round3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B=noise-cpp_amd/bin/transport_test
for len in 256 1024; do timeout -k 10 200 $B bench pipeline 1000 1048576 $len 8 || exit 1; done
timeout -k 10 200 $B bench pipeline 1000 1048576 256 16 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg2 -o run -- \
    python3 bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-config1 > gpurun_out/prof_cfg2.log 2>&1 || { tail -20 gpurun_out/prof_cfg2.log; exit 1; }
find gpurun_out/prof_cfg2 -name "*stats*" | head
