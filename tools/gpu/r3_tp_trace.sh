#!/bin/bash
# round 3: where a Pipeline slot's time goes at 1 KiB -- HIP API, copy and
# kernel durations of the transport bench (no counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B=noise-cpp_amd/bin/transport_test
rm -rf gpurun_out/tp_trace
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d gpurun_out/tp_trace -o run -- $B bench pipeline 1000 1048576 1024 8 ${DEPTH:-3} > gpurun_out/tp_trace.log 2>&1 || { tail -20 gpurun_out/tp_trace.log; exit 1; }
cat gpurun_out/tp_trace.log | grep mode
find gpurun_out/tp_trace -name "*.csv" | head -20
