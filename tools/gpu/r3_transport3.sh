#!/bin/bash
# round 3: Pipeline depth 3 vs 4 vs 5 (same box), batched mode, 8 copy threads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=noise-cpp_amd/bin/transport_test
for len in 1024 256; do for d in 3 4 5; do
  timeout -k 10 200 $B bench pipeline 1000 1048576 $len 8 $d || exit 1
done; done
for d in 3 4; do timeout -k 10 200 $B bench pipeline 100 65536 16384 8 $d || exit 1; done
timeout -k 10 200 $B bench pipeline 1000 1048576 1024 16 4 || exit 1
