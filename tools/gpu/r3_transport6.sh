#!/bin/bash
# round 3: Pipeline with SDMA copies (default) vs blit-kernel copies
# (HSA_ENABLE_SDMA=0), depth 4, launcher thread, 128K-record slots
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=noise-cpp_amd/bin/transport_test
for rep in 1 2; do
  for len in 256 1024; do
    timeout -k 10 200 $B bench pipeline 1000 1048576 $len 8 4 1 131072 || exit 1
    HSA_ENABLE_SDMA=0 timeout -k 10 200 $B bench pipeline 1000 1048576 $len 8 4 1 131072 || exit 1
  done
done
HSA_ENABLE_SDMA=0 timeout -k 10 200 $B bench pipeline 100 65536 16384 8 4 1 || exit 1
