#!/bin/bash
# round 3: Pipeline slot_records 64K vs 128K at 256 B (depth 4, launcher
# thread), with 4 (the box default) and 8 hardware queues, two repetitions;
# 16 KiB
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=noise-cpp_amd/bin/transport_test
for rep in 1 2; do
  for sr in 65536 131072; do
    timeout -k 10 200 $B bench pipeline 1000 1048576 256 8 4 1 $sr || exit 1
    GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B bench pipeline 1000 1048576 256 8 4 1 $sr || exit 1
  done
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B bench pipeline 1000 1048576 1024 8 4 1 || exit 1
done
timeout -k 10 200 $B bench pipeline 100 65536 16384 8 4 1 || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B bench pipeline 100 65536 16384 8 4 1 || exit 1
