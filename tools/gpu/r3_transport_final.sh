#!/bin/bash
# round 3: Pipeline with the round-3 defaults (depth 4, launcher thread,
# 128K-record slots, 8 copy threads), three repetitions per message size,
# and the same-box 16-thread / nproc CPU baseline at the same sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=noise-cpp_amd/bin/transport_test
O=gpurun_out/transport_final.jsonl
: > $O
timeout -k 10 300 python3 tools/cpu_msgs_baseline.py 256 1024 >> $O || exit 1
for rep in 1 2 3; do
  for len in 256 1024; do timeout -k 10 200 $B bench pipeline 1000 1048576 $len 8 >> $O || exit 1; done
  timeout -k 10 200 $B bench pipeline 100 65536 16384 8 >> $O || exit 1
done
cat $O
