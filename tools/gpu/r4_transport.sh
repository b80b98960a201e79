#!/bin/bash
# round 4: Pipeline rates (1 KiB and 16 KiB, three repetitions, 8 copy
# threads, defaults) and a kernel + copy trace of each size
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B=noise-cpp_amd/bin/transport_test
O=gpurun_out/r4_transport.jsonl
: > $O
for rep in 1 2 3; do
  timeout -k 10 200 $B bench pipeline 1000 1048576 1024 8 >> $O || exit 1
  timeout -k 10 200 $B bench pipeline 100 65536 16384 8 >> $O || exit 1
done
cat $O
for len in 1024 16384; do
  M=$((1073741824 / len))
  rm -rf gpurun_out/tp_trace_$len
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
      -d gpurun_out/tp_trace_$len -o run -- $B bench pipeline 1000 $M $len 8 > gpurun_out/tp_trace_$len.log 2>&1 || { tail -20 gpurun_out/tp_trace_$len.log; exit 1; }
done
find gpurun_out/tp_trace_* -name "*stats.csv" | head
