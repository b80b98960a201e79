#!/bin/bash
# round 4: classifier threshold A/B -- small device batches and the Pipeline
# at 16 KiB (2046 messages per 32 MiB slot) with each ab/*.so
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
B=noise-cpp_amd/bin/transport_test
LIB=noise-cpp_amd/lib/libnoise_amd.so
cp $LIB /tmp/keep.so
for lib in ab/*.so; do
  NOISE_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 tools/bench_small_records.py || { cp /tmp/keep.so $LIB; exit 1; }
done
for rep in 1 2; do
  for lib in ab/*.so; do
    cp $lib $LIB
    echo -n "$(basename $lib .so) "
    timeout -k 10 200 $B bench pipeline 100 65536 16384 8 || { cp /tmp/keep.so $LIB; exit 1; }
  done
done
cp /tmp/keep.so $LIB
