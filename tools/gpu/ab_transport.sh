#!/bin/bash
# Same-box A/B of the host Pipeline: transport_test bench against each
# ab/*.so (copied over the in-tree library in turn, restored at the end).
#   bash tools/gpu/ab_transport.sh [threads...]
set -o pipefail
R=$GRAFT_REPO_ROOT
LIB=$R/noise-cpp_amd/lib/libnoise_amd.so
B=$R/noise-cpp_amd/bin/transport_test
cp $LIB /tmp/libnoise_amd.keep.so
for rep in 1 2; do
  for lib in $R/ab/*.so; do
    n=$(basename $lib .so)
    cp $lib $LIB
    for t in ${@:-4 8}; do
      out=$(timeout -k 10 200 $B bench pipeline 1000 1048576 1024 $t) || { cp /tmp/libnoise_amd.keep.so $LIB; exit 1; }
      echo "$n $out"
    done
  done
done
cp /tmp/libnoise_amd.keep.so $LIB
