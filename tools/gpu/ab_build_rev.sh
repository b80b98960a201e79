#!/bin/bash
# Build the engine library of a git revision into ab/<name>.so (CPU side):
#   bash tools/gpu/ab_build_rev.sh <name> <rev> [-DFLAG=...]...
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
N=$1; REV=$2; shift 2
D=/tmp/abrev_$N
rm -rf $D && mkdir -p $D
git -C $R archive $REV noise-cpp_amd include | tar -x -C $D
make -s -j8 -C $D/noise-cpp_amd ARCH=gfx950 \
  HIPFLAGS="-O3 -std=c++20 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -I$D/include -I$D/noise-cpp_amd/csrc -I$D/noise-cpp_amd/host $*" \
  $D/noise-cpp_amd/lib/libnoise_amd.so
mkdir -p $R/ab
cp $D/noise-cpp_amd/lib/libnoise_amd.so $R/ab/$N.so
echo "ab/$N.so built from $REV ($*)"
