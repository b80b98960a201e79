#!/bin/bash
# Build an A/B variant of the engine library into ab/<name>.so (CPU side):
#   bash tools/gpu/ab_build.sh <name> [-DFLAG=...]...
# The tree is copied to /tmp/ab_<name> so the in-tree build is untouched.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
N=$1; shift
D=/tmp/ab_$N
rm -rf $D && mkdir -p $D
cp -r $R/noise-cpp_amd $R/include $D/
rm -rf $D/noise-cpp_amd/build $D/noise-cpp_amd/lib $D/noise-cpp_amd/bin
make -s -j8 -C $D/noise-cpp_amd ARCH=gfx950 \
  HIPFLAGS="-O3 -std=c++20 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -I$D/include -I$D/noise-cpp_amd/csrc -I$D/noise-cpp_amd/host $*" \
  $D/noise-cpp_amd/lib/libnoise_amd.so
mkdir -p $R/ab
cp $D/noise-cpp_amd/lib/libnoise_amd.so $R/ab/$N.so
echo "ab/$N.so built ($*)"
