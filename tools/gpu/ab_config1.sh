#!/bin/bash
# A/B of the single-record latency path: noise-cpp_amd/bin/config1_bench
# against each ab/*.so (copied over the in-tree library in turn; the in-tree
# build is put back at the end).  bash tools/gpu/ab_config1.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
LIB=$R/noise-cpp_amd/lib/libnoise_amd.so
cp $LIB /tmp/libnoise_amd.keep.so
for rep in 1 2; do
  for lib in $R/ab/*.so; do
    n=$(basename $lib .so)
    cp $lib $LIB
    timeout -k 10 120 $R/noise-cpp_amd/bin/config1_bench 1000 1024 > $R/gpurun_out/c1_$n.json || { cp /tmp/libnoise_amd.keep.so $LIB; exit 1; }
    python3 -c "import json;d=json.load(open('$R/gpurun_out/c1_$n.json'));print('$n', d['per_record']['per_record_us'], {k: (v['encrypt_us'], v['decrypt_us']) for k, v in d['latency_by_size'].items()})"
  done
done
cp /tmp/libnoise_amd.keep.so $LIB
