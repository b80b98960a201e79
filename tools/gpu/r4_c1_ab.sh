#!/bin/bash
# round 4: config-1 latency, resident and launch modes, each ab/*.so copied
# over the in-tree library in turn (config1_bench links it), three rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
LIB=$R/noise-cpp_amd/lib/libnoise_amd.so
cp $LIB /tmp/keep.so
for rep in 1 2 3; do
  for lib in $R/ab/*.so; do
    n=$(basename $lib .so)
    cp $lib $LIB
    for mode in resident launch; do
      timeout -k 10 120 $R/noise-cpp_amd/bin/config1_bench 1000 1024 $mode > $R/gpurun_out/c1_$n.json || { cp /tmp/keep.so $LIB; exit 1; }
      python3 -c "import json;d=json.load(open('$R/gpurun_out/c1_$n.json'));print('$n $mode', d['per_record']['per_record_us'], d['latency_by_size']['1024'])"
    done
  done
done
cp /tmp/keep.so $LIB
