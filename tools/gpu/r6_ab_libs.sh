#!/bin/bash
# Round 6: A/B of library builds in ab/*.so (tools/gpu/ab_build.sh) on config
# 4 exact and jittered, alternating, plus a records sweep per build:
#   LENS="16000 16321 16383" bash tools/gpu/r6_ab_libs.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ablib
mkdir -p $O
for rep in 1 2; do
  for lib in $R/ab/*.so; do
    n=$(basename $lib .so)
    for j in "" "--jitter"; do
      NOISE_AMD_LIB=$lib timeout -k 10 300 python $R/bench.py --config 4 $j --steps 10 --no-cpu-baseline --no-config1 > $O/${n}_$rep$j.json 2>> $O/err.log || exit 1
      python3 -c "import json;d=json.load(open('$O/${n}_$rep$j.json'));r=d['roofline'];print('$n $rep $j', d['value'], r['enc_ms'], r['dec_ms'])"
    done
  done
done
for lib in $R/ab/*.so; do
  n=$(basename $lib .so)
  NOISE_AMD_LIB=$lib timeout -k 10 300 python $R/tools/bench_lengths.py --layouts records ${LENS:-16000 16321 16383} > $O/sweep_$n.jsonl 2>> $O/err.log || exit 1
  python3 -c "
import json
for l in open('$O/sweep_$n.jsonl'):
    d=json.loads(l); print('$n', d['len'], d['enc_gib_s'], d['dec_gib_s'], d['round_trip_gib_s'])"
done
