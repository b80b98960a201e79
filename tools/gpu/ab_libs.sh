#!/bin/bash
# A/B of library builds in ab/*.so on the config-2 bench (alternating runs):
#   bash tools/gpu/ab_libs.sh [config]
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-2}
for rep in 1 2 3; do
  for lib in $R/ab/*.so; do
    n=$(basename $lib .so)
    NOISE_AMD_LIB=$lib timeout -k 10 200 python $R/bench.py --config $C --steps 20 --no-cpu-baseline --no-config1 > $R/gpurun_out/ab_$n.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$R/gpurun_out/ab_$n.json'));r=d['roofline'];print('$n', d['value'], r['enc_ms'], r['dec_ms'], r['frac'])"
  done
done
