#!/bin/bash
# Per-launch rate of the uniform 1 KiB kernels against batch size (launch
# ramp / tail share): bash tools/gpu/size_sweep.sh [records...]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for n in ${@:-262144 1048576 4194304 8388608}; do
    timeout -k 10 200 python $R/bench.py --config 2 --records $n --steps 10 --no-cpu-baseline --no-config1 \
      > $R/gpurun_out/sweep_$n.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$R/gpurun_out/sweep_$n.json'));r=d['roofline'];print($n, d['value'], r['enc_ms'], r['dec_ms'], round($n*1024/r['enc_ms']/1e6/1.073741824,1), r['frac'])"
  done
done
