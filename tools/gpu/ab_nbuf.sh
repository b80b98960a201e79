#!/bin/bash
# A/B of the uniform 1 KiB tile kernel's LDS buffering (NOISE_TILE_NBUF=1|2):
# parity tests under NBUF=2, then the config-2 bench both ways.
set -o pipefail
R=$GRAFT_REPO_ROOT
NOISE_TILE_NBUF=2 timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_nbuf2.log 2>&1 || { tail -20 $R/gpurun_out/pytest_nbuf2.log; exit 1; }
tail -1 $R/gpurun_out/pytest_nbuf2.log
for n in 1 2 1 2; do
  NOISE_TILE_NBUF=$n timeout -k 10 200 python $R/bench.py --steps 10 --no-cpu-baseline > $R/gpurun_out/ab_nbuf$n.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$R/gpurun_out/ab_nbuf$n.json'));r=d['roofline'];print('nbuf $n', d['value'], r['enc_ms'], r['dec_ms'], r['frac'])"
done
