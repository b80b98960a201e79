#!/bin/bash
# Config 4 with record offsets aligned to 16 (the product layout), 128 and
# 1024 bytes: how much of the segment kernel's gap is memory alignment.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for a in 16 128 1024; do
    timeout -k 10 200 python $R/bench.py --config 4 --rec-align $a --steps 10 --no-cpu-baseline \
      > $R/gpurun_out/align_$a.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$R/gpurun_out/align_$a.json'));r=d['roofline'];print('align', $a, d['value'], r['enc_ms'], r['dec_ms'])"
  done
done
