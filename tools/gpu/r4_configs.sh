#!/bin/bash
# round 4, final tree: bench lines of configs 3, 4 and 5 (one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in 3 4 5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 --no-config1 > gpurun_out/r4_cfg$c.json 2> gpurun_out/r4_cfg$c.err || { tail -20 gpurun_out/r4_cfg$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4_cfg$c.json'));r=d['roofline'];print($c, d['value'], r['enc_ms'], r['dec_ms'], r['frac'], r.get('traffic'), r['pmc_source'], d['cpu_baseline']['value'])"
done
