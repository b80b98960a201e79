#!/bin/bash
# round 5, final tree: full_round.sh (suite, smoke, default bench line,
# configs 2 and 4 profiles), then a 2-rank --share-device line (per-rank
# fields) and config 4 / 3 / 5 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/full_round.sh 2 4 || exit 1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --gpus 2 --share-device --steps 10 --no-cpu-baseline > gpurun_out/r5_mr2.json 2> gpurun_out/r5_mr2.err || { tail -20 gpurun_out/r5_mr2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5_mr2.json'));print('2 ranks', d['value'], [(s['rank'], s['enc_ms'], s['dec_ms'], s['device'].get('pci_bus_id')) for s in d['shards']])"
for c in 4 3 5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 > gpurun_out/r5_cfg$c.json 2> gpurun_out/r5_cfg$c.err || { tail -20 gpurun_out/r5_cfg$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r5_cfg$c.json'));r=d['roofline'];print('cfg$c', d['value'], r['enc_ms'], r['dec_ms'], r['frac'], r.get('valu_cap_hbm_frac'), r['pmc_source'])"
done
