#!/bin/bash
# round 4, final tree: the -m gpu suite (one process), smoke(), the default
# bench line (driver's command) -> gpurun_out/r4_final_*
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --durations 10 > gpurun_out/r4_final_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r4_final_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_final_smoke.log 2>&1 || { tail -20 gpurun_out/r4_final_smoke.log; exit 1; }
tail -1 gpurun_out/r4_final_smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err || { tail -20 gpurun_out/r4_final_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4_final_bench.json'));r=d['roofline'];print(d['value'], r['enc_ms'], r['dec_ms'], r['frac'], r['pmc_source'], d['cpu_baseline']['value'], d['config1']['build']['per_record'])"
