#!/bin/bash
# round 5: the decrypt unit kernel -- GPU suite, then config 4 units vs the
# round-4 segment path (NOISE_GPU_LONG=segments), alternating, then the bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r5_units_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5_units_tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  NOISE_GPU_LONG=segments timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/segments /' || exit 1
  timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/units /' || exit 1
done
timeout -k 10 300 python bench.py --config 4 --steps 20 --no-cpu-baseline --no-config1 > gpurun_out/r5_units_cfg4.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r5_units_cfg4.json'));r=d['roofline'];print('cfg4', d['value'], r['enc_ms'], r['dec_ms'])"
