#!/bin/bash
# round 5: the unit kernel (unit_kernel.hpp) -- GPU suite, then config 4
# units vs the round-4 segment path (NOISE_GPU_LONG=segments), alternating,
# then a kernel trace of the units build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --durations 5 > gpurun_out/r5_call2_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r5_call2_tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for mode in units segments; do
    NOISE_GPU_LONG=$mode timeout -k 10 200 python bench.py --config 4 --steps 20 --no-cpu-baseline --no-config1 > gpurun_out/r5c2_$mode.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/r5c2_$mode.json'));r=d['roofline'];print('$mode', d['value'], r['enc_ms'], r['dec_ms'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5c2_trace -o trace --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > /dev/null 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r5c2_trace -name "*kernel_stats.csv" | head -1)
head -20 "$f"
