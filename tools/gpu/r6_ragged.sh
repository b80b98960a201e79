#!/bin/bash
# Round 6: the masked tile kernel on the GPU -- its parity tests (and the
# exact tile shapes beside them), then the length sweep of the given layouts.
#   SWEEP_LAYOUTS=uniform-aligned bash tools/gpu/r6_ragged.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6r
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_ragged.py tests/test_gpu_tile_shapes.py} > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 900 python tools/bench_lengths.py --layouts ${SWEEP_LAYOUTS:-uniform-aligned} ${SWEEP_LENS:-} > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail -5 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
echo done
