#!/bin/bash
# round 3: the new tile-shape, multi-rank and whole-batch full-size tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_tile_shapes.py tests/test_gpu_multirank.py \
    "tests/test_gpu_parity.py::test_config2_full_size_round_trip" tests/test_gpu_full_size.py \
    -x -v --timeout 400 --timeout-method thread --durations 15 > gpurun_out/r3_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r3_tests.log
exit $rc
