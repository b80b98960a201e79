#!/bin/bash
# Round 6 round trip: masked-kernel parity tests, config 4 exact / jitter,
# the length sweep (uniform aligned + records) and the lengths PMC.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TESTS="tests/test_gpu_ragged.py tests/test_gpu_tile_shapes.py tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py::test_config4_full_size_zipf" SWEEP_LAYOUTS=uniform-aligned,records bash tools/gpu/r6_records.sh || exit 1
bash tools/gpu/r6_pmc_lengths.sh || exit 1
