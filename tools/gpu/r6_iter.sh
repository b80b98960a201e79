#!/bin/bash
# Round 6 iteration: parity tests of the masked kernels, config 4 exact /
# jitter, sweep, lengths PMC, config-4 traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TESTS="tests/test_gpu_ragged.py tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py::test_config4_full_size_zipf" SWEEP_LAYOUTS=uniform-aligned,records bash tools/gpu/r6_records.sh || exit 1
bash tools/gpu/r6_pmc_lengths.sh || exit 1
bash tools/gpu/r6_cfg4_trace.sh || exit 1
