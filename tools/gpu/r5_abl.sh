#!/bin/bash
# round 5: timing-only A/B of ab/*.so on config 4 (tools/cfg4_calls.py), the
# in-tree library with the segment path as the reference, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  NOISE_GPU_LONG=segments timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null | sed 's/^/segments /' || exit 1
  for lib in ab/*.so; do
    NOISE_AMD_LIB=$lib timeout -k 10 200 python tools/cfg4_calls.py 15 2>/dev/null || exit 1
  done
done
# one PMC pass of the in-tree (units) build
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5_abl_pmc -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/cfg4_calls.py 3 > /dev/null 2>&1 || exit 1
echo pmc ok
