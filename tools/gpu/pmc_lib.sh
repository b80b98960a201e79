#!/bin/bash
# One rocprofv3 PMC pass (VALU count, busy cycles) over config-4 calls through
# one library build (dispatches serialise under --pmc: per-kernel figures):
#   bash tools/gpu/pmc_lib.sh <ab/name.so | in-tree> [reps]
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$1
N=$(basename ${L%.so})
O=$R/gpurun_out/pmc_$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "$L" != "in-tree" ]; then export NOISE_AMD_LIB=$R/$L; fi
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES --kernel-trace -d $O -o pmc --output-format csv -- python3 $R/tools/cfg4_calls.py ${2:-3} > $O/calls.txt 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
echo "$N pmc ok"
