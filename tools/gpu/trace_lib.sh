#!/bin/bash
# rocprofv3 kernel trace of config-4 calls through one library build:
#   bash tools/gpu/trace_lib.sh <ab/name.so | in-tree> [reps]
# -> gpurun_out/trace_<name>/  (tools/cfg4_timeline.py reads it on the CPU)
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$1
N=$(basename ${L%.so})
O=$R/gpurun_out/trace_$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "$L" != "in-tree" ]; then export NOISE_AMD_LIB=$R/$L; fi
timeout -k 10 240 rocprofv3 --kernel-trace -d $O -o run --output-format csv -- python3 $R/tools/cfg4_calls.py ${2:-10} > $O/calls.txt 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
cat $O/calls.txt
