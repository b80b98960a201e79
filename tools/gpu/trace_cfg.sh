#!/bin/bash
# Kernel trace + per-kernel stats of one bench config:
#   bash tools/gpu/trace_cfg.sh <config> [extra bench args]
# -> gpurun_out/trace_cfg<config>/ (rocprofv3 csv) + bench json/err
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-2}
shift
O=$R/gpurun_out/trace_cfg$C
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o trace --output-format csv -- python3 $R/bench.py --config $C --steps 5 --warmup 3 --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || exit 1
echo "trace cfg$C ok"
