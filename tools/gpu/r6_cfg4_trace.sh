#!/bin/bash
# Round 6: rocprofv3 kernel traces of config 4, exact and jittered lengths
# (tools/cfg4_timeline.py / kernel_stats per kernel), for the jitter gap.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in exact jitter; do
  J=""; [ $v = jitter ] && J="--jitter"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o trace --output-format csv -- python3 $R/bench.py --config 4 $J --steps 5 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/$v.err || { echo "trace $v failed"; tail -5 $O/$v.err; exit 1; }
  echo "trace $v ok"
done
