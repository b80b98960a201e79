#!/bin/bash
# bench lines for every BASELINE config shape at N=1, plus the
# host-inclusive (pinned H2D -> kernel -> D2H) rate for config 2.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/configs
for c in 2 3 4; do
  timeout -k 10 300 python $R/bench.py --config $c --steps 5 --no-cpu-baseline > $R/gpurun_out/configs/cfg$c.json 2> $R/gpurun_out/configs/cfg$c.err || { echo "cfg$c failed"; tail -5 $R/gpurun_out/configs/cfg$c.err; exit 1; }
  echo "cfg$c ok"
done
timeout -k 10 400 python $R/bench.py --config 5 --records 2097152 --steps 3 --no-cpu-baseline > $R/gpurun_out/configs/cfg5_2M.json 2> $R/gpurun_out/configs/cfg5.err || { echo "cfg5 failed"; exit 1; }
timeout -k 10 300 python $R/bench.py --config 2 --steps 3 --no-cpu-baseline --host-inclusive > $R/gpurun_out/configs/cfg2_host.json 2> $R/gpurun_out/configs/cfg2_host.err || { echo "host failed"; tail -5 $R/gpurun_out/configs/cfg2_host.err; exit 1; }
echo done
