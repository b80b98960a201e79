#!/bin/bash
# Same-box A/B: the config-2 bench with and without an initialised RCCL
# process group (bench.py --force-dist at world size 1).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for rep in 1 2 3; do
  for mode in plain nccl gloo; do
    extra=""; [ $mode != plain ] && extra="--force-dist --dist-backend $mode"
    MASTER_PORT=$((29600 + rep * 10 + ${#mode})) timeout -k 10 200 python $R/bench.py --gpus 1 $extra --steps 20 --no-cpu-baseline --no-config1 \
      > $R/gpurun_out/dab_$mode.out 2> $R/gpurun_out/dab_$mode.err || { tail -5 $R/gpurun_out/dab_$mode.err; exit 1; }
    python3 -c "
import json
for l in open('$R/gpurun_out/dab_$mode.out'):
    if l.startswith('{'): d = json.loads(l); print('$mode', d['value'], d['roofline']['enc_ms'], d['roofline']['dec_ms'])"
  done
done
