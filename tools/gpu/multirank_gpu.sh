#!/bin/bash
# The N-rank bench path end to end on a 1-GPU box: ranks share the GPU
# (--share-device test hook).  Both launch forms: the driver's
# torch.distributed.run command and bench.py's own launcher.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 5 --share-device \
  > gpurun_out/mr_torchrun_cfg2.json 2> gpurun_out/mr_torchrun_cfg2.err || { tail -30 gpurun_out/mr_torchrun_cfg2.err; exit 1; }
cat gpurun_out/mr_torchrun_cfg2.json
timeout -k 10 240 python bench.py --gpus 4 --config 5 --records 1048576 --steps 3 --warmup 2 --share-device \
  > gpurun_out/mr_launch_cfg5.json 2> gpurun_out/mr_launch_cfg5.err || { tail -30 gpurun_out/mr_launch_cfg5.err; exit 1; }
cat gpurun_out/mr_launch_cfg5.json
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29518 bench.py --gpus 2 --config 4 --records 262144 --steps 3 --warmup 2 --share-device \
  > gpurun_out/mr_torchrun_cfg4.json 2> gpurun_out/mr_torchrun_cfg4.err || { tail -30 gpurun_out/mr_torchrun_cfg4.err; exit 1; }
cat gpurun_out/mr_torchrun_cfg4.json
