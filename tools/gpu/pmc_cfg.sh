#!/bin/bash
# PMC counters (one group per pass) of one bench config:
#   bash tools/gpu/pmc_cfg.sh <config>  ->  gpurun_out/pmc_cfg<config>/
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-4}
O=$R/gpurun_out/pmc_cfg$C
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o pmc --output-format csv -- python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_pmc$i.json 2> $O/pmc$i.err || exit 1
  echo "pmc $i ok"
done
