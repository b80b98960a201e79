#!/bin/bash
# Round 6: per-kernel PMC of the masked (ragged) tile kernels beside the exact
# ones -- bench_lengths.py under rocprofv3, one --pmc pass per counter group
# (dispatches serialise under --pmc: per-kernel figures).  tools/pmc_per_kernel.py
# summarises.   LENS="1000 1024" LAYOUT=uniform-aligned bash tools/gpu/r6_pmc_lengths.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6pmc${TAG:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_lengths.py --mib ${MIB:-512} --reps 2 --layouts ${LAYOUT:-uniform-aligned} ${LENS:-1000 1024 9000 16000 16384 300 512 100 128}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 $B > $O/trace.jsonl 2> $O/trace.err || { echo "trace failed"; tail -5 $O/trace.err; exit 1; }
echo "trace ok"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o pmc --output-format csv -- python3 $B > $O/pmc$i.jsonl 2> $O/pmc$i.err || { echo "pmc $i failed"; tail -5 $O/pmc$i.err; exit 1; }
  echo "pmc $i ok"
done
echo done
