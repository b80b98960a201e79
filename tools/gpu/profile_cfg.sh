#!/bin/bash
# rocprofv3 evidence for one BASELINE config (bench.py --config N):
# kernel trace + stats, then PMC counters in separate passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass; SQ counters in groups of <= 8).
#   bash tools/gpu/profile_cfg.sh <cfg> [steps]
set -o pipefail
R=$GRAFT_REPO_ROOT
CFG=${1:-2}
STEPS=${2:-20}
O=${PROF_OUT:-$R/gpurun_out/prof_cfg$CFG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --config $CFG --no-cpu-baseline --no-config1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 $B --steps $STEPS --warmup 3 > $O/bench_trace.json 2> $O/trace.err || { echo "trace failed"; tail -5 $O/trace.err; exit 1; }
echo "cfg$CFG trace ok"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o pmc --output-format csv -- python3 $B --steps 3 --warmup 1 > $O/bench_pmc$i.json 2> $O/pmc$i.err || { echo "pmc $i failed"; tail -5 $O/pmc$i.err; exit 1; }
  echo "cfg$CFG pmc $i ok"
done
