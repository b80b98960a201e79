#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then PMC
# counters in separate passes (TCC FETCH_SIZE / WRITE_SIZE cannot share one).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 $BENCH > $O/bench_trace.json 2> $O/trace.err || exit 1
echo "trace ok"
timeout -k 10 300 rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d $O/pmc$i -o pmc --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_pmc$i.json 2> $O/pmc$i.err || exit 1
  echo "pmc $i ok"
done
