#!/bin/bash
# Round 6, VERDICT item 1a/5: config 4 exact and jittered, the record-length
# sweep (uniform aligned / packed, descriptor records), the host-inclusive
# rate at 1 KiB and 16 KiB.  Output under gpurun_out/r6m/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6m
mkdir -p $O
timeout -k 10 300 python $R/bench.py --config 4 --steps 10 --no-cpu-baseline > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 failed"; tail -5 $O/cfg4.err; exit 1; }
echo "cfg4 ok"
timeout -k 10 300 python $R/bench.py --config 4 --jitter --steps 10 --no-cpu-baseline > $O/cfg4_jitter.json 2> $O/cfg4_jitter.err || { echo "cfg4 jitter failed"; tail -5 $O/cfg4_jitter.err; exit 1; }
echo "cfg4 jitter ok"
timeout -k 10 300 python $R/bench.py --config 4 --steps 10 --no-cpu-baseline > $O/cfg4_run2.json 2> $O/cfg4_run2.err || { echo "cfg4 run2 failed"; exit 1; }
timeout -k 10 600 python $R/tools/bench_lengths.py ${SWEEP_ARGS:-} > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail -5 $O/sweep.err; exit 1; }
echo "sweep ok"
if [ -n "${HOST_INCL:-}" ]; then
  timeout -k 10 300 python $R/bench.py --config 2 --steps 3 --no-cpu-baseline --no-config1 --host-inclusive > $O/cfg2_host.json 2> $O/cfg2_host.err || { echo "host failed"; tail -5 $O/cfg2_host.err; exit 1; }
  echo "host ok"
fi
echo done
