#!/bin/bash
# Round 6: descriptor batches with the masked classes -- parity tests, then
# config 4 exact and jittered, then the records / uniform length sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_records_mixed.py tests/test_gpu_full_size.py::test_config4_full_size_zipf} > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in "" "--jitter"; do
  timeout -k 10 300 python bench.py --config 4 $v --steps 10 --no-cpu-baseline > $O/cfg4$v.json 2> $O/cfg4$v.err || { echo "cfg4 $v failed"; tail -5 $O/cfg4$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/cfg4$v.json'));print('cfg4 $v', d['value'], d['roofline']['enc_ms'], d['roofline']['dec_ms'])"
done
timeout -k 10 900 python tools/bench_lengths.py --layouts ${SWEEP_LAYOUTS:-records} ${SWEEP_LENS:-} > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail -5 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
echo done
