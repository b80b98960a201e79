#!/bin/bash
# round 6, final tree: full_round.sh (suite, smoke, default bench line,
# configs 2 and 4 trace + PMC), then config 4 jittered, configs 3 and 5,
# the host-inclusive rates (1 KiB and 16 KiB records, both directions) and
# the record-length sweep -> gpurun_out/r6f
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6f
mkdir -p $O
if [ "${SKIP_FULL:-0}" != 1 ]; then
  bash tools/gpu/full_round.sh ${CFGS:-2 4} || exit 1
fi
cd "$GRAFT_REPO_ROOT"
for v in "--config 4" "--config 4 --jitter" "--config 3" "--config 5"; do
  n=$(echo $v | tr -d ' -')
  timeout -k 10 400 python bench.py $v --steps 10 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));r=d['roofline'];print('$n', d['value'], r['enc_ms'], r['dec_ms'], r['frac'], r.get('valu_cap_hbm_frac'))"
done
timeout -k 10 400 python bench.py --config 2 --steps 3 --no-cpu-baseline --host-inclusive > $O/host.json 2> $O/host.err || { tail -20 $O/host.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/host.json'));print('host', d.get('host_inclusive'), d.get('host_inclusive_16k'))"
timeout -k 10 900 python tools/bench_lengths.py --layouts ${SWEEP_LAYOUTS:-uniform-aligned,records} > $O/sweep.jsonl 2> $O/sweep.err || { tail -5 $O/sweep.err; exit 1; }
echo done
