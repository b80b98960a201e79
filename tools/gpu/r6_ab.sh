#!/bin/bash
# Round 6 A/B of a runtime switch on config 4 (exact and jittered lengths):
#   AB_VAR=NOISE_AB_ENC_TAILS bash tools/gpu/r6_ab.sh
# alternates the variable 0 / 1 over two rounds; one JSON line per run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6ab
mkdir -p $O
cd $R
V=${AB_VAR:-NOISE_AB_ENC_TAILS}
for rep in 1 2; do
  for val in 0 1; do
    for j in "" "--jitter"; do
      env $V=$val timeout -k 10 300 python bench.py --config 4 $j --steps 10 --no-cpu-baseline > $O/ab_${val}_${rep}$j.json 2> $O/ab.err || { echo "bench failed"; tail -5 $O/ab.err; exit 1; }
      python -c "import json;d=json.load(open('$O/ab_${val}_${rep}$j.json'));print('$V=$val rep $rep $j', d['value'], d['roofline']['enc_ms'], d['roofline']['dec_ms'])"
    done
  done
done
