#!/bin/bash
# round 3: config-4 A/B of ab/*.so (alternating bench runs), then one
# rocprofv3 kernel-trace stats pass per library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/ab_libs.sh 4 || exit 1
for lib in ab/*.so; do
  n=$(basename $lib .so)
  NOISE_AMD_LIB=$PWD/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run -- \
      python3 bench.py --config 4 --steps 5 --warmup 5 --no-cpu-baseline --no-config1 > gpurun_out/prof_$n.log 2>&1 || { tail -20 gpurun_out/prof_$n.log; exit 1; }
  f=$(find gpurun_out/prof_$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:10]:
    print('%-70s %6s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
"
done
