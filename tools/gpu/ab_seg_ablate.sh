#!/bin/bash
# Segment-kernel ablations (timing only, results wrong by design): every
# ab/*.so on 2^18 records of 4 KiB (1 M segments) through the records path,
# kernel-traced; prints the segment kernel's average duration per variant.
#   bash tools/gpu/ab_seg_ablate.sh [len]
set -o pipefail
R=$GRAFT_REPO_ROOT
L=${1:-4096}
mkdir -p $R/gpurun_out/ablate
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for lib in $R/ab/*.so; do
  n=$(basename $lib .so)
  NOISE_NO_CHECK=1 NOISE_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ablate/$n -o tr --output-format csv \
    -- python3 $R/tools/bench_records.py $((1073741824 / L)) 4096 $L > $R/gpurun_out/ablate/$n.json 2> $R/gpurun_out/ablate/$n.err || { echo "$n failed"; tail -5 $R/gpurun_out/ablate/$n.err; exit 1; }
  python3 - $R/gpurun_out/ablate/$n $n <<'PY'
import csv, glob, json, sys
d, name = sys.argv[1], sys.argv[2]
f = sorted(glob.glob(d + "/**/*kernel_stats.csv", recursive=True))[-1]
seg = {r["Name"].split("(")[0][-40:]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(f)) if ", 3, 0, 1, 256>" in r["Name"]}
b = json.load(open(d + ".json"))
print(name, b["enc_ms"], b["dec_ms"], {k: round(v, 1) for k, v in seg.items()})
PY
  rm -rf $R/gpurun_out/ablate/$n
done
done
