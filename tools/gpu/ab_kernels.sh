#!/bin/bash
# Per-kernel A/B of ab/*.so on one bench config: rocprofv3 kernel stats of
# each library in turn, the rows whose name matches PATTERN printed:
#   bash tools/gpu/ab_kernels.sh <config> <pattern>
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-4}
PAT=${2:-k_seg}
cd /tmp && export TMPDIR=/tmp
for lib in $R/ab/*.so; do
  n=$(basename $lib .so)
  O=$R/gpurun_out/abk_$n
  mkdir -p $O
  export NOISE_AMD_LIB=$lib
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o t --output-format csv -- \
    python3 $R/bench.py --config $C --steps 5 --warmup 3 --no-cpu-baseline --no-config1 > $O/bench.json 2> $O/err.log || exit 1
  python3 - "$O" "$n" "$PAT" <<'PY'
import csv, glob, json, sys
o, n, pat = sys.argv[1:]
f = glob.glob(o + "/**/t_kernel_stats.csv", recursive=True)[0]
b = json.loads(open(o + "/bench.json").read().strip().splitlines()[-1])
print(n, "value", b["value"])
for r in csv.DictReader(open(f)):
    if pat in r["Name"]:
        print("   %-60s %8.1f us" % (r["Name"].split("(")[0][-60:], float(r["AverageNs"]) / 1e3))
PY
done
