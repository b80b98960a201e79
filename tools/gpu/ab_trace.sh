#!/bin/bash
# Kernel-trace of every ab/*.so on one config: bench value + per-kernel
# average durations (rocprofv3 --kernel-trace --stats), for timeline A/Bs.
#   bash tools/gpu/ab_trace.sh [config]
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-4}
mkdir -p $R/gpurun_out/ab_trace
cd /tmp && export TMPDIR=/tmp
for lib in $R/ab/*.so; do
  n=$(basename $lib .so)
  NOISE_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_trace/$n -o tr --output-format csv \
    -- python3 $R/bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline --no-config1 \
    > $R/gpurun_out/ab_trace/$n.json 2> $R/gpurun_out/ab_trace/$n.err || { echo "trace $n failed"; tail -5 $R/gpurun_out/ab_trace/$n.err; exit 1; }
  python3 - $R/gpurun_out/ab_trace/$n $n <<'PY'
import csv, glob, json, sys
d, name = sys.argv[1], sys.argv[2]
b = json.load(open(d + ".json"))
print(name, "value", b["value"], "ms/step", b["ms_per_step"])
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "noise_amd" in r["Name"] and "fill" not in r["Name"]:
        print("   %-66s %5s %9.1f us" % (r["Name"].split("(")[0][-66:], r["Calls"], float(r["AverageNs"]) / 1000))
PY
done
