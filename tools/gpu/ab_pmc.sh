#!/bin/bash
# Instruction counts of every ab/*.so on one config (one PMC pass each):
# SQ_INSTS_VALU / SALU / waves / GRBM_GUI_ACTIVE per dispatch of the tile
# kernel, to back an A/B with the dynamic instruction count.
#   bash tools/gpu/ab_pmc.sh [config]
#   PMC="WRITE_SIZE" bash tools/gpu/ab_pmc.sh 2    (other counters: means printed)
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-2}
mkdir -p $R/gpurun_out/ab_pmc
cd /tmp && export TMPDIR=/tmp
for lib in $R/ab/*.so; do
  n=$(basename $lib .so)
  NOISE_AMD_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE} --kernel-trace \
    -d $R/gpurun_out/ab_pmc/$n -o pmc --output-format csv -- python3 $R/bench.py --config $C --steps 3 --warmup 1 \
    --no-cpu-baseline --no-config1 > $R/gpurun_out/ab_pmc/$n.json 2> $R/gpurun_out/ab_pmc/$n.err || { echo "pmc $n failed"; tail -5 $R/gpurun_out/ab_pmc/$n.err; exit 1; }
  python3 - $R/gpurun_out/ab_pmc/$n $n <<'PY'
import csv, glob, sys, collections
d, name = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_aead_tile" not in k:
        continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    if "SQ_INSTS_VALU" not in m:
        print(name, k.split("(")[0][-60:], " ".join("%s %.0f" % kv for kv in sorted(m.items())))
        continue
    w = m.get("SQ_WAVES", 1)
    print(name, k.split("(")[0][-60:], "VALU/wave %.0f SALU/wave %.0f gui %.0f util %.3f" % (
        m["SQ_INSTS_VALU"] / w, m["SQ_INSTS_SALU"] / w, m["GRBM_GUI_ACTIVE"],
        m["SQ_INSTS_VALU"] * 4 / 1024 / (m["GRBM_GUI_ACTIVE"] / 8)))
PY
done
