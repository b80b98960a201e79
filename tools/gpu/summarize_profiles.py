#!/usr/bin/env python3
"""Copy the rocprofv3 summaries of a gpurun_out/prof run into profiles/<name>/:
kernel_stats.csv (trace --stats), pmc_summary.json (per-kernel counter
means) and pmc_traffic.json (HBM bytes per launch, gfx950-corrected:
FETCH_SIZE counts half of a wide coalesced stream, so bytes read =
2 x FETCH_SIZE KiB; WRITE_SIZE is exact for 16-B stores -- see
/opt/skills/guides/MI355X_MICROARCH.md 'HBM')."""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
src = os.path.join(ROOT, "gpurun_out", "prof")
name = sys.argv[1] if len(sys.argv) > 1 else "round1"
dst = os.path.join(ROOT, "profiles", name)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))


def short(n):
    if "k_aead_tile<false" in n:
        return "k_aead_uniform<encrypt>"
    if "k_aead_tile<true" in n:
        return "k_aead_uniform<decrypt>"
    return n.split("(")[0][:80]


agg = collections.defaultdict(lambda: collections.defaultdict(list))
full = {}
for i in range(1, 10):
    f = os.path.join(src, "pmc%d" % i, "pmc_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        full[k] = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}
json.dump({"source": "rocprofv3 --pmc, one counter group per pass (tools/gpu/profile.sh)",
           "kernels": summary, "names": full}, open(os.path.join(dst, "pmc_summary.json"), "w"),
          indent=1)
bench = json.load(open(os.path.join(src, "bench_pmc1.json")))
traffic = {}
for k, d in summary.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        traffic[k] = int((2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024)
json.dump({"workload": bench["config"]["workload"], "per_launch_bytes": traffic,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB per dispatch (gfx950 FETCH_SIZE "
                         "reports half of a wide coalesced stream)"},
          open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
for f in ("bench_trace.json",):
    if os.path.exists(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))
print(json.dumps(traffic))
