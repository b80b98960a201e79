#!/usr/bin/env python3
"""gpurun_out/prof_cfgN (tools/gpu/profile_cfg.sh) -> profiles/<round>/cfgN/:
kernel_stats.csv (rocprofv3 --kernel-trace --stats), pmc_summary.json
(per-dispatch means of every counter, keyed by the kernel symbol without its
argument list) and pmc_traffic.json (HBM bytes per dispatch with the gfx950
FETCH_SIZE correction: bytes read = 2 x FETCH_SIZE KiB for wide coalesced
streams, WRITE_SIZE exact -- MI355X_MICROARCH.md 'HBM').  bench.py reads
pmc_summary.json for its roofline traffic and VALU fields.

    python3 tools/gpu/summarize_cfg.py <cfg> [round2]"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
cfg = int(sys.argv[1])
rnd = sys.argv[2] if len(sys.argv) > 2 else "round2"
src = os.path.join(ROOT, "gpurun_out", "prof_cfg%d" % cfg)
dst = os.path.join(ROOT, "profiles", rnd, "cfg%d" % cfg)
os.makedirs(dst, exist_ok=True)


def find(pattern):
    hits = glob.glob(os.path.join(src, "**", pattern), recursive=True)
    return hits[0] if hits else None


stats = find("trace_kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))


def symbol(name):
    name = name.split("(")[0]
    return name[5:] if name.startswith("void ") else name


agg = collections.defaultdict(lambda: collections.defaultdict(list))
for i in range(1, 10):
    f = find(os.path.join("pmc%d" % i, "**", "*counter_collection.csv")) if os.path.isdir(
        os.path.join(src, "pmc%d" % i)) else None
    if not f:
        continue
    for r in csv.DictReader(open(f)):
        agg[symbol(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}
# dispatches of each kernel in one PMC pass (a kernel launched more than once
# per call -- the decrypt pipeline's chunks -- counts that many times per
# call: bench.py scales its per-dispatch means by the ratio to a
# once-per-call kernel)
for k, d in agg.items():
    summary[k]["_dispatches"] = max(len(v) for v in d.values()) if d else 0
bench_line = None
for f in ("bench_trace.json", "bench_pmc1.json"):
    p = os.path.join(src, f)
    if os.path.exists(p) and open(p).read().strip():
        bench_line = json.loads(open(p).read().strip().splitlines()[-1])
        shutil.copy(p, os.path.join(dst, f))
json.dump({"source": "rocprofv3 --pmc, one counter group per pass (tools/gpu/profile_cfg.sh %d); "
                     "per-dispatch means" % cfg,
           "workload": bench_line["config"]["workload"] if bench_line else None,
           # records per launch of the profiled run: bench.py scales the
           # per-launch counts to its own shard size
           "records_per_launch": bench_line["config"]["records_per_gpu"] if bench_line else None,
           "kernels": summary}, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
traffic = {k: int((2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024)
           for k, d in summary.items() if "FETCH_SIZE" in d and "WRITE_SIZE" in d}
json.dump({"workload": bench_line["config"]["workload"] if bench_line else None,
           "per_dispatch_bytes": traffic,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB per dispatch (gfx950 FETCH_SIZE "
                         "reports half of a wide coalesced stream)"},
          open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in traffic.items() if k.startswith("noise_amd")}, indent=1))
