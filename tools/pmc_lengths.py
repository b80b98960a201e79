#!/usr/bin/env python3
"""Per-dispatch-shape PMC summary of a bench_lengths.py run under rocprofv3
(tools/gpu/r6_pmc_lengths.sh): counters per wave, grouped by (kernel, grid
size) -- one masked kernel serves several lengths, told apart by their grids.
    python tools/pmc_lengths.py gpurun_out/r6pmc
Columns: waves, VALU / SALU / LDS / VMEM-read / VMEM-write instructions per
wave, wave cycles per wave (quad-cycles x 4), the share of the wave's cycles
parked on s_waitcnt (WAIT_ANY) and stalled at issue (WAIT_INST_ANY), LDS bank
conflict cycles per wave, and the VALU issue utilisation
(VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs))."""
import collections
import csv
import glob
import re
import sys


def load(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.Counter())
    for f in glob.glob(d + "/pmc*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("noise_amd::", "").replace("void ", ""))
            if "tile" not in k:
                continue
            key = (k, int(r.get("Grid_Size", 0) or 0))
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[key][r["Counter_Name"]] += 1
    return acc, cnt


def main():
    for d in sys.argv[1:]:
        acc, cnt = load(d)
        print("==", d)
        print("%-44s %9s %7s %6s %6s %5s %5s %8s %5s %5s %7s %5s" % (
            "kernel", "grid", "waves", "VALU", "SALU", "LDS", "VMEM", "cyc", "wait", "stall", "ldsconf",
            "util"))
        for key in sorted(acc):
            a, c = acc[key], cnt[key]

            def m(n):
                return a[n] / c[n] if c[n] else 0.0
            w = m("SQ_WAVES") or 1.0
            wc = m("SQ_WAVE_CYCLES")
            g = m("GRBM_GUI_ACTIVE") / 8
            print("%-44s %9d %7d %6.0f %6.0f %5.0f %5.0f %8.0f %5.2f %5.2f %7.0f %5.3f" % (
                key[0][:44], key[1], w, m("SQ_INSTS_VALU") / w, m("SQ_INSTS_SALU") / w, m("SQ_INSTS_LDS") / w,
                (m("SQ_INSTS_VMEM_RD") + m("SQ_INSTS_VMEM_WR")) / w, 4 * wc / w,
                m("SQ_WAIT_ANY") / wc if wc else 0, m("SQ_WAIT_INST_ANY") / wc if wc else 0,
                m("SQ_LDS_BANK_CONFLICT") / w, m("SQ_INSTS_VALU") * 4 / 1024 / g if g else 0))


if __name__ == "__main__":
    main()
