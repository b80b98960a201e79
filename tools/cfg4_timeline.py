"""Timeline of config-4 records calls from a rocprofv3 kernel trace (CPU).
    python tools/cfg4_timeline.py gpurun_out/trace_<name>/.../run_kernel_trace.csv [call]
A call starts at a k_cls_count dispatch; prints every call's span (encrypt /
decrypt alternate) and the kernels of one call (default: the last decrypt)
with start / end in microseconds from the call's start and their queue."""
import csv
import re
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].find("noise_amd") >= 0]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_cls_count" in r["Kernel_Name"]]
    calls = []
    for n, a in enumerate(starts):
        b = starts[n + 1] if n + 1 < len(starts) else len(rows)
        calls.append(rows[a:b])
    spans = []
    for c in calls:
        t0 = int(c[0]["Start_Timestamp"])
        spans.append((max(int(r["End_Timestamp"]) for r in c) - t0) / 1000.0)
    print("calls: %d; spans (us): %s" % (len(calls), " ".join("%.0f" % s for s in spans)))
    kind = lambda c: "dec" if any("<true" in r["Kernel_Name"] for r in c) else "enc"
    for k in ("enc", "dec"):
        ss = sorted(s for c, s in zip(calls, spans) if kind(c) == k)
        if ss:
            print("%s median span %.1f us over %d calls" % (k, ss[len(ss) // 2], len(ss)))
    pick = int(sys.argv[2]) if len(sys.argv) > 2 else max(i for i, c in enumerate(calls) if kind(c) == "dec")
    c = calls[pick]
    t0 = int(c[0]["Start_Timestamp"])
    for r in c:
        s = (int(r["Start_Timestamp"]) - t0) / 1000.0
        e = (int(r["End_Timestamp"]) - t0) / 1000.0
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("noise_amd::", "").replace("void ", ""))
        print("%8.1f %8.1f %7.1f q%s %s" % (s, e, e - s, r["Queue_Id"], name[:56]))


if __name__ == "__main__":
    main()
