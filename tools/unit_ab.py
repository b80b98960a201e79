"""Timing-only A/B of the records path on BASELINE config 4's batch (no
correctness check: ablation builds produce wrong bytes on purpose).
    NOISE_AMD_LIB=ab/x.so python tools/unit_ab.py [reps]
Prints the median encrypt / decrypt call time (HIP events on the stream)."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.cuda.set_device(0)
    bench.noise_amd.load()
    stream = torch.cuda.current_stream()
    args = types.SimpleNamespace(records=None, rec_align=16)
    wl = bench.make_workload(4, args, 0, 1, stream)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(5):
        wl["step"]()
    enc, dec = [], []
    for _ in range(reps):
        wl["step"](evs)
        torch.cuda.synchronize()
        enc.append(evs[0].elapsed_time(evs[1]))
        dec.append(evs[1].elapsed_time(evs[2]))
    enc.sort()
    dec.sort()
    print("%s enc %.4f dec %.4f ms" % (os.path.basename(os.environ.get("NOISE_AMD_LIB", "in-tree")),
                                      enc[reps // 2], dec[reps // 2]))
    lib = bench.noise_amd.load()
    if hasattr(lib, "noise_amd_unit_stamps"):  # NOISE_UNIT_STAMPS builds: per-phase wave time
        import ctypes
        out = (ctypes.c_ulonglong * 8)()
        lib.noise_amd_unit_stamps(out)  # reset
        wl["step"]()
        torch.cuda.synchronize()
        lib.noise_amd_unit_stamps(out)
        units = out[7]
        names = ["A+dma wait", "C poly", "barrier", "D tags", "E keystream", "F wait", "F stores+dma"]
        tot = sum(out[:7])
        print("  units %d (x4 waves); per wave-unit us: " % units +
              ", ".join("%s %.2f (%.0f%%)" % (n, out[i] / 100.0 / max(units, 1), 100.0 * out[i] / max(tot, 1))
                        for i, n in enumerate(names)))


if __name__ == "__main__":
    main()
