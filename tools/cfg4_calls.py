"""Timing-only A/B of the records path on BASELINE config 4's batch (no
correctness check: ablation builds may produce wrong bytes on purpose).
    NOISE_AMD_LIB=ab/x.so python tools/cfg4_calls.py [reps]
Prints the median encrypt / decrypt call time (HIP events on the stream).
Round 5 used it for the unit-kernel A/Bs (profiles/round5/ab/cfg4_units.md)."""
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


if __name__ == "__main__":
    main()
