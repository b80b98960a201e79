"""Same-box CPU baseline for the Pipeline comparison: the
reference's own monocypher (oracle/_ref, noise::encrypt / decrypt framing of
noise.cpp:202-281; the C restatement if _ref is absent) over L-byte messages
of 1000 sessions (message i: session i mod 1000, nonce i div 1000), one call
per message, encrypt and decrypt timed separately at 16 threads (one GPU's
host share) and at nproc threads.  Test infrastructure: the oracle is the
measured baseline here, never the product.
  python3 tools/cpu_msgs_baseline.py 256 1024"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))
import noise_amd  # noqa: E402  (record dtype only; no GPU call)
import oracle_lib  # noqa: E402


def main():
    orc = oracle_lib.Oracle()
    fn = orc.ref.ref_batch_records if orc.ref is not None else orc.lib.oracle_batch_records
    kind = "reference" if orc.ref is not None else "port"
    ncpu = os.cpu_count() or 1
    for L in [int(a) for a in sys.argv[1:]] or [256, 1024]:
        R = (256 << 20) // L
        S = 1000
        i = np.arange(R, dtype=np.uint64)
        d = np.zeros(R, dtype=noise_amd.record_dtype())
        in_sz, ct_sz = (L + 15) // 16 * 16, (L + 31) // 16 * 16
        d["in_off"], d["out_off"] = i * np.uint64(in_sz), i * np.uint64(ct_sz)
        d["nonce"], d["len"] = i // np.uint64(S), L
        d["key_idx"] = (i % np.uint64(S)).astype(np.uint32)
        dd = d.copy()
        dd["in_off"], dd["out_off"] = d["out_off"], d["in_off"]
        keys = np.frombuffer(orc.synthetic(S * 32, 0x4B4559), dtype=np.uint8).copy()
        pt = np.frombuffer(orc.synthetic(R * in_sz, 7), dtype=np.uint8).copy()
        ct = np.zeros(R * ct_sz, dtype=np.uint8)
        back = np.zeros_like(pt)
        fails = ctypes.c_int(0)

        def run(dec, t):
            if dec:
                return fn(1, keys.ctypes.data, dd.ctypes.data, R, ct.ctypes.data, back.ctypes.data, t,
                          ctypes.byref(fails))
            return fn(0, keys.ctypes.data, d.ctypes.data, R, pt.ctypes.data, ct.ctypes.data, t,
                      ctypes.byref(fails))

        out = {"len": L, "messages": R, "sessions": S, "kind": kind}
        for t in sorted({16, ncpu}):
            for dec in (False, True):
                run(dec, t)
                secs, n = 0.0, 0
                while secs < 0.6:
                    secs += run(dec, t)
                    n += 1
                out["%s_%d" % ("decrypt" if dec else "encrypt", t)] = round(n * R * L / secs / (1 << 30), 2)
        assert fails.value == 0 and np.array_equal(pt, back), "cpu round trip failed"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
