#!/usr/bin/env python3
"""Record-length sweep: GiB/s of plaintext through
encrypt and decrypt for one record length at a time, device-resident, HIP
events on the launch stream, every round trip checked before timing.

Layouts (one JSON line per layout and length):
  uniform-aligned  noise_gpu_{en,de}crypt_uniform, record strides rounded up to
                   16 bytes (plaintext ceil16(L), ciphertext ceil16(L + 16))
  uniform-packed   the same entry points, Noise wire format packed back to back
                   (strides L and L + 16: records at any byte alignment)
  records          noise_gpu_{en,de}crypt_records, one descriptor per record at
                   16-byte aligned offsets (the classifier path of config 4)

    python tools/bench_lengths.py [--mib N] [--layouts a,b] [lengths...]

Default lengths: the VERDICT's odd sizes beside the tile sizes around them."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))
import noise_amd  # noqa: E402

KEY = bytes(range(32))
ODD = [100, 300, 700, 1000, 1040, 1400, 3000, 5000, 9000, 16000]
TILES = [64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384]


def c16(x):
    return (x + 15) // 16 * 16


def run_one(torch, stream, layout, L, mib, reps):
    R = max(4096, (mib << 20) // L)
    if layout == "uniform-packed":
        si, so = L, L + 16
    else:
        si, so = c16(L), c16(L + 16)
    d_pt = torch.empty(R * si, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d_pt, R * si, 5)
    d_ct = torch.empty(R * so, dtype=torch.uint8, device="cuda")
    d_back = torch.zeros(R * si, dtype=torch.uint8, device="cuda")
    d_st = torch.empty(R, dtype=torch.uint8, device="cuda")
    if layout == "records":
        i = np.arange(R, dtype=np.uint64)
        d = np.zeros(R, dtype=noise_amd.record_dtype())
        d["in_off"], d["out_off"] = i * np.uint64(si), i * np.uint64(so)
        d["nonce"], d["len"], d["key_idx"] = i, L, 0
        dd = d.copy()
        dd["in_off"], dd["out_off"] = d["out_off"], d["in_off"]
        d_key = torch.frombuffer(bytearray(KEY), dtype=torch.uint8).cuda()
        d_enc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
        d_dec = torch.from_numpy(dd.view(np.uint8).copy()).cuda()

        def enc():
            noise_amd.encrypt_records(d_key, 1, d_enc, R, d_pt, d_ct, stream=stream)

        def dec():
            noise_amd.decrypt_records(d_key, 1, d_dec, R, d_ct, d_back, d_st, stream=stream)
    else:
        def enc():
            noise_amd.encrypt_uniform(KEY, 0, d_pt, si, d_ct, so, L, R, stream=stream)

        def dec():
            noise_amd.decrypt_uniform(KEY, 0, d_ct, so, d_back, si, L, d_st, R, stream=stream)
    enc()
    dec()
    torch.cuda.synchronize()
    ok = int(d_st.sum()) == 0 and torch.equal(d_pt.view(R, si)[:, :L], d_back.view(R, si)[:, :L])
    if not ok:
        raise SystemExit("round trip failed: %s L=%d" % (layout, L))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(3):
        enc()
        dec()
    te = td = 0.0
    for _ in range(reps):
        ev[0].record(stream)
        enc()
        ev[1].record(stream)
        dec()
        ev[2].record(stream)
        torch.cuda.synchronize()
        te += ev[0].elapsed_time(ev[1])
        td += ev[1].elapsed_time(ev[2])
    te, td = te / reps, td / reps
    return {"layout": layout, "len": L, "records": R, "enc_ms": round(te, 4), "dec_ms": round(td, 4),
            "enc_gib_s": round(R * L / te / 1e-3 / 2 ** 30, 1),
            "dec_gib_s": round(R * L / td / 1e-3 / 2 ** 30, 1),
            "round_trip_gib_s": round(2 * R * L / (te + td) / 1e-3 / 2 ** 30, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=2048, help="plaintext per length (MiB)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--layouts", default="uniform-aligned,uniform-packed,records")
    ap.add_argument("lengths", nargs="*", type=int)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    noise_amd.load()
    stream = torch.cuda.current_stream()
    lengths = a.lengths or sorted(set(ODD + TILES))
    for layout in a.layouts.split(","):
        for L in lengths:
            print(json.dumps(run_one(torch, stream, layout, L, a.mib, a.reps)), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
