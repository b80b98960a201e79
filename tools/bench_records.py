#!/usr/bin/env python3
"""Descriptor batches of uniform-size small records from many sessions
(noise_gpu_{en,de}crypt_records): the classifier routes every record to one
tile class (64 / 128 / 256 / 512 B: kTileDesc) or, at 1 KiB, to the segment
kernel.  Device-resident, HIP-event timed; prints one JSON line per size:
GiB/s of plaintext and M records/s per direction.
    python tools/bench_records.py [records] [sessions] [sizes...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))
import noise_amd  # noqa: E402


def main():
    import torch
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    sizes = [int(x) for x in sys.argv[3:]] or [64, 256, 512, 1024]
    noise_amd.load()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    rng = np.random.default_rng(1)
    d_keys = torch.from_numpy(rng.integers(0, 256, 32 * S, dtype=np.uint8)).cuda()
    for L in sizes:
        i = np.arange(R, dtype=np.uint64)
        d = np.zeros(R, dtype=noise_amd.record_dtype())
        d["in_off"], d["out_off"] = i * np.uint64(L), i * np.uint64(L + 16)
        d["key_idx"] = (i % np.uint64(S)).astype(np.uint32)
        d["nonce"] = i // np.uint64(S)
        d["len"] = L
        dd = d.copy()
        dd["in_off"], dd["out_off"] = d["out_off"], d["in_off"]
        d_pt = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        noise_amd.fill_synthetic(d_pt, R * L, 5)
        d_ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
        d_back = torch.empty_like(d_pt)
        d_st = torch.empty(R, dtype=torch.uint8, device="cuda")
        d_enc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
        d_dec = torch.from_numpy(dd.view(np.uint8).copy()).cuda()

        def once():
            noise_amd.encrypt_records(d_keys, S, d_enc, R, d_pt, d_ct, stream=stream)
            noise_amd.decrypt_records(d_keys, S, d_dec, R, d_ct, d_back, d_st, stream=stream)
        for _ in range(5):
            once()
        torch.cuda.synchronize()
        if not os.environ.get("NOISE_NO_CHECK"):  # ablation builds (timing only) skip it
            assert int(d_st.sum()) == 0 and torch.equal(d_pt, d_back)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        reps, te, td = 10, 0.0, 0.0
        for _ in range(reps):
            ev[0].record(stream)
            noise_amd.encrypt_records(d_keys, S, d_enc, R, d_pt, d_ct, stream=stream)
            ev[1].record(stream)
            noise_amd.decrypt_records(d_keys, S, d_dec, R, d_ct, d_back, d_st, stream=stream)
            ev[2].record(stream)
            torch.cuda.synchronize()
            te += ev[0].elapsed_time(ev[1])
            td += ev[1].elapsed_time(ev[2])
        te, td = te / reps, td / reps
        print(json.dumps({"records": R, "sessions": S, "len": L,
                          "enc_ms": round(te, 4), "dec_ms": round(td, 4),
                          "enc_gib_s": round(R * L / te / 1e-3 / 2 ** 30, 1),
                          "dec_gib_s": round(R * L / td / 1e-3 / 2 ** 30, 1),
                          "enc_mrec_s": round(R / te / 1e3, 1), "dec_mrec_s": round(R / td / 1e3, 1)}))
        del d_pt, d_ct, d_back


if __name__ == "__main__":
    main()
