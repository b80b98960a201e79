#!/usr/bin/env python3
"""Many-session batches by record length (noise_gpu_{en,de}crypt_sessions,
the keyed tile kernel: per-record key row and nonce, strided records) at a
fixed number of plaintext bytes per call.  Device-resident, HIP-event timed;
one JSON line per length: GiB/s of plaintext per direction.
    python tools/bench_sessions.py [total_MiB] [sessions] [lengths...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))
import noise_amd  # noqa: E402


def main():
    import torch
    total = (int(sys.argv[1]) if len(sys.argv) > 1 else 1024) << 20
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    lens = [int(x) for x in sys.argv[3:]] or [1024, 4096]
    noise_amd.load()
    torch.cuda.set_device(0)
    d_keys = torch.empty(S * 32, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d_keys, S * 32, 0x4B4559)
    for L in lens:
        R = total // L
        d_pt = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        noise_amd.fill_synthetic(d_pt, R * L, 7)
        i = torch.arange(R, dtype=torch.int64, device="cuda")
        d_idx = (i % S).to(torch.int32)
        d_non = ((i % S) << 32) + i // S
        d_ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
        d_back = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        d_st = torch.empty(R, dtype=torch.uint8, device="cuda")

        def enc():
            noise_amd.encrypt_sessions(d_keys, S, d_idx, d_non, d_pt, L, d_ct, L + 16, L, R)

        def dec():
            noise_amd.decrypt_sessions(d_keys, S, d_idx, d_non, d_ct, L + 16, d_back, L, L, d_st, R)
        for _ in range(10):
            enc()
            dec()
        torch.cuda.synchronize()
        assert torch.equal(d_pt, d_back) and int(d_st.sum()) == 0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        te = td = 0.0
        K = 20
        for _ in range(K):
            ev[0].record()
            enc()
            ev[1].record()
            dec()
            ev[2].record()
            torch.cuda.synchronize()
            te += ev[0].elapsed_time(ev[1])
            td += ev[1].elapsed_time(ev[2])
        gib = R * L / 2.0 ** 30
        print(json.dumps({"len": L, "records": R, "sessions": S,
                          "encrypt_GiBps": round(gib / (te / K / 1e3), 1),
                          "decrypt_GiBps": round(gib / (td / K / 1e3), 1),
                          "enc_ms": round(te / K, 4), "dec_ms": round(td / K, 4)}), flush=True)
        del d_pt, d_ct, d_back, d_st


if __name__ == "__main__":
    main()
