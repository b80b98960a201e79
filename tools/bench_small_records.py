#!/usr/bin/env python3
"""Device-resident descriptor batches of a few records (noise_gpu_encrypt_records
/ _decrypt_records): time per call (encrypt + decrypt, stream-synchronised)
by batch size and record length -- the classifier threshold's trade-off
(below it the generic lane-per-record kernel runs alone; above it the
classifier and the class kernels).  NOISE_AMD_LIB selects the library.

    python3 tools/bench_small_records.py"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))
import noise_amd  # noqa: E402

noise_amd.load()
key = torch.frombuffer(bytearray(range(32)), dtype=torch.uint8).cuda()
out = {}
for L in (64, 1024, 16384):
    for R in (100, 300, 1000, 2000, 4000):
        d = np.zeros(R, dtype=noise_amd.record_dtype())
        d["in_off"] = np.arange(R, dtype=np.uint64) * np.uint64(L)
        d["out_off"] = np.arange(R, dtype=np.uint64) * np.uint64(L + 16)
        d["nonce"] = np.arange(R, dtype=np.uint64)
        d["len"] = L
        dd = d.copy()
        dd["in_off"], dd["out_off"] = d["out_off"], d["in_off"]
        de = torch.from_numpy(d.view(np.uint8).copy()).cuda()
        ddec = torch.from_numpy(dd.view(np.uint8).copy()).cuda()
        pt = torch.randint(0, 256, (R * L,), dtype=torch.uint8, device="cuda")
        ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
        back = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        st = torch.empty(R, dtype=torch.uint8, device="cuda")
        for _ in range(5):
            noise_amd.encrypt_records(key, 1, de, R, pt, ct)
            noise_amd.decrypt_records(key, 1, ddec, R, ct, back, st)
        torch.cuda.synchronize()
        n = 40
        t0 = time.perf_counter()
        for _ in range(n):
            noise_amd.encrypt_records(key, 1, de, R, pt, ct)
            noise_amd.decrypt_records(key, 1, ddec, R, ct, back, st)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / n
        assert torch.equal(pt, back) and int(st.sum()) == 0
        out["%dx%d" % (R, L)] = round(t * 1e6, 1)
print(json.dumps({"lib": os.path.basename(os.environ.get("NOISE_AMD_LIB", "in-tree")),
                  "us_per_enc_dec_pair": out}))
