#!/usr/bin/env python3
"""In-place (strided) encrypt throughput: records of L bytes at a stride of
L + 16 (the caller encrypts its buffer in place, room for the tag), one key
(uniform) and 65536 keys (sessions).  Strided layouts take the tile kernel's
non-contiguous variants.  NOISE_AMD_LIB selects the library (A/B).

    python3 tools/bench_strided.py [L] [records]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-cpp_amd",
                                "python"))
import noise_amd  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    torch.cuda.set_device(0)
    noise_amd.load()
    buf = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(buf, R * (L + 16), 7)
    key = bytes(range(1, 33))
    t_u = timed(lambda: noise_amd.encrypt_uniform(key, 0, buf, L + 16, buf, L + 16, L, R))
    S = 65536
    keys = torch.empty(S * 32, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(keys, S * 32, 9)
    i = torch.arange(R, dtype=torch.int64, device="cuda")
    idx = (i % S).to(torch.int32)
    non = ((i % S) << 32) + i // S
    t_s = timed(lambda: noise_amd.encrypt_sessions(keys, S, idx, non, buf, L + 16, buf, L + 16, L, R))
    gib = R * L / 2**30
    print("strided in-place encrypt L=%d R=%d: uniform %.1f GiB/s (%.3f ms), sessions %.1f GiB/s (%.3f ms)"
          % (L, R, gib / t_u, t_u * 1e3, gib / t_s, t_s * 1e3))


if __name__ == "__main__":
    main()
