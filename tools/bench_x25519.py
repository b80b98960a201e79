#!/usr/bin/env python3
"""Throughput of the batched X25519 kernel (noise_gpu_x25519): n random
scalar multiplications per launch, HIP-event timed, next to the host X25519
(noise-cpp_amd/host/crypto.cpp via bin/handshake_test is per-call; here the
CPU figure is the pure-C++ ladder timed in a loop of the same binary).
Prints one JSON line.   python tools/bench_x25519.py [n]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))
import noise_amd  # noqa: E402


def main():
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    noise_amd.load()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(25519)
    d_s = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device="cuda", generator=g)
    d_p = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device="cuda", generator=g)
    d_o = torch.empty(32 * n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    def timed(points):
        for _ in range(3):
            noise_amd.x25519(d_s, points, d_o, n, stream=s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(s)
        for _ in range(reps):
            noise_amd.x25519(d_s, points, d_o, n, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    ms = timed(d_p)
    ms_base = timed(None)
    line = {"metric": "X25519 scalar multiplications per second (batched, device-resident)",
            "value": round(n / (ms * 1e-3)), "unit": "ops/s", "n": n, "ms_per_launch": round(ms, 3),
            "public_keys_per_s": round(n / (ms_base * 1e-3)), "ms_per_launch_public_keys": round(ms_base, 3),
            "note": "one lane per scalar multiplication, radix 2^25.5; variable base: RFC 7748 ladder; "
                    "public keys (base point): fixed-base edwards25519 radix-16 table"}
    ref = os.path.join(ROOT, "oracle", "_ref", "libnoise_ref.so")
    if os.path.exists(ref):  # the reference's own crypto_x25519 (monocypher.c) on host cores
        import ctypes
        lib = ctypes.CDLL(ref)
        lib.ref_x25519_bench.restype = ctypes.c_double
        lib.ref_x25519_bench.argtypes = [ctypes.c_long, ctypes.c_int]
        threads = min(16, os.cpu_count() or 1)
        per = 2000
        sec = lib.ref_x25519_bench(per * threads, threads)
        line["cpu_baseline"] = {"value": round(per * threads / sec), "unit": "ops/s", "cores": threads,
                                "kind": "reference",
                                "sample": "%d x crypto_x25519 per thread (monocypher.c via oracle/_ref)" % per}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
