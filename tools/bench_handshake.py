#!/usr/bin/env python3
"""Throughput of the batched GPU handshake (noise_gpu_hs_*, SURVEY §8(f)
rank 4): full Noise handshakes per second -- BOTH parties of each handshake,
fresh device-DRBG ephemerals, empty payloads, one static key per side (a
server key and a client key) -- HIP-event timed by bin/handshake_test
batch_bench, next to the reference's own primitives on host cores
(oracle/_ref ref_xx_bench: the same XX handshake pair composed from
monocypher.c's crypto_x25519 / crypto_blake2b / AEAD, 16 threads).
Prints one JSON line.   python tools/bench_handshake.py [n] [patterns...]"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "noise-cpp_amd", "bin", "handshake_test")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    patterns = sys.argv[2:] or ["XX", "IK", "NN", "XXpsk3"]
    gpu = {}
    for p in patterns:
        r = subprocess.run([BIN, "batch_bench", p, str(n), "3"], capture_output=True, text=True,
                           timeout=300)
        if r.returncode != 0:
            raise SystemExit(r.stdout + r.stderr)
        gpu[p] = json.loads(r.stdout.strip().splitlines()[-1])
    line = {"metric": "full Noise handshakes per second (both parties, batched on one GPU)",
            "value": gpu["XX"]["handshakes_per_s"] if "XX" in gpu else None,
            "unit": "handshakes/s", "sessions_per_batch": n,
            "patterns": {p: {"handshakes_per_s": g["handshakes_per_s"], "ms": g["ms"]}
                         for p, g in gpu.items()},
            "note": "one lane per session, one kernel per token; X25519 radix 2^25.5, "
                    "BLAKE2b/HMAC/HKDF and ChaChaPoly(AD=h) per lane; state in HBM"}
    ref = os.path.join(ROOT, "oracle", "_ref", "libnoise_ref.so")
    if os.path.exists(ref):
        lib = ctypes.CDLL(ref)
        lib.ref_xx_bench.restype = ctypes.c_double
        lib.ref_xx_bench.argtypes = [ctypes.c_long, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        threads = min(16, os.cpu_count() or 1)
        per = 400
        fails = ctypes.c_int()
        sec = lib.ref_xx_bench(per * threads, threads, ctypes.byref(fails))
        assert fails.value == 0
        cpu = open("/proc/cpuinfo").read().split("model name")[1].split(":")[1].split("\n")[0].strip()
        line["cpu_baseline"] = {
            "value": round(per * threads / sec), "unit": "handshakes/s", "cores": threads,
            "kind": "reference",
            "sample": "%d XX handshake pairs per thread on monocypher.c primitives "
                      "(oracle/_ref ref_xx_bench), %s" % (per, cpu)}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
