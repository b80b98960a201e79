#!/usr/bin/env python3
"""Benchmark of the MI355X Noise ChaChaPoly record engine (BASELINE.json).

Metric: GiB/s of ChaChaPoly AEAD over device-resident 1 KiB Noise records.
Workload (default, BASELINE config 2 = configs[1]): per GPU, R = 2^20 records
of 1024 B under one post-handshake key k = 00..1f, nonces n = rank*R + i,
plaintext from splitmix64(seed 0x4E4F495345).  One step = encrypt all R
records (pt -> ct||tag) + decrypt all R records (ct||tag -> pt, tag verified),
two kernel launches on one HIP stream.  `value` counts plaintext bytes through
the AEAD (encrypt + decrypt) of all ranks / wall time of the K timed steps
(max over ranks), in GiB/s (2^30 B/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|3|4|5]
                    [--no-cpu-baseline] [--no-config1] [--host-inclusive]

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
each process is one rank.  Run directly with --gpus N > 1, this process is
only a launcher: before touching any GPU it starts N copies of itself with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set and
exits with their status; rank 0 prints the JSON line.  Records shard per GPU
with no data-path collective (cfg 2/3/4 weak scaling: each rank its own R
records and nonce range; cfg 5 strong scaling: one 8 Mi-record range cut in
contiguous slices).  torch.distributed carries only the barrier, the
max-over-ranks of the elapsed time and the per-rank shard table, over gloo
(host TCP): with no data-path exchange there is nothing for RCCL to carry,
and an initialised RCCL communicator slows every kernel on the GPU by 6-12 %
(same-box A/B, tools/gpu/dist_ab.sh; profiles/round2/ab/ab_experiments.md).
The barriers are bracketed by torch.cuda.synchronize() on both sides.

--stub (tests only, CPU): the same launcher, rank bookkeeping, barriers and
reductions over gloo, with a trivial host workload instead of the GPU.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "noise-cpp_amd", "python"))

import noise_amd  # noqa: E402  (lazy: loads the library on first use)

SEED = 0x4E4F495345
KEY = bytes(range(32))
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue roof: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 4
# cycles per SIMD at the 2.4 GHz max clock.  4 cycles is the measured cost of
# every instruction in a ChaCha / Poly1305 stream on gfx950 (alignbit,
# mad_u64_u32, add_co: "slow" class; a stream mixing them with the 2-cycle
# add/xor runs all of it at ~4 cycles: profiles/round2/issue_bench.txt,
# profiles/round2/valu_classes.txt).
VALU_PEAK = 1024 * 2.4e9 / 4.0  # wave-instructions / s
GIB = float(1 << 30)
SHARE_CPUS = 16  # host CPU share of one GPU on the GPU box


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def shard(total, rank, world):
    """Contiguous [lo, hi) slice of `total` units for `rank` (strong scaling)."""
    return total * rank // world, total * (rank + 1) // world


def rank_nonce_base(cfg, rank, world, per_rank, total):
    """First nonce of a rank's records: weak scaling (cfg 2) gives every rank
    its own R-record nonce range; strong scaling (cfg 5) splits one range."""
    if cfg == 5:
        return shard(total, rank, world)[0]
    return rank * per_rank


def json_stdout():
    """Keep the process's stdout for the one JSON line: point fd 1 at stderr
    and return a writer on the original stdout."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def reduce_over_ranks(dist, elapsed, nrec, device):
    """Max of the elapsed time and sum of the records over ranks."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([nrec], dtype=torch.int64, device=device)
    dist.all_reduce(n)
    return float(t.item()), int(n.item())


def device_info(args, local):
    """The rank's device: index, name and PCI bus id (the stub: the host, with
    a made-up PCI address per rank -- or one shared by all ranks with the
    test hook --stub-same-device -- so that the aliasing check runs)."""
    if args.stub:
        bus = 0 if args.stub_same_device else int(os.environ.get("RANK", "0"))
        return {"index": None, "name": "cpu (stub)", "pci_domain_id": 0, "pci_bus_id": bus,
                "pci_device_id": 0}
    import torch
    p = torch.cuda.get_device_properties(local)
    info = {"index": local, "name": p.name}
    for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"):
        if hasattr(p, k):
            info[k] = getattr(p, k)
    return info


def device_key(dev):
    """A device's identity across processes: its PCI address, or None when the
    runtime does not report one."""
    if not dev or dev.get("pci_bus_id") is None:
        return None
    return (dev.get("pci_domain_id", 0), dev["pci_bus_id"], dev.get("pci_device_id", 0))


def check_shards(shards, share_device=False):
    """Rank shard table -> error text if two ranks share a nonce, or -- unless
    the ranks were told to share the visible GPUs (--share-device, a test
    hook) -- two ranks ran on one device: an N-rank line whose ranks doubled
    up on a card (a LOCAL_RANK or visibility mishap) is not an N-GPU figure."""
    spans = sorted((s["nonce_lo"], s["nonce_hi"], s["rank"]) for s in shards)
    for a, b in zip(spans, spans[1:]):
        if b[0] < a[1]:
            return "ranks %d and %d share nonces [%d, %d)" % (a[2], b[2], b[0], min(a[1], b[1]))
    if not share_device:
        seen = {}
        for s in sorted(shards, key=lambda x: x["rank"]):
            k = device_key(s.get("device"))
            if k is None:
                continue
            if k in seen:
                return "ranks %d and %d ran on the same device (PCI %04x:%02x:%02x); an N-GPU line needs " \
                       "one device per rank" % (seen[k], s["rank"], k[0], k[1], k[2])
            seen[k] = s["rank"]
    return None


def rank_spread(shards):
    """max / min over ranks of each rank's own per-launch times (1.0 = even)."""
    out = {}
    for f in ("enc_ms", "dec_ms", "step_ms"):
        v = [s[f] for s in shards if s.get(f)]
        if v:
            out[f] = {"min": min(v), "max": max(v), "max_over_min": round(max(v) / min(v), 4)}
    return out


# ---------------------------------------------------------------- launcher
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args, argv):
    """--gpus N > 1 without WORLD_SIZE: start N ranks of this script (one per
    GPU) and return their worst exit status.  Nothing here touches a GPU:
    torch.cuda.device_count() does not initialise the device on this image."""
    n = args.gpus
    if not args.stub:
        import torch
        have = torch.cuda.device_count()
        if have < n and not args.share_device:
            raise SystemExit("bench.py --gpus %d: only %d GPU(s) visible" % (n, have))
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log("a rank exited with status %d; stopping the others" % code)
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------- profiles
def latest_profile(cfg):
    """Per-kernel PMC means of the newest committed profile of config `cfg`
    (profiles/roundNN/cfgN/pmc_summary.json, tools/gpu/profile_cfg.sh)."""
    pdir = os.path.join(ROOT, "profiles")
    best = None
    if os.path.isdir(pdir):
        for sub in sorted(os.listdir(pdir)):
            f = os.path.join(pdir, sub, "cfg%d" % cfg, "pmc_summary.json")
            if os.path.exists(f):
                best = (os.path.relpath(f, ROOT), json.load(open(f)))
    return best


def pmc_kernels(prof, names, anchor=None):
    """Sum the per-dispatch PMC means of the kernels whose symbol starts with
    one of `names`, per call: a kernel launched k times per call (the
    decrypt pipeline's chunks) counts k times -- its dispatches in the
    profiled run over those of `anchor`, a kernel launched once per call of
    this direction (kernels both directions launch, over both anchors)."""
    if not prof:
        return None
    ks = prof[1]["kernels"]
    rows = [(k, v) for k, v in ks.items() if any(k.startswith(n) for n in names)]
    if not rows:
        return None

    def calls(k):
        if not anchor or "_dispatches" not in ks.get(anchor, {}):
            return None
        if "<true" in k or "<false" in k:
            return ks[anchor]["_dispatches"]
        other = anchor.replace("<true", "<false") if "<true" in anchor else anchor.replace("<false", "<true")
        return ks[anchor]["_dispatches"] + ks.get(other, {}).get("_dispatches", 0)

    out = {}
    for k, r in rows:
        n = calls(k)
        f = r["_dispatches"] / n if n and r.get("_dispatches") else 1.0
        for c, v in r.items():
            if c != "_dispatches":
                out[c] = out.get(c, 0.0) + v * f
    return out


# ---------------------------------------------------------------- cpu leg
def cpu_sample(cfg, orc, nbytes, jitter=False):
    """A bounded sample of config `cfg`'s own records (same seeds, shapes and
    nonces as make_workload, rank 0), about `nbytes` of plaintext, as a
    descriptor batch: (key table, descriptors, plaintext, ct buffer size,
    description)."""
    import numpy as np
    rd = noise_amd.record_dtype()
    if cfg in (2, 5):
        L = 1024 if cfg == 2 else 4096
        R = max(64, nbytes // L)
        lens = np.full(R, L, dtype=np.uint64)
        keys = np.frombuffer(KEY, dtype=np.uint8).copy()
        kidx = np.zeros(R, dtype=np.uint32)
        nonce = np.arange(R, dtype=np.uint64)
        what = "%d x %d B records, one key, nonces 0.." % (R, L)
    elif cfg == 3:
        S, L = 65536, 1024
        R = max(64, nbytes // L)
        i = np.arange(R, dtype=np.uint64)
        lens = np.full(R, L, dtype=np.uint64)
        keys = np.frombuffer(orc.synthetic(S * 32, 0x4B4559), dtype=np.uint8).copy()
        kidx = (i % np.uint64(S)).astype(np.uint32)
        nonce = ((i % np.uint64(S)) << np.uint64(32)) + i // np.uint64(S)
        what = ("the first %d records of the 65536-session x 16 batch (record i: session i mod "
                "65536, nonce (s << 32) + i div 65536), 1 KiB" % R)
    elif cfg == 4:
        allr = zipf_lengths(1 << 20, jitter)
        csum = np.cumsum(allr)
        R = int(max(64, np.searchsorted(csum, nbytes)))
        lens = allr[:R]
        keys = np.frombuffer(KEY, dtype=np.uint8).copy()
        kidx = np.zeros(R, dtype=np.uint32)
        nonce = np.arange(R, dtype=np.uint64)
        what = ("the first %d records of the %sZipf batch (64 B .. 65519 B, mean %d B), one key"
                % (R, "jittered " if jitter else "", int(lens.sum() // R)))
    else:
        raise ValueError(cfg)
    in_sz = (lens + np.uint64(15)) // np.uint64(16) * np.uint64(16)
    ct_sz = (lens + np.uint64(31)) // np.uint64(16) * np.uint64(16)
    d = np.zeros(R, dtype=rd)
    d["in_off"] = np.concatenate([[0], np.cumsum(in_sz)[:-1]]).astype(np.uint64)
    d["out_off"] = np.concatenate([[0], np.cumsum(ct_sz)[:-1]]).astype(np.uint64)
    d["nonce"], d["len"], d["key_idx"] = nonce, lens, kidx
    pt = np.frombuffer(orc.synthetic(int(in_sz.sum()), SEED), dtype=np.uint8).copy()
    return keys, d, pt, int(ct_sz.sum()), int(lens.sum()), what


def cpu_baseline(cfg=2, jitter=False):
    """The reference's own monocypher.c (oracle/_ref: the reference source
    built by oracle/Makefile, with the noise::encrypt / decrypt nonce framing
    of noise.cpp:202-281) -- or the build's C restatement if _ref is absent --
    on this host's cores, BASELINE.md section 3: a bounded sample of this
    config's own records (cpu_sample), one noise::encrypt / decrypt call per
    record, encrypt and decrypt timed separately at 1 thread, at the GPU's
    host CPU share (16) and at nproc threads, plus a 1 -> 16 thread encrypt
    line.  Each figure repeats whole passes over the sample until it has
    >= 0.5-1 s of wall time (~8 s in all)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    orc = oracle_lib.Oracle()
    ncpu = os.cpu_count() or 1
    share = min(SHARE_CPUS, ncpu)
    keys, desc, pt, ct_bytes, pt_bytes, what = cpu_sample(cfg, orc, 256 << 20, jitter)
    R = len(desc)
    ct = np.zeros(ct_bytes, dtype=np.uint8)
    back = np.zeros(len(pt), dtype=np.uint8)
    ddesc = desc.copy()
    ddesc["in_off"], ddesc["out_off"] = desc["out_off"], desc["in_off"]
    kind = "reference" if orc.ref is not None else "port"
    fn = orc.ref.ref_batch_records if orc.ref is not None else orc.lib.oracle_batch_records
    fails = ctypes.c_int(0)

    def run(dec, nthr):
        if dec:
            return fn(1, keys.ctypes.data, ddesc.ctypes.data, R, ct.ctypes.data, back.ctypes.data,
                      nthr, ctypes.byref(fails))
        return fn(0, keys.ctypes.data, desc.ctypes.data, R, pt.ctypes.data, ct.ctypes.data, nthr,
                  ctypes.byref(fails))

    def rate(dec, nthr, seconds):
        run(dec, nthr)  # warm (and, for decrypt, checks the ciphertext below)
        t, passes = 0.0, 0
        while t < seconds:
            t += run(dec, nthr)
            passes += 1
        return passes * pt_bytes / t / GIB

    enc, dec = {}, {}
    for nthr, secs in ((1, 1.0), (share, 0.6), (ncpu, 0.6)):
        if str(nthr) in enc:
            continue
        enc[str(nthr)] = rate(False, nthr, secs)
        dec[str(nthr)] = rate(True, nthr, secs)
    # the round trip of the sample is exact: every tag verified, plaintext back
    lens = desc["len"].astype(np.int64)
    ok = fails.value == 0
    for i in range(0, R, max(1, R // 512)):
        o = int(desc["in_off"][i])
        ok = ok and np.array_equal(pt[o:o + lens[i]], back[o:o + lens[i]])
    assert ok, "cpu baseline round trip failed"
    scaling = {}
    t = 1
    while t <= share:
        scaling[str(t)] = round(enc[str(t)] if str(t) in enc else rate(False, t, 0.3), 3)
        t *= 2
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    rt = {k: 2.0 / (1.0 / enc[k] + 1.0 / dec[k]) for k in enc}  # enc+dec round trip, like `value`
    best = max(rt, key=lambda k: rt[k])
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = ncpu
    return {"value": round(rt[best], 3), "unit": "GiB/s", "cores": int(best), "kind": kind,
            "config": cfg,
            "encrypt_GiBps": {k: round(v, 3) for k, v in enc.items()},
            "decrypt_GiBps": {k: round(v, 3) for k, v in dec.items()},
            "round_trip_GiBps": {k: round(v, 3) for k, v in rt.items()},
            "encrypt_thread_scaling_GiBps": scaling,
            "cpu_model": model, "nproc": ncpu, "affinity_cpus": affinity, "host_share": share,
            "sample": "%s (%.0f MiB of plaintext); one noise::encrypt / decrypt call per record, "
                      "encrypt and decrypt timed separately at 1, %d (the GPU's host CPU share) and "
                      "%d (nproc) threads; value = the best enc+dec round-trip rate, at %s threads; %s"
                      % (what, pt_bytes / 2**20, share, ncpu, best,
                         "monocypher.c via oracle/_ref" if kind == "reference"
                         else "oracle/chachapoly_oracle.c")}


def config1(orc=None):
    """BASELINE config 1 (examples/Noise_XX_25519_ChaChaPoly_Blake2b.cpp:26-75):
    XX loopback handshake + 1000 x 1 KiB records each way, record by record
    (encrypt_with_ad / decrypt_with_ad), through the build's noise::
    HandshakeState / CipherState (noise-cpp_amd/bin/config1_bench, every AEAD
    on the GPU), beside the reference's Monocypher AEAD + handshake on one
    host thread (oracle/_ref), in the same run."""
    tool = os.path.join(ROOT, "noise-cpp_amd", "bin", "config1_bench")
    if not os.path.exists(tool):
        return {"error": "noise-cpp_amd/bin/config1_bench not built"}
    # resident: the opt-in latency mode (noise_gpu_set_resident: one resident
    # workgroup, no launch per record); launch: one kernel launch per record
    out = {}
    for mode in ("resident", "launch"):
        p = subprocess.run([tool, "1000", "1024", mode], capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            return {"error": "config1_bench %s failed: %s" % (mode, p.stderr[-500:])}
        out["build" if mode == "resident" else "build_launch"] = json.loads(p.stdout.strip().splitlines()[-1])
    if orc is None:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        orc = oracle_lib.Oracle()
    if orc.ref is not None:
        import numpy as np
        fails = ctypes.c_int(0)
        hs = min(orc.ref.ref_xx_bench(64, 1, ctypes.byref(fails)) / 64 for _ in range(3))
        L, R = 1024, 1000
        pt = np.frombuffer(orc.synthetic(R * L, SEED), dtype=np.uint8).copy()
        ct = np.zeros(R * (L + 16), dtype=np.uint8)
        back = np.zeros(R * L, dtype=np.uint8)
        te = min(orc.ref.ref_batch_uniform(0, KEY, 0, pt.ctypes.data, L, ct.ctypes.data, L + 16, L, R, 1,
                                           ctypes.byref(fails)) for _ in range(5))
        td = min(orc.ref.ref_batch_uniform(1, KEY, 0, ct.ctypes.data, L + 16, back.ctypes.data, L, L, R,
                                           1, ctypes.byref(fails)) for _ in range(5))
        out["reference"] = {"handshake_ms": round(hs * 1e3, 4),
                            "encrypt_1000_ms": round(te * 1e3, 3), "decrypt_1000_ms": round(td * 1e3, 3),
                            "per_record_us": round((te + td) / 2 / R * 1e6, 3),
                            "note": "monocypher.c (oracle/_ref), 1 host thread; XX handshake = both "
                                    "parties incl. key generation (ref_xx_bench)"}
    return out


# ---------------------------------------------------------------- workloads
METRIC = "GiB/s ChaChaPoly AEAD over device-resident 1 KiB Noise records, 1 & 8 GPU"


def mix64_np(z):
    import numpy as np
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


JITTER_SEED = 0x4A4954  # "JIT"


def zipf_lengths(R, jitter=False):
    """Config 4 record lengths: 64 * 2^k, P(k) ~ 1/(k+1), k = 0..10 drawn by
    inverse CDF from splitmix64(seed 4); the top bucket clamped to 65519.
    jitter: the same buckets, each length lowered by
    U(0..63) (splitmix64(seed 0x4A4954) mod 64), so that almost no record has
    a power-of-two size: 64 * 2^k - U, clamped to 1 .. 65519."""
    import numpy as np
    w = np.array([1.0 / (k + 1) for k in range(11)])
    cdf = np.cumsum(w / w.sum())
    i1 = np.arange(R, dtype=np.uint64) + np.uint64(1)
    u = mix64_np(np.uint64(4) + i1 * np.uint64(0x9e3779b97f4a7c15)).astype(np.float64) / 2.0 ** 64
    k = np.minimum(np.searchsorted(cdf, u, side="right"), 10)
    lens = (64 << k).astype(np.int64)
    if jitter:
        lens -= (mix64_np(np.uint64(JITTER_SEED) + i1 * np.uint64(0x9e3779b97f4a7c15)) %
                 np.uint64(64)).astype(np.int64)
    return np.clip(lens, 1, 65519).astype(np.uint64)


def tile_symbol(dec, L, contig, mode):
    return "noise_amd::k_aead_tile<%s, %d, %s, %d, 0, 1, 256>" % (
        "true" if dec else "false", L, "true" if contig else "false", mode)


def make_stub_workload(args, rank, world):
    """--stub: host-only stand-in with the real shard bookkeeping."""
    import numpy as np
    if args.config == 5:  # strong scaling: this rank's slice of one 8 Mi-record range
        total = args.records or (8 << 20)
        lo, hi = shard(total, rank, world)
        R, L = hi - lo, 16
        n_base = rank_nonce_base(5, rank, world, R, total)
    else:
        R, L = args.records or 1024, 64
        n_base = rank_nonce_base(2, rank, world, R, R * world)
    buf = np.zeros(R * L, dtype=np.uint8)

    def step(evs=None):
        np.bitwise_xor(buf, 0x5A, out=buf)
    return {"R": R, "L": L, "n_base": n_base, "workload": "stub: %d x %d B host records per rank" % (R, L),
            "step": step, "check": lambda: True, "metric": "stub", "config": {"record_bytes": L},
            "pt_bytes": R * L, "enc_bytes": R * (2 * L + 16), "dec_bytes": R * (2 * L + 17),
            "read_bytes": (R * L, R * (L + 16)), "knames": (("stub",), ("stub",))}


def make_workload(cfg, args, rank, world, stream):
    """Synthetic inputs of BASELINE config `cfg`, resident in
    HBM, and the step that runs the hot path over them once."""
    import numpy as np
    import torch
    if cfg in (2, 5):
        if cfg == 2:
            R, L = args.records or (1 << 20), 1024
            workload = "cfg2: 2^20 x 1 KiB records per GPU, one key, encrypt+decrypt round trip"
            if args.records:
                workload = "cfg2-shape: %d x 1 KiB records per GPU" % R
            n_base = rank_nonce_base(cfg, rank, world, R, R * world)
            metric = METRIC
        else:  # strong scaling: 8 Mi x 4 KiB split over the GPUs
            total = args.records or (8 << 20)
            lo, hi = shard(total, rank, world)
            R, L = hi - lo, 4096
            n_base = rank_nonce_base(cfg, rank, world, R, total)
            workload = "cfg5: %d x 4 KiB records total, sharded over %d GPU(s)" % (total, world)
            metric = "GiB/s ChaChaPoly AEAD over device-resident 4 KiB Noise records"
        d_pt = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        noise_amd.fill_synthetic(d_pt, R * L, SEED, offset=n_base * L)
        d_ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
        d_back = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        d_st = torch.empty(R, dtype=torch.uint8, device="cuda")

        def step(evs=None):
            if evs:
                evs[0].record(stream)
            noise_amd.encrypt_uniform(KEY, n_base, d_pt, L, d_ct, L + 16, L, R, stream=stream)
            if evs:
                evs[1].record(stream)
            noise_amd.decrypt_uniform(KEY, n_base, d_ct, L + 16, d_back, L, L, d_st, R, stream=stream)
            if evs:
                evs[2].record(stream)
        cfgd = {"record_bytes": L, "ct_stride": L + 16, "keys": 1}
        knames = ((tile_symbol(False, L, True, 0),), (tile_symbol(True, L, True, 0),))
        meta = 0
        oracle = {"kind": "uniform", "R": R, "L": L, "n_base": n_base, "key": KEY, "seed": SEED,
                  "data_offset": n_base * L, "pt": d_pt, "ct": d_ct, "back": d_back, "status": d_st}
    elif cfg == 3:
        # 65536 sessions x 16 records x 1 KiB, interleaved: record i belongs to
        # session s = i mod S with nonce (s << 32) + i // S; key of session s =
        # bytes [32s, 32s+32) of the splitmix64 stream with seed 0x4B4559.
        S, per, L = 65536, 16, 1024
        R = S * per
        n_base = rank * R
        d_pt = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        noise_amd.fill_synthetic(d_pt, R * L, SEED, offset=rank * R * L)
        d_keys = torch.empty(S * 32, dtype=torch.uint8, device="cuda")
        noise_amd.fill_synthetic(d_keys, S * 32, 0x4B4559, offset=rank * S * 32)
        i = torch.arange(R, dtype=torch.int64, device="cuda")
        d_idx = (i % S).to(torch.int32)
        d_non = ((i % S) << 32) + i // S
        d_ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
        d_back = torch.empty(R * L, dtype=torch.uint8, device="cuda")
        d_st = torch.empty(R, dtype=torch.uint8, device="cuda")

        def step(evs=None):
            if evs:
                evs[0].record(stream)
            noise_amd.encrypt_sessions(d_keys, S, d_idx, d_non, d_pt, L, d_ct, L + 16, L, R,
                                       stream=stream)
            if evs:
                evs[1].record(stream)
            noise_amd.decrypt_sessions(d_keys, S, d_idx, d_non, d_ct, L + 16, d_back, L, L, d_st, R,
                                       stream=stream)
            if evs:
                evs[2].record(stream)
        workload = "cfg3: 65536 sessions x 16 records x 1 KiB per GPU, interleaved, per-record key+nonce"
        metric = "GiB/s ChaChaPoly AEAD over device-resident 1 KiB Noise records, 64K sessions"
        cfgd = {"record_bytes": L, "ct_stride": L + 16, "keys": S,
                "session_nonces": "(s << 32) + i // 65536 (the rank is in the key, not the nonce)"}
        knames = ((tile_symbol(False, L, True, 1),), (tile_symbol(True, L, True, 1),))
        meta = 12 * R + 32 * S  # 4-B key index + 8-B nonce per record, key table

        def oracle_descs():
            r = np.arange(R, dtype=np.uint64)
            enc = np.zeros(R, dtype=noise_amd.record_dtype())
            enc["in_off"], enc["out_off"] = r * np.uint64(L), r * np.uint64(L + 16)
            enc["nonce"] = ((r % np.uint64(S)) << np.uint64(32)) + r // np.uint64(S)
            enc["len"], enc["key_idx"] = L, (r % np.uint64(S)).astype(np.uint32)
            dec = enc.copy()
            dec["in_off"], dec["out_off"] = enc["out_off"], enc["in_off"]
            return enc, dec
        oracle = {"kind": "records", "n_base": n_base, "keys": d_keys, "descs": oracle_descs,
                  "seed": SEED, "data_offset": rank * R * L, "pt_bytes": R * L,
                  "pt": d_pt, "ct": d_ct, "back": d_back, "status": d_st}
    elif cfg == 4:
        R = args.records or (1 << 20)
        lens = zipf_lengths(R, args.jitter)
        # records packed at 16-byte alignment (--rec-align: a layout study)
        al = np.uint64(args.rec_align)
        in_sz = (lens + al - np.uint64(1)) // al * al
        ct_sz = (lens + np.uint64(16) + al - np.uint64(1)) // al * al
        in_off = np.concatenate([[0], np.cumsum(in_sz)[:-1]]).astype(np.uint64)
        ct_off = np.concatenate([[0], np.cumsum(ct_sz)[:-1]]).astype(np.uint64)
        n_base = rank * R
        enc_d = np.zeros(R, dtype=noise_amd.record_dtype())
        enc_d["in_off"], enc_d["out_off"] = in_off, ct_off
        enc_d["nonce"] = np.arange(R, dtype=np.uint64) + np.uint64(n_base)
        enc_d["len"] = lens
        dec_d = enc_d.copy()
        dec_d["in_off"], dec_d["out_off"] = ct_off, in_off
        tot_in, tot_ct = int(in_sz.sum()), int(ct_sz.sum())
        d_pt = torch.empty(tot_in, dtype=torch.uint8, device="cuda")
        noise_amd.fill_synthetic(d_pt, tot_in, SEED)
        d_ct = torch.empty(tot_ct, dtype=torch.uint8, device="cuda")
        d_back = torch.empty(tot_in, dtype=torch.uint8, device="cuda")
        d_st = torch.empty(R, dtype=torch.uint8, device="cuda")
        d_key = torch.frombuffer(bytearray(KEY), dtype=torch.uint8).cuda()
        d_enc = torch.from_numpy(enc_d.view(np.uint8).copy()).cuda()
        d_dec = torch.from_numpy(dec_d.view(np.uint8).copy()).cuda()
        L = int(lens.sum() // R)

        def step(evs=None):
            if evs:
                evs[0].record(stream)
            noise_amd.encrypt_records(d_key, 1, d_enc, R, d_pt, d_ct, stream=stream)
            if evs:
                evs[1].record(stream)
            noise_amd.decrypt_records(d_key, 1, d_dec, R, d_ct, d_back, d_st, stream=stream)
            if evs:
                evs[2].record(stream)
        workload = "cfg4: 2^20 records per GPU, 64 B .. 65519 B (P(k) ~ 1/(k+1)), one key"
        if args.jitter:
            workload = ("cfg4-jitter: 2^20 records per GPU, 64 * 2^k - U(0..63) B (P(k) ~ 1/(k+1)), "
                        "clamped to 1 .. 65519, one key")
        metric = "GiB/s ChaChaPoly AEAD over device-resident mixed-size Noise records"
        cfgd = {"mean_record_bytes": L, "total_plaintext_bytes": int(lens.sum()), "keys": 1,
                "jitter": bool(args.jitter), "record_align": int(args.rec_align),
                "records_pow2_len": int(np.count_nonzero((lens & (lens - np.uint64(1))) == 0))}
        pt_bytes = int(lens.sum())
        lens_t = torch.from_numpy(lens.astype(np.int64)).cuda()
        off_t = torch.from_numpy(in_off.astype(np.int64)).cuda()

        def check():
            if int(d_st.sum().item()) != 0:
                return False
            # sampled exact comparison of whole records (the padding is not a record byte)
            idx = torch.randint(0, R, (256,), device="cuda").tolist() + [R - 1]
            for r in idx:
                o, n = int(off_t[r]), int(lens_t[r])
                if not torch.equal(d_pt[o:o + n], d_back[o:o + n]):
                    return False
            return True
        ct_bytes = int((lens + 16).sum())
        oracle = {"kind": "records", "n_base": n_base, "keys": np.frombuffer(KEY, dtype=np.uint8).copy(),
                  "descs": lambda: (enc_d, dec_d), "seed": SEED, "data_offset": 0,
                  "pt_bytes": tot_in, "pt": d_pt, "ct": d_ct, "back": d_back, "status": d_st}
        # the whole records call (classifier, segment / tail / small-class /
        # generic kernels, finalize): every noise_amd kernel of the direction
        return {"R": R, "L": L, "n_base": n_base, "workload": workload, "step": step, "check": check,
                "metric": metric, "config": cfgd, "pt_bytes": pt_bytes,
                "enc_bytes": pt_bytes + ct_bytes + 48 * R, "dec_bytes": pt_bytes + ct_bytes + 49 * R,
                "read_bytes": (pt_bytes + 48 * R, ct_bytes + 48 * R),
                "knames": (("noise_amd::k_cls_", "noise_amd::k_seg_prep", "noise_amd::k_aead_mtile<false",
                            "noise_amd::k_seg_finalize_w<false", "noise_amd::k_aead_tile<false",
                            "noise_amd::k_aead_records<false"),
                           ("noise_amd::k_cls_", "noise_amd::k_seg_prep", "noise_amd::k_aead_mtile<true",
                            "noise_amd::k_seg_finalize_w<true", "noise_amd::k_aead_tile<true",
                            "noise_amd::k_aead_records<true")),
                "call_level": True, "oracle": oracle,
                "pmc_anchor": ("noise_amd::k_aead_records<false>", "noise_amd::k_aead_records<true>")}
    else:
        raise SystemExit("unknown config %d" % cfg)

    def check():
        return int(d_st.sum().item()) == 0 and torch.equal(d_pt, d_back)
    return {"R": R, "L": L, "n_base": n_base, "workload": workload, "step": step, "check": check,
            "metric": metric, "config": cfgd, "pt_bytes": R * L,
            "enc_bytes": R * (2 * L + 16) + meta, "dec_bytes": R * (2 * L + 17) + meta,
            "read_bytes": (R * L + meta, R * (L + 16) + meta), "knames": knames, "oracle": oracle}


def host_inclusive(R, L):
    """Pinned host buffers -> chunked H2D || kernel || D2H pipeline (3 streams),
    the whole call timed (persistent per-device pipeline context)."""
    import torch
    lib = noise_amd.load()
    pt = torch.empty(R * L, dtype=torch.uint8).pin_memory()
    d = torch.empty(R * L, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d, R * L, SEED)
    pt.copy_(d)
    del d
    ct = torch.empty(R * (L + 16), dtype=torch.uint8).pin_memory()
    back = torch.empty(R * L, dtype=torch.uint8).pin_memory()
    st = torch.empty(R, dtype=torch.uint8).pin_memory()
    te, td = ctypes.c_double(), ctypes.c_double()
    best_e = best_d = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        assert lib.noise_gpu_encrypt_uniform_host(KEY, 0, ctypes.c_void_p(pt.data_ptr()), L,
                                                  ctypes.c_void_p(ct.data_ptr()), L + 16, L, R,
                                                  ctypes.byref(te)) == 0
        t1 = time.perf_counter()
        assert lib.noise_gpu_decrypt_uniform_host(KEY, 0, ctypes.c_void_p(ct.data_ptr()), L + 16,
                                                  ctypes.c_void_p(back.data_ptr()), L, L,
                                                  ctypes.c_void_p(st.data_ptr()), R,
                                                  ctypes.byref(td)) == 0
        t2 = time.perf_counter()
        best_e, best_d = min(best_e, t1 - t0), min(best_d, t2 - t1)
    assert torch.equal(pt, back) and int(st.sum()) == 0
    return {"encrypt_GiBps": round(R * L / best_e / GIB, 2),
            "decrypt_GiBps": round(R * L / best_d / GIB, 2),
            "note": "whole call (python wall clock), pinned host -> device -> host, 32 MiB chunks "
                    "over 3 HIP streams, best of 3"}


# ---------------------------------------------------------------- main
def parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--min-warmup-s", type=float, default=0.3,
                    help="keep running untimed warmup steps until this much wall time has passed "
                         "(the GPU clock ramps over ~0.1 s; see DESIGN.md)")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--records", type=int, default=0, help="override records per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config1", action="store_true",
                    help="skip the config-1 (XX loopback + 1000 x 1 KiB) leg of the N=1 line")
    # test hook: initialise the process group (RCCL on GPUs) even at world
    # size 1, so the barrier / reduction / gather path runs on a 1-GPU box
    ap.add_argument("--force-dist", action="store_true", help=argparse.SUPPRESS)
    # control-plane backend (tests / A/B only: gloo is the product choice)
    ap.add_argument("--dist-backend", choices=("gloo", "nccl"), default="gloo",
                    help=argparse.SUPPRESS)
    ap.add_argument("--host-inclusive", action="store_true",
                    help="also time the pinned-host H2D->kernel->D2H pipeline (DESIGN.md)")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    # test hook (tests/test_gpu_multirank.py): after the timed run, every rank
    # compares its WHOLE shard with the CPU oracle (tests/fullcheck.py) at its
    # global nonce base and data offset; off by default, outside the timing
    ap.add_argument("--check-oracle", action="store_true", help=argparse.SUPPRESS)
    # layout study (config 4): byte alignment of each record's offsets
    ap.add_argument("--rec-align", type=int, default=16, help=argparse.SUPPRESS)
    # config 4 with ragged lengths: 64 * 2^k - U(0..63) (zipf_lengths)
    ap.add_argument("--jitter", action="store_true",
                    help="config 4: lower each record length by U(0..63) bytes")
    # test hook: ranks share the visible GPUs (rank r -> device r mod count),
    # so the N-rank path runs end to end on a 1-GPU box (the rate is then
    # not a scaling figure: the ranks split one GPU)
    ap.add_argument("--share-device", action="store_true", help=argparse.SUPPRESS)
    # test hook (--stub only): every rank reports the same device, which the
    # shard check must refuse unless --share-device is given
    ap.add_argument("--stub-same-device", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.config == 1:
        print(json.dumps(dict({"metric": "config 1: XX loopback + 1000 x 1 KiB each way, per record",
                               "config": {"workload": "cfg1"}}, **config1())), flush=True)
        return 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args, argv)

    # the JSON line goes to the original stdout; everything else written to
    # fd 1 from here on (library banners: RCCL, profilers) lands on stderr
    out = json_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("note: WORLD_SIZE=%d, --gpus %d; n_gpus reports the world size" % (world, args.gpus))
    dist = None
    if args.stub:
        import torch
        dev = "cpu"
        if world > 1 or args.force_dist:
            import torch.distributed as dist
            dist.init_process_group("gloo")

        def sync():
            pass
        stream = None
        wl = make_stub_workload(args, rank, world)
    else:
        import torch
        if args.share_device:
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dev = "cuda"
        if world > 1 or args.force_dist:
            import torch.distributed as dist
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
        noise_amd.load()
        stream = torch.cuda.current_stream()
        sync = torch.cuda.synchronize
        wl = make_workload(args.config, args, rank, world, stream)
    cfg = args.config
    R, L, workload, step = wl["R"], wl["L"], wl["workload"], wl["step"]

    log("rank %d/%d: %d records x %d B, nonces [%d, %d), warmup %d" %
        (rank, world, R, L, wl["n_base"], wl["n_base"] + R, args.warmup))
    # correctness of the step about to be timed: all tags verify, round trip
    # exact (checked before the warmup so no host-side idle gap -- during which
    # the GPU clock drops -- separates the warmup from the timed steps)
    step()
    sync()
    if not wl["check"]():
        raise SystemExit("round trip failed on rank %d" % rank)
    evs = None
    if not args.stub:
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    sync()
    while time.perf_counter() - tw < args.min_warmup_s:
        for _ in range(4):
            step()
        sync()

    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i] if evs else None)
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if evs:
        enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
        dec_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    else:
        enc_ms = dec_ms = elapsed * 1e3 / args.steps / 2
    # this rank's own figures: with them the N-GPU line shows each GPU's
    # balance beside the max-over-ranks wall time
    mine = {"rank": rank, "nonce_lo": wl["n_base"], "nonce_hi": wl["n_base"] + R, "records": R,
            "enc_ms": round(enc_ms, 4), "dec_ms": round(dec_ms, 4),
            "step_ms": round(elapsed * 1e3 / args.steps, 4), "device": device_info(args, local)}
    # the timed work was correct too
    if not wl["check"]():
        raise SystemExit("timed round trip failed on rank %d" % rank)
    if args.check_oracle and not args.stub:
        # test infrastructure (tests/fullcheck.py, the oracle): a checker of
        # this rank's whole shard, run after the timed region
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import fullcheck
        import oracle_lib
        res = fullcheck.check_bench_shard(oracle_lib.Oracle(), torch, wl["oracle"])
        log("rank %d: oracle check of the whole shard passed: %s" % (rank, json.dumps(res)))
        mine["oracle_check"] = res
    shards = [mine]
    if dist:
        red_dev = "cuda" if (dev == "cuda" and args.dist_backend == "nccl") else "cpu"
        elapsed, total_rec = reduce_over_ranks(dist, elapsed, R, red_dev)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        shards = gathered
    else:
        total_rec = R
    if cfg == 3:  # sessions: nonces are per session, so only the devices are compared
        bad = check_shards([dict(s, nonce_lo=s["rank"], nonce_hi=s["rank"] + 1) for s in shards],
                           args.share_device)
    else:
        bad = check_shards(shards, args.share_device)
    if bad:
        raise SystemExit("shard table: " + bad)
    log("enc %.3f ms, dec %.3f ms per launch; step %.3f ms" %
        (enc_ms, dec_ms, elapsed * 1e3 / args.steps))

    # plaintext through the AEAD (enc + dec), scaled from this rank's records
    total_bytes = 2.0 * wl["pt_bytes"] * (total_rec / R) * args.steps
    value = total_bytes / elapsed / GIB

    line = {"metric": wl["metric"],
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong" if cfg == 5 else "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic (splitmix64)",
            "config": dict({"workload": workload, "records_per_gpu": R,
                            "bytes_counted": "plaintext bytes through the AEAD, encrypt + decrypt",
                            "parallelism": "records sharded per GPU, no collective"},
                           **wl["config"]),
            "roofline": roofline(cfg, wl, enc_ms, dec_ms),
            "shards": shards, "rank_spread": rank_spread(shards)}
    if args.share_device:
        line["note"] = "--share-device test run: the ranks split the visible GPU(s); not a scaling figure"
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.stub:
        log("cpu baseline ...")
        line["cpu_baseline"] = cpu_baseline(cfg, args.jitter)
    if rank == 0 and world == 1 and cfg == 2 and not args.no_config1 and not args.stub:
        log("config 1 leg ...")
        line["config1"] = config1()
    if rank == 0 and args.host_inclusive and cfg == 2 and not args.stub:
        # 1 KiB (the config-2 shape) and 16 KiB records, the same 1 GiB each
        line["host_inclusive"] = dict(host_inclusive(R, L), record_bytes=L)
        line["host_inclusive_16k"] = dict(host_inclusive(R * L // 16384, 16384), record_bytes=16384)
    if rank == 0:
        out.write(json.dumps(line) + "\n")
        out.flush()
    if dist:
        dist.destroy_process_group()
    return 0


def roofline(cfg, wl, enc_ms, dec_ms):
    """Roofline of the dominant kernel: algorithmic bytes per launch / its
    average duration from the HIP events on its own stream (cfg 4: the whole
    records call).  HBM traffic and VALU instruction counts come from the
    committed rocprofv3 PMC summary of the same workload."""
    if enc_ms >= dec_ms:
        d, kbytes, rbytes, kms = 0, wl["enc_bytes"], wl["read_bytes"][0], enc_ms
    else:
        d, kbytes, rbytes, kms = 1, wl["dec_bytes"], wl["read_bytes"][1], dec_ms
    names = wl["knames"][d]
    achieved = kbytes / (kms * 1e-3)
    prof = latest_profile(cfg)
    pmc = pmc_kernels(prof, names, wl.get("pmc_anchor", (None, None))[d])
    # the profile's per-launch counts, scaled to this launch's records (a
    # strong-scaling shard, or --records, launches fewer than were profiled)
    scale = 1.0
    if pmc and prof[1].get("records_per_launch"):
        scale = wl["R"] / float(prof[1]["records_per_launch"])
    traffic = None
    if pmc and "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        # gfx950: FETCH_SIZE reports half of a wide coalesced read stream
        traffic = int((2.0 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024 * scale)
    roof = {"bound": "hbm", "kernel": names[0] if len(names) == 1 else
            "records call: " + ", ".join(n.replace("noise_amd::", "") + "*" for n in names),
            "direction": "decrypt" if d else "encrypt",
            "achieved": round(achieved / 1e9, 1), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic,
            "hbm_frac_rw": round(achieved / HBM_PEAK, 4),
            "hbm_frac_read": round(rbytes / (kms * 1e-3) / HBM_PEAK, 4),
            "hbm_frac_note": "rw = (bytes read + written) / t / 8 TB/s (north_star target 0.70); read = "
                             "bytes read / t / 8 TB/s (a 1:1 read/write stream cannot exceed ~0.5)",
            "algorithmic_bytes_per_launch": kbytes, "read_bytes_per_launch": rbytes,
            "avg_launch_ms": round(kms, 4), "enc_ms": round(enc_ms, 4), "dec_ms": round(dec_ms, 4),
            "pmc_source": prof[0] if prof else None,
            "binding_roof": "valu"}
    if scale != 1.0:
        roof["pmc_scaled"] = round(scale, 6)
    if pmc and "SQ_INSTS_VALU" in pmc:
        vi = pmc["SQ_INSTS_VALU"] * scale
        valu = {"insts_per_launch": int(vi), "achieved": round(vi / (kms * 1e-3) / 1e9, 2),
                "peak": round(VALU_PEAK / 1e9, 1), "unit": "G wave-instr/s",
                "frac": round(vi / (kms * 1e-3) / VALU_PEAK, 4),
                "issue_model": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction (measured cost "
                               "of every instruction in a ChaCha/Poly1305 stream on gfx950)"}
        # the HBM fraction the VALU work alone allows: the launch cannot be
        # shorter than its instructions at the issue model's rate, so its
        # bytes cannot move faster than bytes / (VALU / peak issue rate)
        cap = kbytes * VALU_PEAK / (vi * HBM_PEAK) if vi else None
        valu["hbm_frac_cap"] = round(cap, 4) if cap else None
        valu["hbm_frac_cap_note"] = ("bytes per launch / (VALU per launch / %.1f G/s) / 8 TB/s: the rw "
                                     "fraction reachable at 100 %% VALU issue" % (VALU_PEAK / 1e9))
        roof["valu_cap_hbm_frac"] = valu["hbm_frac_cap"]
        if "SQ_WAVES" in pmc and pmc["SQ_WAVES"]:
            valu["insts_per_wave"] = int(pmc["SQ_INSTS_VALU"] / pmc["SQ_WAVES"])
        if pmc.get("GRBM_GUI_ACTIVE"):
            # effective clock of the profiled dispatch (GRBM_GUI_ACTIVE sums 8 XCDs)
            busy = pmc["GRBM_GUI_ACTIVE"] / 8.0
            valu["issue_util_profiled"] = round(pmc["SQ_INSTS_VALU"] * 4.0 / 1024.0 / busy, 4)
        roof["valu"] = valu
    return roof


if __name__ == "__main__":
    sys.exit(main())
