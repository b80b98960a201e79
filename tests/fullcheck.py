"""Whole-batch bit-exact parity for the full-size GPU tests (test
infrastructure): device buffers are copied to pinned host memory in chunks
and every record is recomputed by the CPU oracle (oracle_check_uniform /
oracle_check_records, multi-threaded) and compared byte for byte.

Used by test_gpu_parity.py (config 2) and test_gpu_full_size.py (configs 3,
4, 5).  Reference path: crypto_aead_write / _read, monocypher.c:2899-2929,
with the Noise nonce framing of noise.cpp:207-215."""
import time

import numpy as np

CHUNK = 1 << 30  # bytes per side per chunk


def _sync(torch):
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class _Pinned:
    def __init__(self, torch, nbytes):
        self.t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        self.a = self.t.numpy()

    def fill(self, dev, lo, hi):
        n = hi - lo
        self.t[:n].copy_(dev[lo:hi])
        return self.a[:n]


def check_uniform(oracle, torch, key, n0, d_in, in_stride, d_out, out_stride, length, nrec,
                  decrypt=False, d_status=None, chunk=CHUNK):
    """Every record of a uniform batch vs the oracle.  Returns a dict of
    figures (records, bytes, seconds) and asserts zero mismatches."""
    per = max(1, chunk // max(in_stride, out_stride))
    _sync(torch)
    t0 = time.time()
    hin = _Pinned(torch, min(nrec, per) * in_stride)
    hout = _Pinned(torch, min(nrec, per) * out_stride)
    st = d_status.cpu().numpy() if d_status is not None else None
    bad = 0
    first = -1
    for r0 in range(0, nrec, per):
        r1 = min(nrec, r0 + per)
        n = r1 - r0
        a = hin.fill(d_in, r0 * in_stride, r0 * in_stride + (n - 1) * in_stride +
                     (length + 16 if decrypt else length))
        b = hout.fill(d_out, r0 * out_stride, r0 * out_stride + (n - 1) * out_stride +
                      (length if decrypt else length + 16))
        _sync(torch)
        nb, f = oracle.check_uniform(1 if decrypt else 0, key, n0 + r0, a, in_stride, b,
                                     out_stride, length, n,
                                     status=None if st is None else st[r0:r1])
        bad += nb
        if f >= 0 and first < 0:
            first = r0 + f
    assert bad == 0, "%d of %d records differ from the oracle, first %d" % (bad, nrec, first)
    return {"records": nrec, "mismatches": 0, "seconds": round(time.time() - t0, 2)}


def check_synthetic(oracle, torch, d_buf, nbytes, seed, offset, chunk=CHUNK // 4):
    """The device buffer holds bytes [offset, offset + nbytes) of the
    splitmix64 stream `seed` (bench.py's per-rank data offset)."""
    _sync(torch)
    h = _Pinned(torch, min(nbytes, chunk))
    for lo in range(0, nbytes, chunk):
        hi = min(nbytes, lo + chunk)
        a = h.fill(d_buf, lo, hi)
        _sync(torch)
        want = np.frombuffer(oracle.synthetic(hi - lo, seed, offset=offset + lo), dtype=np.uint8)
        if not np.array_equal(a, want):
            bad = int(np.flatnonzero(a != want)[0])
            raise AssertionError("synthetic data differs at byte %d (stream offset %d)"
                                 % (lo + bad, offset + lo + bad))
    return {"bytes": nbytes}


def check_bench_shard(oracle, torch, shard):
    """bench.py --check-oracle: one rank's whole shard after the timed run.
    `shard` (bench.make_workload's "oracle" entry) names the rank's buffers,
    its global nonce base and data offset.  Every record is recomputed by the
    oracle in both directions at the rank's GLOBAL nonces (noise.cpp:207-215,
    monocypher.c:2891-2929), and the plaintext is checked against the
    synthetic stream at the rank's global data offset -- an error in either
    that is the same in both directions round-trips and self-authenticates,
    so only this check sees it."""
    kind = shard["kind"]
    out = {"kind": kind, "nonce_base": int(shard["n_base"])}
    if kind == "uniform":
        R, L, n0 = shard["R"], shard["L"], shard["n_base"]
        out["synthetic"] = check_synthetic(oracle, torch, shard["pt"], R * L, shard["seed"],
                                           shard["data_offset"])
        out["encrypt"] = check_uniform(oracle, torch, shard["key"], n0, shard["pt"], L, shard["ct"],
                                       L + 16, L, R)
        out["decrypt"] = check_uniform(oracle, torch, shard["key"], n0, shard["ct"], L + 16,
                                       shard["back"], L, L, R, decrypt=True,
                                       d_status=shard["status"])
    else:  # descriptor batches (sessions, records)
        keys = shard["keys"].cpu().numpy() if hasattr(shard["keys"], "cpu") else shard["keys"]
        keys = np.ascontiguousarray(keys)
        if shard.get("seed") is not None:
            out["synthetic"] = check_synthetic(oracle, torch, shard["pt"], shard["pt_bytes"],
                                               shard["seed"], shard["data_offset"])
        enc, dec = shard["descs"]()
        out["encrypt"] = check_records(oracle, torch, keys, enc, shard["pt"], shard["ct"])
        out["decrypt"] = check_records(oracle, torch, keys, dec, shard["ct"], shard["back"],
                                       decrypt=True, d_status=shard["status"])
    return out


def check_records(oracle, torch, keys, desc, d_in, d_out, decrypt=False, d_status=None,
                  chunk=CHUNK):
    """Every descriptor of a batch whose in_off / out_off both increase with
    the record index (the bench layouts) vs the oracle, in record windows of
    about `chunk` bytes per side."""
    _sync(torch)
    t0 = time.time()
    nrec = len(desc)
    ilen = desc["len"].astype(np.uint64) + (np.uint64(16) if decrypt else np.uint64(0))
    olen = desc["len"].astype(np.uint64) + (np.uint64(0) if decrypt else np.uint64(16))
    iend = desc["in_off"] + ilen
    oend = desc["out_off"] + olen
    assert np.all(np.diff(desc["in_off"].astype(np.int64)) > 0)
    assert np.all(np.diff(desc["out_off"].astype(np.int64)) > 0)
    st = d_status.cpu().numpy() if d_status is not None else None
    kt = np.ascontiguousarray(keys)
    hin = hout = None
    bad, first, r0 = 0, -1, 0
    while r0 < nrec:
        # the largest window starting at r0 with both sides <= chunk bytes
        lo_i, lo_o = int(desc["in_off"][r0]), int(desc["out_off"][r0])
        r1 = int(min(np.searchsorted(iend, lo_i + chunk, side="right"),
                     np.searchsorted(oend, lo_o + chunk, side="right")))
        r1 = max(r1, r0 + 1)
        hi_i, hi_o = int(iend[r0:r1].max()), int(oend[r0:r1].max())
        if hin is None or hin.t.numel() < hi_i - lo_i:
            hin = _Pinned(torch, max(hi_i - lo_i, min(chunk, int(iend.max()))))
        if hout is None or hout.t.numel() < hi_o - lo_o:
            hout = _Pinned(torch, max(hi_o - lo_o, min(chunk, int(oend.max()))))
        a = hin.fill(d_in, lo_i, hi_i)
        b = hout.fill(d_out, lo_o, hi_o)
        _sync(torch)
        sub = np.ascontiguousarray(desc[r0:r1])
        nb, f = oracle.check_records(1 if decrypt else 0, kt, len(kt) // 32, sub, a, b,
                                     status=None if st is None else np.ascontiguousarray(st[r0:r1]),
                                     in_base=lo_i, out_base=lo_o)
        bad += nb
        if f >= 0 and first < 0:
            first = r0 + f
        r0 = r1
    assert bad == 0, "%d of %d records differ from the oracle, first %d" % (bad, nrec, first)
    return {"records": nrec, "mismatches": 0, "seconds": round(time.time() - t0, 2)}
