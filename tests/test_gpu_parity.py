"""GPU parity: the gfx950 kernels, called through the C ABI, against the CPU
oracle and the golden records from the reference's tests/vectors.
Bit-exact everywhere (integer/byte work)."""
import hashlib
import os
import random
import subprocess

import numpy as np
import pytest

import noise_amd
import oracle_lib

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
SEED = 0x4E4F495345  # splitmix64 seed of BASELINE config 2


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    noise_amd.load()
    torch.cuda.set_device(0)


def dev(b):
    """bytes/np.uint8 -> uint8 CUDA tensor (at least 1 element)."""
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b
    if a.size == 0:
        a = np.zeros(1, dtype=np.uint8)
    return torch.from_numpy(a.copy()).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().tobytes()


def pack_records(recs, decrypt=False, align=16):
    """Lay golden-style records out in buffers + descriptors (records kernel)."""
    keys, desc, inb, adb = [], [], bytearray(), bytearray()
    out_off = 0
    for i, r in enumerate(recs):
        data = r["ct"] if decrypt else r["pt"]
        L = len(r["pt"])
        in_off = len(inb)
        inb += data + bytes(-len(data) % align)
        ad_off = len(adb)
        adb += r["ad"] + bytes(-len(r["ad"]) % align)
        out_len = L if decrypt else L + 16
        desc.append((in_off, out_off, r["nonce"], ad_off, L, len(r["ad"]), i, 0))
        out_off += out_len + (-out_len % align)
        keys.append(r["key"])
    d = np.array(desc, dtype=noise_amd.record_dtype())
    return (b"".join(keys), d, bytes(inb), bytes(adb), out_off)


def run_records(recs, decrypt=False):
    keys, d, inb, adb, out_bytes = pack_records(recs, decrypt)
    d_keys, d_desc = dev(keys), dev(d.view(np.uint8))
    d_in, d_ad = dev(inb), dev(adb)
    d_out = torch.zeros(max(out_bytes, 1), dtype=torch.uint8, device="cuda")
    if decrypt:
        d_st = torch.full((len(recs),), 7, dtype=torch.uint8, device="cuda")
        noise_amd.decrypt_records(d_keys, len(recs), d_desc, len(recs), d_in, d_out, d_st, d_ad)
        st = host(d_st)
    else:
        noise_amd.encrypt_records(d_keys, len(recs), d_desc, len(recs), d_in, d_out, d_ad)
        st = None
    out = host(d_out)
    res = []
    for i, r in enumerate(recs):
        L = len(r["pt"])
        o = int(d[i]["out_off"])
        res.append(out[o:o + (L if decrypt else L + 16)])
    return res, st


@pytest.mark.parametrize("kind", ["transport", "handshake"])
def test_golden_records_kernel(golden, kind):
    recs = golden[kind]
    enc, _ = run_records(recs)
    bad = [r["vector"] for r, c in zip(recs, enc) if c != r["ct"]]
    assert not bad, "%d/%d mismatches, first %s" % (len(bad), len(recs), bad[:3])
    dec, st = run_records(recs, decrypt=True)
    assert set(st) == {0}
    assert all(p == r["pt"] for r, p in zip(recs, dec))


def test_golden_single_record_host_path(golden):
    for r in golden["transport"][::7] + golden["handshake"][::11]:
        assert noise_amd.encrypt_host(r["key"], r["nonce"], r["ad"], r["pt"]) == r["ct"]
        assert noise_amd.decrypt_host(r["key"], r["nonce"], r["ad"], r["ct"]) == r["pt"]


@pytest.mark.parametrize("ad_len", [0, 64, 100, 9000])
def test_single_record_host_lengths(oracle, ad_len):
    """CipherState's per-record path (noise_gpu_encrypt_host / _decrypt_host:
    the latency kernel for AD <= 8 KiB and records <= 65535 B, the staged lane
    walk otherwise) at every record-size regime up to the Noise maximum and
    beyond, vs the oracle; a tampered record fails and is left untouched."""
    rng = random.Random(ad_len + 1)
    key = rng.randbytes(32)
    for length in (0, 1, 15, 16, 17, 64, 65, 1000, 1024, 4095, 16384, 16385, 65472, 65473, 65519,
                   65535, 70000):
        if ad_len == 9000 and length > 20000:
            continue
        n = rng.getrandbits(64) % (2**64 - 2)
        ad, pt = rng.randbytes(ad_len), rng.randbytes(length)
        ct = noise_amd.encrypt_host(key, n, ad, pt)
        assert ct == oracle.encrypt(key, n, ad, pt), (length, ad_len)
        assert noise_amd.decrypt_host(key, n, ad, ct) == pt, (length, ad_len)
        bad = bytearray(ct)
        bad[rng.randrange(len(bad))] ^= 4
        with pytest.raises(noise_amd.NoiseGpuError) as e:
            noise_amd.decrypt_host(key, n, ad, bytes(bad))
        assert e.value.code == noise_amd.E_MAC


def test_kats_and_rekey(oracle):
    for k, n, ad, pt, ct in (oracle_lib.KAT_K1, oracle_lib.KAT_K2, oracle_lib.KAT_K3):
        assert noise_amd.encrypt_host(bytes.fromhex(k), n, bytes.fromhex(ad),
                                      bytes.fromhex(pt)).hex() == ct
    for n, (head, tag, digest) in oracle_lib.KAT_K5.items():
        out = noise_amd.encrypt_host(bytes(range(32)), n, b"", oracle_lib.k5_plaintext())
        assert out[:16].hex() == head and out[1024:].hex() == tag
        assert hashlib.blake2b(out[:1024], digest_size=32).hexdigest() == digest
    assert noise_amd.rekey_host(bytes(32)).hex() == oracle_lib.KAT_K4_REKEY_ZERO
    rng = random.Random(3)
    keys = [rng.randbytes(32) for _ in range(1000)]
    d_keys = dev(b"".join(keys))
    noise_amd.rekey_keys(d_keys, len(keys))
    got = host(d_keys)
    assert all(got[32 * i:32 * i + 32] == oracle.rekey(k) for i, k in enumerate(keys))


LENGTHS = [0, 1, 3, 15, 16, 17, 31, 32, 48, 63, 64, 65, 100, 127, 128, 129, 192, 255, 256, 512,
           1000, 1023, 1024, 1025, 1040, 2048, 4096, 8192, 16384, 65519]

# lengths served by the LDS-staged tile kernel (tile_kernel.hpp)
TILE_LENGTHS = [64, 128, 192, 256, 512, 1024, 2048, 4096, 8192, 16384]


@pytest.mark.parametrize("length", TILE_LENGTHS)
@pytest.mark.parametrize("nrec", [1, 63, 64, 65, 200, 1000])
@pytest.mark.parametrize("in_place", [False, True])
def test_tile_kernel_shapes(oracle, length, nrec, in_place):
    """Partial tiles / super-tiles, in-place and out-of-place, both directions."""
    rng = random.Random(length * 1000 + nrec * 2 + in_place)
    key, n0 = rng.randbytes(32), rng.getrandbits(64)
    in_stride = length + 16 if in_place else length
    out_stride = length + 16 if in_place else length + 32  # padded output rows
    pts = [rng.randbytes(length) for _ in range(nrec)]
    src = bytearray(in_stride * nrec)
    for i, p in enumerate(pts):
        src[i * in_stride:i * in_stride + length] = p
    d_in = dev(bytes(src))
    d_out = d_in if in_place else torch.zeros(out_stride * nrec, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, n0, d_in, in_stride, d_out, out_stride, length, nrec)
    out = host(d_out)
    for i in list(range(min(nrec, 70))) + list(range(max(0, nrec - 70), nrec)):
        want = oracle.encrypt(key, n0 + i, b"", pts[i])
        assert out[i * out_stride:i * out_stride + length + 16] == want, i
    # decrypt (into separate rows, or back in place)
    d_pt = d_out if in_place else torch.zeros(in_stride * nrec, dtype=torch.uint8, device="cuda")
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_uniform(key, n0, d_out, out_stride, d_pt, out_stride if in_place else in_stride,
                              length, d_st, nrec)
    assert set(host(d_st)) == {0}
    back = host(d_pt)
    st = out_stride if in_place else in_stride
    for i in range(nrec):
        assert back[i * st:i * st + length] == pts[i], i


@pytest.mark.parametrize("length", LENGTHS)
@pytest.mark.parametrize("layout", ["packed16", "odd"])
def test_uniform_lengths_vs_oracle(oracle, length, layout):
    rng = random.Random(length * 31 + len(layout))
    nrec = 37 if length <= 16384 else 5
    key = rng.randbytes(32)
    n0 = rng.getrandbits(64)
    if layout == "packed16":
        in_stride = (length + 15) & ~15
        out_stride = (length + 16 + 15) & ~15
    else:  # strides and base offsets that break 16-byte alignment
        in_stride, out_stride = length + 3, length + 16 + 5
    in_off, out_off = (0, 0) if layout == "packed16" else (1, 7)
    pt = np.frombuffer(rng.randbytes(in_stride * nrec + 8), dtype=np.uint8)
    d_in = dev(pt)
    d_out = torch.zeros(out_stride * nrec + 16, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, n0, d_in, in_stride, d_out, out_stride, length, nrec,
                              in_offset=in_off, out_offset=out_off)
    out = host(d_out)
    for i in range(nrec):
        p = pt[in_off + i * in_stride: in_off + i * in_stride + length].tobytes()
        want = oracle.encrypt(key, n0 + i, b"", p)
        assert out[out_off + i * out_stride: out_off + i * out_stride + length + 16] == want, i
    # decrypt back (out-of-place) and compare
    d_pt = torch.zeros(in_stride * nrec + 16, dtype=torch.uint8, device="cuda")
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_uniform(key, n0, d_out, out_stride, d_pt, in_stride, length, d_st, nrec,
                              in_offset=out_off, out_offset=in_off)
    assert set(host(d_st)) == {0}
    back = host(d_pt)
    for i in range(nrec):
        s = in_off + i * in_stride
        assert back[s:s + length] == pt[s:s + length].tobytes()


@pytest.mark.parametrize("ad_mode", ["shared", "per_record"])
def test_uniform_with_ad(oracle, ad_mode):
    rng = random.Random(11)
    nrec, length, ad_len = 50, 200, 64
    key, n0 = rng.randbytes(32), 5
    ad = rng.randbytes(ad_len * (nrec if ad_mode == "per_record" else 1))
    ad_stride = ad_len if ad_mode == "per_record" else 0
    pt = rng.randbytes(length * nrec)
    d_out = torch.zeros((length + 16) * nrec, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, n0, dev(pt), length, d_out, length + 16, length, nrec,
                              d_ad=dev(ad), ad_stride=ad_stride, ad_len=ad_len)
    out = host(d_out)
    for i in range(nrec):
        a = ad[i * ad_stride:i * ad_stride + ad_len]
        assert out[i * (length + 16):(i + 1) * (length + 16)] == \
            oracle.encrypt(key, n0 + i, a, pt[i * length:(i + 1) * length])


@pytest.mark.parametrize("n0", [2**32 - 3, 2**64 - 3, 2**64 - 1, 2**63 - 2])
def test_nonce_edges(oracle, n0):
    """Nonce words 14/15 carry, and (nonce0 + i) wrapping mod 2^64."""
    rng = random.Random(n0 & 0xffff)
    key, nrec, length = rng.randbytes(32), 8, 64
    pt = rng.randbytes(length * nrec)
    d_out = torch.zeros((length + 16) * nrec, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, n0, dev(pt), length, d_out, length + 16, length, nrec)
    out = host(d_out)
    for i in range(nrec):
        assert out[i * 80:(i + 1) * 80] == oracle.encrypt(key, (n0 + i) % 2**64, b"",
                                                           pt[i * 64:(i + 1) * 64])


@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("length", [1024, 77])
def test_decrypt_rejects_tampering(oracle, in_place, length):
    rng = random.Random(length + in_place)
    nrec = 64
    stride = (length + 16 + 15) & ~15
    key, n0 = rng.randbytes(32), rng.getrandbits(40)
    buf = bytearray(stride * nrec)
    for i in range(nrec):
        buf[i * stride:i * stride + length + 16] = oracle.encrypt(key, n0 + i, b"",
                                                                  rng.randbytes(length))
    orig = bytes(buf)
    bad = {3: 0, 17: length + 5, 40: length + 15, 63: length // 2}  # record -> byte flipped
    for i, off in bad.items():
        buf[i * stride + off] ^= 0x01
    tampered = bytes(buf)
    d_in = dev(tampered)
    d_out = d_in if in_place else torch.full((stride * nrec,), 0xAB, dtype=torch.uint8, device="cuda")
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_uniform(key, n0, d_in, stride, d_out, stride, length, d_st, nrec)
    st = host(d_st)
    out = host(d_out)
    for i in range(nrec):
        rec = out[i * stride:i * stride + length]
        if i in bad:
            assert st[i] == noise_amd.REC_BAD_MAC
            # in place: buffer untouched; out of place: no unauthenticated plaintext
            want = tampered[i * stride:i * stride + length] if in_place else bytes(length)
            assert rec == want, i
        else:
            assert st[i] == noise_amd.REC_OK
            assert rec == oracle.decrypt(key, n0 + i, b"", orig[i * stride:i * stride + length + 16])


def test_in_place_encrypt(oracle):
    rng = random.Random(5)
    nrec, length, stride = 100, 512, 528
    key = rng.randbytes(32)
    buf = bytearray(stride * nrec)
    pts = [rng.randbytes(length) for _ in range(nrec)]
    for i, p in enumerate(pts):
        buf[i * stride:i * stride + length] = p
    d = dev(bytes(buf))
    noise_amd.encrypt_uniform(key, 0, d, stride, d, stride, length, nrec)
    out = host(d)
    for i, p in enumerate(pts):
        assert out[i * stride:(i + 1) * stride] == oracle.encrypt(key, i, b"", p)


def test_many_sessions_records(oracle):
    """Config-3 shape at reduced size: 4096 keys x 4 records, interleaved,
    nonce = (s << 32) + j (exercises nonce word 15)."""
    rng = random.Random(9)
    nkeys, per, length = 4096, 4, 1024
    keys = [rng.randbytes(32) for _ in range(nkeys)]
    nrec = nkeys * per
    pt = np.frombuffer(rng.randbytes(nrec * length), dtype=np.uint8)
    desc = np.zeros(nrec, dtype=noise_amd.record_dtype())
    i = np.arange(nrec, dtype=np.uint64)
    desc["in_off"] = i * length
    desc["out_off"] = i * (length + 16)
    s = i % nkeys
    desc["nonce"] = (s << np.uint64(32)) + i // nkeys
    desc["len"] = length
    desc["key_idx"] = s.astype(np.uint32)
    d_out = torch.zeros(nrec * (length + 16), dtype=torch.uint8, device="cuda")
    d_keys = dev(b"".join(keys))
    noise_amd.encrypt_records(d_keys, nkeys, dev(desc.view(np.uint8)), nrec, dev(pt), d_out)
    out = host(d_out)
    for j in rng.sample(range(nrec), 300) + [0, nrec - 1]:
        want = oracle.encrypt(keys[j % nkeys], int(desc["nonce"][j]), b"",
                              pt[j * length:(j + 1) * length].tobytes())
        assert out[j * (length + 16):(j + 1) * (length + 16)] == want, j


def test_fill_synthetic_matches_oracle(oracle):
    for offset, n in [(0, 4096), (16, 1000), (3, 77)]:
        d = torch.zeros(n, dtype=torch.uint8, device="cuda")
        noise_amd.fill_synthetic(d, n, SEED, offset=offset)
        assert host(d) == oracle.synthetic(n, SEED, offset=offset)


def test_config2_full_size_round_trip(oracle):
    """BASELINE config 2 at full size: 2^20 x 1 KiB, one key, nonces 0..R-1.
    Every record of both directions bit-exact against the oracle (chunked
    D2H + oracle_check_uniform), plus the size-independent properties: every
    tag verifies, decrypt(encrypt(x)) == x."""
    import fullcheck
    R, L = 1 << 20, 1024
    key = bytes(range(32))
    d_pt = torch.empty(R * L, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d_pt, R * L, SEED)
    d_ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
    d_back = torch.empty(R * L, dtype=torch.uint8, device="cuda")
    d_st = torch.full((R,), 9, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, 0, d_pt, L, d_ct, L + 16, L, R)
    noise_amd.decrypt_uniform(key, 0, d_ct, L + 16, d_back, L, L, d_st, R)
    torch.cuda.synchronize()
    assert int(d_st.sum().item()) == 0
    assert torch.equal(d_pt, d_back)
    fullcheck.check_uniform(oracle, torch, key, 0, d_pt, L, d_ct, L + 16, L, R)
    fullcheck.check_uniform(oracle, torch, key, 0, d_ct, L + 16, d_back, L, L, R, decrypt=True,
                            d_status=d_st)
    # the device generator is the one the oracle restates
    for i in (0, 12345, R - 1):
        assert d_pt[i * L:(i + 1) * L].cpu().numpy().tobytes() == oracle.synthetic(L, SEED, i * L)


def test_host_pipeline_matches_device(oracle):
    """Transfer-inclusive host API == device kernels (pinned buffers)."""
    rng = random.Random(4)
    R, L = 3000, 1024
    key = rng.randbytes(32)
    pt = torch.from_numpy(np.frombuffer(rng.randbytes(R * L), dtype=np.uint8).copy()).pin_memory()
    ct = torch.zeros(R * (L + 16), dtype=torch.uint8).pin_memory()
    back = torch.zeros(R * L, dtype=torch.uint8).pin_memory()
    st = torch.full((R,), 9, dtype=torch.uint8).pin_memory()
    import ctypes
    lib = noise_amd.load()
    secs = ctypes.c_double()
    assert lib.noise_gpu_encrypt_uniform_host(key, 10, ctypes.c_void_p(pt.data_ptr()), L,
                                              ctypes.c_void_p(ct.data_ptr()), L + 16, L, R,
                                              ctypes.byref(secs)) == 0
    assert lib.noise_gpu_decrypt_uniform_host(key, 10, ctypes.c_void_p(ct.data_ptr()), L + 16,
                                              ctypes.c_void_p(back.data_ptr()), L, L,
                                              ctypes.c_void_p(st.data_ptr()), R,
                                              ctypes.byref(secs)) == 0
    assert torch.equal(pt, back) and int(st.sum()) == 0
    c = ct.numpy().tobytes()
    for i in (0, 1, 1234, R - 1):
        assert c[i * (L + 16):(i + 1) * (L + 16)] == oracle.encrypt(
            key, 10 + i, b"", pt[i * L:(i + 1) * L].numpy().tobytes())


def test_device_context_api(oracle, golden):
    """noise_gpu_ctx_*: an explicit device context gives the context-free
    entry points' results (single records, rekey, descriptor and uniform host
    batches), keeps the caller's current device, and refuses bad indices."""
    import ctypes
    lib = noise_amd.load()
    h = ctypes.c_void_p()
    assert lib.noise_gpu_ctx_create(torch.cuda.device_count(), ctypes.byref(h)) == noise_amd.E_ARG
    assert lib.noise_gpu_ctx_create(0, ctypes.byref(h)) == 0 and h.value
    try:
        d = ctypes.c_int(-1)
        assert lib.noise_gpu_ctx_device(h, ctypes.byref(d)) == 0 and d.value == 0
        rng = random.Random(21)
        key = rng.randbytes(32)
        for L, A in ((0, 0), (33, 64), (1024, 0), (20000, 9000), (70000, 0)):
            pt, ad = rng.randbytes(L), rng.randbytes(A)
            buf = ctypes.create_string_buffer(pt, L + 16)
            assert lib.noise_gpu_ctx_encrypt_host(h, key, 5, ad or None, A, buf, L) == 0
            assert buf.raw == oracle.encrypt(key, 5, ad, pt)
            assert lib.noise_gpu_ctx_decrypt_host(h, key, 5, ad or None, A, buf, L + 16) == 0
            assert buf.raw[:L] == pt
        kb = ctypes.create_string_buffer(bytes(32), 32)
        assert lib.noise_gpu_ctx_rekey_host(h, kb) == 0
        assert kb.raw.hex() == oracle_lib.KAT_K4_REKEY_ZERO
        recs = golden["transport"][:300]
        keys, dsc, inb, adb, out_bytes = pack_records(recs)
        out = ctypes.create_string_buffer(out_bytes)
        dbuf = dsc.view(np.uint8).tobytes()
        assert lib.noise_gpu_ctx_encrypt_records_host(h, keys, len(recs), dbuf, len(recs), inb,
                                                      len(inb), out, out_bytes, adb or None,
                                                      len(adb)) == 0
        for i, r in enumerate(recs):
            o = int(dsc[i]["out_off"])
            assert out.raw[o:o + len(r["pt"]) + 16] == r["ct"]
        R, L = 500, 1024
        pt = rng.randbytes(R * L)
        ct = ctypes.create_string_buffer(R * (L + 16))
        back = ctypes.create_string_buffer(R * L)
        st = ctypes.create_string_buffer(b"\x09" * R, R)
        secs = ctypes.c_double()
        assert lib.noise_gpu_ctx_encrypt_uniform_host(h, key, 9, pt, L, ct, L + 16, L, R,
                                                      ctypes.byref(secs)) == 0
        assert lib.noise_gpu_ctx_decrypt_uniform_host(h, key, 9, ct, L + 16, back, L, L, st, R,
                                                      ctypes.byref(secs)) == 0
        assert back.raw == pt and st.raw == bytes(R)
        assert ct.raw[(R - 1) * (L + 16):] == oracle.encrypt(key, 9 + R - 1, b"", pt[(R - 1) * L:])
        assert torch.cuda.current_device() == 0
    finally:
        assert lib.noise_gpu_ctx_destroy(h) == 0


def test_resident_latency_path(oracle, golden):
    """noise_gpu_set_resident: single records served by a resident workgroup
    polling a doorbell (single_kernels.hip k_aead_resident) -- golden records,
    every size regime with and without AD, tampering (E_MAC, buffer left as
    it was), the idle exit and relaunch, the explicit stop, and the launch
    path afterwards.  Bit-exact vs the oracle / golden fixtures."""
    import time
    noise_amd.set_resident(True, 50000)
    try:
        for r in golden["transport"][::9] + golden["handshake"][::13]:
            assert noise_amd.encrypt_host(r["key"], r["nonce"], r["ad"], r["pt"]) == r["ct"]
            assert noise_amd.decrypt_host(r["key"], r["nonce"], r["ad"], r["ct"]) == r["pt"]
        rng = random.Random(31)
        key = rng.randbytes(32)
        for length in (0, 1, 16, 17, 1024, 4096, 16384, 65519, 65535, 70000):
            for ad_len in (0, 64, 9000):
                if ad_len == 9000 and length > 20000:
                    continue
                n = rng.getrandbits(64) % (2**64 - 2)
                ad, pt = rng.randbytes(ad_len), rng.randbytes(length)
                ct = noise_amd.encrypt_host(key, n, ad, pt)
                assert ct == oracle.encrypt(key, n, ad, pt), (length, ad_len)
                assert noise_amd.decrypt_host(key, n, ad, ct) == pt
                bad = bytearray(ct)
                bad[rng.randrange(len(bad))] ^= 8
                with pytest.raises(noise_amd.NoiseGpuError) as e:
                    noise_amd.decrypt_host(key, n, ad, bytes(bad))
                assert e.value.code == noise_amd.E_MAC
        # a short idle time: the workgroup leaves between calls and the next
        # request relaunches it
        noise_amd.set_resident(True, 1000)
        for i in range(5):
            pt = rng.randbytes(1000)
            assert noise_amd.encrypt_host(key, i, b"", pt) == oracle.encrypt(key, i, b"", pt)
            time.sleep(0.01)
    finally:
        noise_amd.set_resident(False)
    pt = rng.randbytes(333)
    assert noise_amd.encrypt_host(key, 7, b"", pt) == oracle.encrypt(key, 7, b"", pt)
    # a context in resident mode, destroyed while its workgroup runs
    import ctypes
    lib = noise_amd.load()
    h = ctypes.c_void_p()
    assert lib.noise_gpu_ctx_create(0, ctypes.byref(h)) == 0
    assert lib.noise_gpu_ctx_set_resident(h, 1, 0) == 0
    buf = ctypes.create_string_buffer(pt, len(pt) + 16)
    assert lib.noise_gpu_ctx_encrypt_host(h, key, 9, None, 0, buf, len(pt)) == 0
    assert buf.raw == oracle.encrypt(key, 9, b"", pt)
    assert lib.noise_gpu_ctx_destroy(h) == 0
    torch.cuda.synchronize()  # nothing left running on the device


@pytest.mark.parametrize("req", ["fine", "host"])
def test_resident_speculated_runs(oracle, req, monkeypatch):
    """Resident mode speculates on (key, n + 1) after serving (key, n):
    consecutive nonces under two interleaved keys (a session's send and
    receive states) take the precomputed keystream + r-power path
    (single_kernels.hip one_body_fast) from the second record of a run on.
    Every size around its limits (63 keystream blocks, 256 Poly1305 blocks)
    and past them, AD, tampering on the speculated path, a wrong nonce --
    bit-exact vs the oracle, for each place the request image can live
    (NOISE_GPU_RESIDENT_REQ)."""
    monkeypatch.setenv("NOISE_GPU_RESIDENT_REQ", req)
    noise_amd.set_resident(False)  # a fresh request image, of this kind
    noise_amd.set_resident(True, 2000000)
    try:
        rng = random.Random(77)
        keys = [rng.randbytes(32), rng.randbytes(32)]
        for length in (0, 1, 16, 17, 1000, 1024, 3952, 4032, 4033, 4096, 16384, 65535):
            for ad_len in (0, 64):
                base = [rng.getrandbits(63), rng.getrandbits(63)]
                for i in range(4):
                    for w in (0, 1):
                        n = base[w] + i
                        ad, pt = rng.randbytes(ad_len), rng.randbytes(length)
                        ct = noise_amd.encrypt_host(keys[w], n, ad, pt)
                        assert ct == oracle.encrypt(keys[w], n, ad, pt), (length, ad_len, i, w)
                # decrypt run under key 0: n misses, n + 1 .. hit; one tampered
                for i in range(4):
                    n = base[0] + 100 + i
                    ad, pt = rng.randbytes(ad_len), rng.randbytes(length)
                    ct = oracle.encrypt(keys[0], n, ad, pt)
                    if i == 2:
                        bad = bytearray(ct)
                        bad[rng.randrange(len(bad))] ^= 4
                        with pytest.raises(noise_amd.NoiseGpuError) as e:
                            noise_amd.decrypt_host(keys[0], n, ad, bytes(bad))
                        assert e.value.code == noise_amd.E_MAC
                    else:
                        assert noise_amd.decrypt_host(keys[0], n, ad, ct) == pt
                # the speculated slot holds n + 1 of key 0: a record of another nonce
                with pytest.raises(noise_amd.NoiseGpuError):
                    noise_amd.decrypt_host(keys[0], base[0] + 104, ad, oracle.encrypt(keys[0], 7, ad, pt))
    finally:
        noise_amd.set_resident(False)


def test_cipherstate_cpp_surface():
    """The drop-in noise::CipherState (C++20) on the golden records."""
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "cipherstate_test")
    r = subprocess.run([exe, os.path.join(noise_amd.ROOT, "tests", "golden")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "PASSED" in r.stdout


def test_handshake_vectors():
    """Host HandshakeState (host/handshake.cpp) over the reference's 110
    Noise_*_25519_ChaChaPoly_BLAKE2b vectors (tests/golden/handshake_vectors.tsv,
    extracted from /root/reference/tests/vectors): every handshake message
    byte-exact, the handshake hash, and the transport records through the
    GPU-backed CipherState pair that split() returns."""
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "handshake_test")
    r = subprocess.run([exe, "vectors", os.path.join(noise_amd.ROOT, "tests", "golden",
                                                     "handshake_vectors.tsv")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "vectors 110, failed 0" in r.stdout, r.stdout


def test_xx_loopback_config1_shape():
    """BASELINE config 1 shape: XX loopback handshake with fresh keys, then
    1000 x 1 KiB transport records each way (examples/Noise_XX_*.cpp:26-71)."""
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "handshake_test")
    r = subprocess.run([exe, "loopback", "1000", "1024"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert '"ok": true' in r.stdout


def test_config1_bench_resident():
    """BASELINE config 1 through the drop-in classes with the resident latency
    workgroup (tools/config1_bench.cpp resident): XX handshake + 1000 x 1 KiB
    records each way, round trip exact, then the explicit stop and a
    launch-path record after it."""
    import json
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "config1_bench")
    r = subprocess.run([exe, "1000", "1024", "resident"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["ok"] and line["mode"] == "resident" and line["stopped"]
    print("config1 resident:", json.dumps(line["per_record"]), json.dumps(line["latency_by_size"]))


@pytest.mark.parametrize("sessions,messages,seed", [(100, 1000, 1), (300, 5000, 2)])
def test_transport_batcher(sessions, messages, seed):
    """noise::transport (host/transport.cpp): many sessions' messages in one
    descriptor batch each way (below and above the 2048-record classifier
    threshold), ciphertexts vs the CPU oracle, BE16 framing through a chunked
    Deframer, tampered records rejected, per-session nonce accounting."""
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "transport_test")
    r = subprocess.run([exe, str(sessions), str(messages), str(seed)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ok (0 failures)" in r.stdout


@pytest.mark.parametrize("sessions,messages,seed", [(50, 1500, 3), (400, 6000, 4)])
def test_transport_pipeline(sessions, messages, seed):
    """noise::transport::Pipeline (pinned ring slots, asynchronous flushes):
    tiny slots force many flushes in flight and full-slot retries; ciphertexts
    vs the CPU oracle and vs the Batcher, decrypt round trip with tampered
    records, per-session nonce accounting, stale tickets refused."""
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "transport_test")
    r = subprocess.run([exe, "pipeline", str(sessions), str(messages), str(seed)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ok (0 failures)" in r.stdout


@pytest.mark.parametrize("sessions,messages,seed,big", [(60, 2500, 5, False), (700, 40000, 6, True),
                                                       (3, 30000, 7, True), (40, 30000, 8, "T96")])
def test_transport_pipeline_batched_copies(sessions, messages, seed, big):
    """Pipeline::submit_batch / copy_out with 4 copy threads: ragged batches
    crossing slot boundaries, ciphertexts vs the oracle, nonce accounting,
    decrypt round trip with tampered records rejected.  big: slots of 8192
    records / 2 MiB and batches of up to 20000 messages (the parallel
    bookkeeping: per-chunk session counts, the nonce scan, slots cut by the
    record and the byte capacity; 3 sessions: long runs per session)."""
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "transport_test")
    extra = ["8192", str(2 << 20), "600", "20000"] if big else []
    if big == "T96":  # 96 copy threads, byte cut below the thread count
        extra = ["8192", str(256 << 10), "6000", "20000", "96"]
    r = subprocess.run([exe, "pipeline_batch", str(sessions), str(messages), str(seed)] + extra,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ok (0 failures)" in r.stdout


def test_transport_pipeline_key_upload_order():
    """Pipeline key table: slot A uploads 2^18 new sessions'
    key rows (8 MiB) on its stream; slot B, flushed immediately on another
    stream with no upload of its own, encrypts messages of the last sessions.
    B's stream must wait for A's upload: ciphertexts equal the oracle's."""
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "transport_test")
    r = subprocess.run([exe, "keyrace", str(1 << 18)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ok (0 failures)" in r.stdout


def test_transport_pipeline_beside_resident_traffic():
    """one thread sends resident single-record traffic
    back to back (noise_gpu_set_resident) while another builds a Pipeline,
    grows its key table three times (1024 -> 8192 rows) and pushes growing
    batches (a slot stream's records scratch grows).  Key tables, scratch and
    staging are freed stream-ordered (noise_amd/dev_mem.hpp), so the Pipeline
    work never waits for the resident instance: it must finish while the
    resident thread is still sending (which it does for up to 60 s).  Both
    threads' records are checked against the oracle."""
    import json
    exe = os.path.join(noise_amd.ROOT, "noise-cpp_amd", "bin", "transport_test")
    r = subprocess.run([exe, "resident_race", "5000", "60"], capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["resident_race"] == "ok" and line["pipeline_s"] < 30, line
    assert line["resident_records_meanwhile"] > 1000, line
    print("resident race:", json.dumps(line))


def _sessions_case(rng, nkeys, per, length):
    keys = [rng.randbytes(32) for _ in range(nkeys)]
    nrec = nkeys * per
    i = np.arange(nrec, dtype=np.uint64)
    s = (i % nkeys).astype(np.uint32)
    nonces = (s.astype(np.uint64) << np.uint64(32)) + i // nkeys
    pt = np.frombuffer(rng.randbytes(nrec * length), dtype=np.uint8)
    return keys, s, nonces, pt, nrec


@pytest.mark.parametrize("length", [64, 256, 1024, 4096])
@pytest.mark.parametrize("packed", [True, False])
def test_sessions_tile_kernel(oracle, length, packed):
    """Config-3 shape (interleaved sessions, nonce = (s << 32) + round) through
    the KEYED tile kernel: bit-exact vs oracle, decrypt round trip, tamper."""
    rng = random.Random(length + packed)
    nkeys, per = 512, 5
    keys, s, nonces, pt, nrec = _sessions_case(rng, nkeys, per, length)
    in_stride = length if packed else length + 32
    out_stride = length + 16 if packed else length + 48
    src = np.zeros(nrec * in_stride, dtype=np.uint8)
    for r in range(nrec):
        src[r * in_stride:r * in_stride + length] = pt[r * length:(r + 1) * length]
    d_keys, d_idx, d_non = dev(b"".join(keys)), dev(s.view(np.uint8)), dev(nonces.view(np.uint8))
    d_out = torch.zeros(nrec * out_stride, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_sessions(d_keys, nkeys, d_idx, d_non, dev(src), in_stride, d_out, out_stride,
                               length, nrec)
    out = host(d_out)
    for r in rng.sample(range(nrec), 200) + [0, nrec - 1]:
        want = oracle.encrypt(keys[s[r]], int(nonces[r]), b"", pt[r * length:(r + 1) * length].tobytes())
        assert out[r * out_stride:r * out_stride + length + 16] == want, r
    # tamper two records, decrypt all
    ct = bytearray(out)
    ct[7 * out_stride + 3] ^= 1
    ct[100 * out_stride + length] ^= 0x40  # tag byte
    d_back = torch.full((nrec * in_stride,), 0xCD, dtype=torch.uint8, device="cuda")
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_sessions(d_keys, nkeys, d_idx, d_non, dev(bytes(ct)), out_stride, d_back, in_stride,
                               length, d_st, nrec)
    st = host(d_st)
    back = host(d_back)
    assert st[7] == noise_amd.REC_BAD_MAC and st[100] == noise_amd.REC_BAD_MAC
    assert sum(st) == 2
    assert back[7 * in_stride:7 * in_stride + length] == bytes(length)  # zeroed copy
    for r in range(0, nrec, 37):
        if r in (7, 100):
            continue
        assert back[r * in_stride:r * in_stride + length] == pt[r * length:(r + 1) * length].tobytes()


def test_sessions_bad_key_index(oracle):
    rng = random.Random(77)
    nkeys, per, length = 64, 2, 1024
    keys, s, nonces, pt, nrec = _sessions_case(rng, nkeys, per, length)
    s = s.copy()
    s[5] = nkeys + 3  # out of the table
    d_out = torch.full((nrec * (length + 16),), 0xEE, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_sessions(dev(b"".join(keys)), nkeys, dev(s.view(np.uint8)),
                               dev(nonces.view(np.uint8)), dev(pt), length, d_out, length + 16,
                               length, nrec)
    out = host(d_out)
    assert out[5 * 1040:6 * 1040] == b"\xee" * 1040  # not written
    assert out[6 * 1040:7 * 1040] == oracle.encrypt(keys[s[6]], int(nonces[6]), b"",
                                                     pt[6 * 1024:7 * 1024].tobytes())
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    d_back = torch.zeros(nrec * length, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_sessions(dev(b"".join(keys)), nkeys, dev(s.view(np.uint8)),
                               dev(nonces.view(np.uint8)), d_out, length + 16, d_back, length,
                               length, d_st, nrec)
    st = host(d_st)
    assert st[5] == noise_amd.REC_BAD_KEY and sum(st) == noise_amd.REC_BAD_KEY


def test_sessions_zero_key_row_refused(oracle):
    """An all-zero key row (Noise HasKey() false; what noise_gpu_hs_split
    leaves for a failed handshake) is never used to encrypt: the sessions
    kernel skips the record (nothing written) and decrypt reports BAD_KEY."""
    rng = random.Random(78)
    nkeys, per, length = 64, 2, 1024
    keys, s, nonces, pt, nrec = _sessions_case(rng, nkeys, per, length)
    keys = list(keys)
    keys[int(s[9])] = bytes(32)
    zero_recs = [r for r in range(nrec) if s[r] == s[9]]
    d_keys = dev(b"".join(keys))
    d_out = torch.full((nrec * (length + 16),), 0xEE, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_sessions(d_keys, nkeys, dev(s.view(np.uint8)), dev(nonces.view(np.uint8)), dev(pt),
                               length, d_out, length + 16, length, nrec)
    out = host(d_out)
    for r in range(nrec):
        blk = out[r * 1040:(r + 1) * 1040]
        if r in zero_recs:
            assert blk == b"\xee" * 1040, r
        else:
            assert blk == oracle.encrypt(keys[s[r]], int(nonces[r]), b"", pt[r * 1024:(r + 1) * 1024].tobytes())
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    d_back = torch.zeros(nrec * length, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_sessions(d_keys, nkeys, dev(s.view(np.uint8)), dev(nonces.view(np.uint8)), d_out,
                               length + 16, d_back, length, length, d_st, nrec)
    st = host(d_st)
    for r in range(nrec):
        assert st[r] == (noise_amd.REC_BAD_KEY if r in zero_recs else noise_amd.REC_OK), r
