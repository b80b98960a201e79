"""GPU parity for descriptor batches big enough to take the classified path
(records_kernels.hip): tile classes (64..512 B), long records cut into 1 KiB
segments + tails (1024..65535 B, any length: tails of 1..1023 bytes, 64-block
tails, the 65519 Noise maximum) and the generic lane-per-record class (AD,
odd lengths, unaligned offsets, bad key index, > 65535 B), all in ONE batch,
against the CPU oracle.  Bit-exact."""
import random

import numpy as np
import pytest

import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TILE = [64, 128, 192, 256, 512, 1024, 2048, 4096, 8192, 16384]
WAVE = [16385, 16400, 20000, 32768, 40001, 65519, 65520, 49152 + 7, 1025, 2047, 3071, 65535,
        70000, 1024 * 9 + 1009]
GENERIC = [0, 1, 15, 17, 100, 1000, 3000, 5000, 16383]


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    noise_amd.load()
    torch.cuda.set_device(0)


def dev(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8).copy()
    if a.size == 0:
        a = np.zeros(1, dtype=np.uint8)
    return torch.from_numpy(a).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().tobytes()


def make_batch(rng, n_small=2200, n_big=48, nkeys=37):
    """Records: (len, ad, key_idx, nonce, misalign_in, misalign_out)."""
    recs = []
    for _ in range(n_small):
        u = rng.random()
        if u < 0.55:
            L = rng.choice(TILE[:8])
        elif u < 0.85:
            L = rng.choice(GENERIC)
        else:
            L = rng.choice(TILE[8:] + [3000, 5000])
        ad = rng.randbytes(64) if rng.random() < 0.05 else b""
        mis_in = rng.choice([0] * 9 + [1, 3, 8])
        mis_out = rng.choice([0] * 9 + [4, 5])
        recs.append([L, ad, rng.randrange(nkeys), rng.getrandbits(64) % (2**64 - 2), mis_in, mis_out])
    for i in range(n_big):
        L = WAVE[i % len(WAVE)]
        recs.append([L, b"", rng.randrange(nkeys), rng.getrandbits(64) % (2**64 - 2), 0, 0])
    rng.shuffle(recs)
    keys = [rng.randbytes(32) for _ in range(nkeys)]
    return keys, recs


def layout(recs, decrypt, in_place=False):
    """Offsets: 16-byte aligned slots (+ the record's misalignment)."""
    desc = np.zeros(len(recs), dtype=noise_amd.record_dtype())
    in_off = out_off = ad_off = 0
    for i, (L, ad, ki, n, mi, mo) in enumerate(recs):
        lin = L + 16 if decrypt else L
        lout = L if decrypt else L + 16
        if in_place:
            mi = mo = 0
            slot = L + 16
            desc[i] = (in_off, in_off, n, ad_off, L, len(ad), ki, 0)
            in_off += slot + (-slot % 16)
        else:
            desc[i] = (in_off + mi, out_off + mo, n, ad_off, L, len(ad), ki, 0)
            in_off += lin + mi + 32 + (-(lin + mi) % 16)
            out_off += lout + mo + 32 + (-(lout + mo) % 16)
        ad_off += len(ad) + (-len(ad) % 16)
    return desc, max(in_off, 1), max(out_off, 1), max(ad_off, 1)


def fill(buf, desc, datas, field):
    for i, b in enumerate(datas):
        o = int(desc[i][field])
        buf[o:o + len(b)] = b


def test_mixed_batch_encrypt_decrypt_tamper(oracle):
    rng = random.Random(2024)
    keys, recs = make_batch(rng)
    pts = [rng.randbytes(r[0]) for r in recs]
    desc, in_bytes, out_bytes, ad_bytes = layout(recs, decrypt=False)
    inb = bytearray(in_bytes)
    fill(inb, desc, pts, "in_off")
    adb = bytearray(ad_bytes)
    fill(adb, desc, [r[1] for r in recs], "ad_off")
    d_keys, d_desc, d_ad = dev(b"".join(keys)), dev(desc.view(np.uint8)), dev(adb)
    d_out = torch.full((out_bytes,), 0xA5, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_records(d_keys, len(keys), d_desc, len(recs), dev(inb), d_out, d_ad)
    out = host(d_out)
    cts = []
    for i, (L, ad, ki, n, _, _) in enumerate(recs):
        o = int(desc[i]["out_off"])
        got = out[o:o + L + 16]
        want = oracle.encrypt(keys[ki], n, ad, pts[i])
        assert got == want, (i, L, len(ad), int(desc[i]["in_off"]) % 16, o % 16)
        assert out[o + L + 16:o + L + 32] == b"\xa5" * 16, ("wrote past the record", i, L)
        cts.append(bytearray(want))

    # tamper: a tile record, wave records (partial last piece and not),
    # generic records; one ct byte or one tag byte each
    by_len = {}
    for i, r in enumerate(recs):
        by_len.setdefault(r[0], []).append(i)
    bad = set()
    for L in (1024, 64, 16384, 65519, 32768, 40001, 17, 3000):
        if L in by_len:
            i = by_len[L][0]
            pos = rng.randrange(L + 16)
            cts[i][pos] ^= 1 << rng.randrange(8)
            bad.add(i)
    ddesc, din, dout, _ = layout(recs, decrypt=True)
    cin = bytearray(din)
    fill(cin, ddesc, cts, "in_off")
    d_back = torch.full((dout,), 0x3C, dtype=torch.uint8, device="cuda")
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, len(keys), dev(ddesc.view(np.uint8)), len(recs), dev(cin),
                              d_back, d_st, d_ad)
    st = host(d_st)
    back = host(d_back)
    for i, (L, ad, ki, n, _, _) in enumerate(recs):
        o = int(ddesc[i]["out_off"])
        if i in bad:
            assert st[i] == noise_amd.REC_BAD_MAC, (i, L)
            assert back[o:o + L] == bytes(L), ("failed copy must be zeroed", i, L)
        else:
            assert st[i] == noise_amd.REC_OK, (i, L, st[i])
            assert back[o:o + L] == pts[i], (i, L)
        assert back[o + L:o + L + 16] == b"\x3c" * 16, ("wrote past the record", i, L)


def test_mixed_batch_in_place(oracle):
    rng = random.Random(77)
    keys, recs = make_batch(rng, n_small=2100, n_big=24)
    pts = [rng.randbytes(r[0]) for r in recs]
    desc, nbytes, _, ad_bytes = layout(recs, decrypt=False, in_place=True)
    buf = bytearray(nbytes)
    fill(buf, desc, pts, "in_off")
    adb = bytearray(ad_bytes)
    fill(adb, desc, [r[1] for r in recs], "ad_off")
    d_keys, d_desc, d_ad = dev(b"".join(keys)), dev(desc.view(np.uint8)), dev(adb)
    d_buf = dev(buf)
    noise_amd.encrypt_records(d_keys, len(keys), d_desc, len(recs), d_buf, d_buf, d_ad)
    out = bytearray(host(d_buf))
    for i, (L, ad, ki, n, _, _) in enumerate(recs):
        o = int(desc[i]["in_off"])
        assert bytes(out[o:o + L + 16]) == oracle.encrypt(keys[ki], n, ad, pts[i]), (i, L)
    # tamper some, decrypt in place: failures keep their ciphertext
    bad = [i for i, r in enumerate(recs) if r[0] in (65519, 20000, 2048, 100)][:6]
    for i in bad:
        o = int(desc[i]["in_off"])
        out[o + recs[i][0] + 5] ^= 0x80  # tag byte
    snapshot = bytes(out)
    d_buf = dev(out)
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, len(keys), d_desc, len(recs), d_buf, d_buf, d_st, d_ad)
    st = host(d_st)
    res = host(d_buf)
    for i, (L, ad, ki, n, _, _) in enumerate(recs):
        o = int(desc[i]["in_off"])
        if i in bad:
            assert st[i] == noise_amd.REC_BAD_MAC
            assert res[o:o + L + 16] == snapshot[o:o + L + 16], ("in-place failure must keep ct", i, L)
        else:
            assert st[i] == noise_amd.REC_OK, (i, L)
            assert res[o:o + L] == pts[i], (i, L)


def test_mixed_batch_bad_key_index(oracle):
    rng = random.Random(5)
    keys, recs = make_batch(rng, n_small=2100, n_big=8, nkeys=5)
    for i in (3, 10, 11):
        recs[i][2] = 5 + i  # outside the table
    pts = [rng.randbytes(r[0]) for r in recs]
    desc, in_bytes, out_bytes, ad_bytes = layout(recs, decrypt=False)
    inb = bytearray(in_bytes)
    fill(inb, desc, pts, "in_off")
    adb = bytearray(ad_bytes)
    fill(adb, desc, [r[1] for r in recs], "ad_off")
    d_keys, d_ad = dev(b"".join(keys)), dev(adb)
    d_out = torch.full((out_bytes,), 0xEE, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_records(d_keys, len(keys), dev(desc.view(np.uint8)), len(recs), dev(inb),
                              d_out, d_ad)
    out = host(d_out)
    for i in (3, 10, 11):
        o, L = int(desc[i]["out_off"]), recs[i][0]
        assert out[o:o + L + 16] == b"\xee" * (L + 16)
    ddesc, din, dout, _ = layout(recs, decrypt=True)
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    d_back = torch.zeros(dout, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, len(keys), dev(ddesc.view(np.uint8)), len(recs),
                              torch.zeros(din, dtype=torch.uint8, device="cuda"), d_back, d_st, d_ad)
    st = host(d_st)
    for i in (3, 10, 11):
        assert st[i] == noise_amd.REC_BAD_KEY
    assert all(s in (noise_amd.REC_BAD_MAC, noise_amd.REC_BAD_KEY) for s in st)


def test_offsets_beyond_2gib(oracle):
    """Records placed more than 2^31 (and 2^32) bytes into their buffers: the
    64-bit offset paths of the tile / wave / generic kernels (an offset whose
    low word has bit 31 set must not sign-extend)."""
    rng = random.Random(31)
    keys, recs = make_batch(rng, n_small=2100, n_big=24)
    gap_in, gap_out = (1 << 31) + 4096 * 3, (1 << 32) + 16 * 5
    pts = [rng.randbytes(r[0]) for r in recs]
    desc, in_bytes, out_bytes, ad_bytes = layout(recs, decrypt=False)
    inb = bytearray(in_bytes)
    fill(inb, desc, pts, "in_off")
    adb = bytearray(ad_bytes)
    fill(adb, desc, [r[1] for r in recs], "ad_off")
    desc["in_off"] += np.uint64(gap_in)
    desc["out_off"] += np.uint64(gap_out)
    d_in = torch.empty(gap_in + in_bytes, dtype=torch.uint8, device="cuda")
    d_in[gap_in:] = dev(inb)
    d_out = torch.full((gap_out + out_bytes,), 0xA5, dtype=torch.uint8, device="cuda")
    d_keys, d_ad = dev(b"".join(keys)), dev(adb)
    noise_amd.encrypt_records(d_keys, len(keys), dev(desc.view(np.uint8)), len(recs), d_in, d_out,
                              d_ad)
    out = host(d_out[gap_out:])
    for i, (L, ad, ki, n, _, _) in enumerate(recs):
        o = int(desc[i]["out_off"]) - gap_out
        assert out[o:o + L + 16] == oracle.encrypt(keys[ki], n, ad, pts[i]), (i, L)
    # and back, decrypting from beyond 4 GiB into beyond 2 GiB
    ddesc = desc.copy()
    ddesc["in_off"], ddesc["out_off"] = desc["out_off"], desc["in_off"]
    d_back = torch.zeros(gap_in + in_bytes, dtype=torch.uint8, device="cuda")
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, len(keys), dev(ddesc.view(np.uint8)), len(recs), d_out,
                              d_back, d_st, d_ad)
    st = host(d_st)
    back = host(d_back[gap_in:])
    assert all(s == noise_amd.REC_OK for s in st)
    for i, (L, *_rest) in enumerate(recs):
        o = int(desc[i]["in_off"]) - gap_in
        assert back[o:o + L] == pts[i], (i, L)


def test_mixed_batch_zero_key_rows(oracle):
    """All-zero key rows are "no key": records of every class (tile sizes,
    1 KiB, long segmented records, generic) under such a row are not written
    and decrypt reports BAD_KEY; the rest of the batch is unaffected."""
    rng = random.Random(6)
    keys, recs = make_batch(rng, n_small=2100, n_big=30, nkeys=6)
    keys[4] = bytes(32)
    pts = [rng.randbytes(r[0]) for r in recs]
    zero = {i for i, r in enumerate(recs) if r[2] == 4}
    assert len(zero) > 100 and any(recs[i][0] >= 16385 for i in zero)
    desc, in_bytes, out_bytes, ad_bytes = layout(recs, decrypt=False)
    inb = bytearray(in_bytes)
    fill(inb, desc, pts, "in_off")
    adb = bytearray(ad_bytes)
    fill(adb, desc, [r[1] for r in recs], "ad_off")
    d_keys, d_ad = dev(b"".join(keys)), dev(adb)
    d_out = torch.full((out_bytes,), 0xEE, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_records(d_keys, len(keys), dev(desc.view(np.uint8)), len(recs), dev(inb), d_out, d_ad)
    out = host(d_out)
    cts = []
    for i, (L, ad, ki, n, _, _) in enumerate(recs):
        o = int(desc[i]["out_off"])
        if i in zero:
            assert out[o:o + L + 16] == b"\xee" * (L + 16), (i, L)
            cts.append(bytearray(L + 16))
        else:
            want = oracle.encrypt(keys[ki], n, ad, pts[i])
            assert out[o:o + L + 16] == want, (i, L)
            cts.append(bytearray(want))
    ddesc, din, dout, _ = layout(recs, decrypt=True)
    cin = bytearray(din)
    fill(cin, ddesc, cts, "in_off")
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    d_back = torch.full((dout,), 0x77, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, len(keys), dev(ddesc.view(np.uint8)), len(recs), dev(cin), d_back,
                              d_st, d_ad)
    st = host(d_st)
    back = host(d_back)
    for i, (L, *_rest) in enumerate(recs):
        o = int(ddesc[i]["out_off"])
        if i in zero:
            assert st[i] == noise_amd.REC_BAD_KEY, (i, L)
            assert back[o:o + L] == b"\x77" * L, ("nothing written", i, L)
        else:
            assert st[i] == noise_amd.REC_OK and back[o:o + L] == pts[i], (i, L)


@pytest.mark.parametrize("in_place", [False, True])
def test_chunked_decrypt_pipeline_tamper(oracle, in_place):
    """Batches of >= 65536 records run the verify-first decrypt of the long
    records in kSegChunks chunks over three streams (records_kernels.hip
    launch_classes: Poly1305 pass + tag check on the caller's stream, the
    segments' keystream pass on the second companion stream, the tails' on
    the first, joined by the fin[c] / xdone / join2 events).  Tampered long
    records (with and without tails; ct and tag bytes) sit in every chunk:
    their status is BAD_MAC, a failed copy's output is zeroed, a failed
    in-place record keeps its ciphertext, and every other record matches the
    oracle -- on the GPU, where those events really order the passes
    (crypto_aead_read, monocypher.c:2912-2929)."""
    rng = random.Random(4242 + in_place)
    nkeys = 11
    keys = [rng.randbytes(32) for _ in range(nkeys)]
    longs = [1024 * 2, 1024 * 5 + 1, 16384, 16385, 65519, 40001, 1024 * 9 + 1009, 3071, 32768, 20000]
    recs = []
    for i in range(70000):
        if i % 70 == 35:
            L = longs[(i // 70) % len(longs)]
        else:
            L = 64 if i % 3 else 128
        recs.append([L, b"", rng.randrange(nkeys), rng.getrandbits(64) % (2**64 - 2), 0, 0])
    pts = [rng.randbytes(r[0]) for r in recs]
    long_idx = [i for i, r in enumerate(recs) if r[0] > 1024]
    assert len(long_idx) == 1000
    # every 13th long record is tampered: ~77, spread over the record order
    # (the chunks split the long records in record order)
    bad = set(long_idx[5::13])
    cts = []
    for i, (L, ad, ki, n, _, _) in enumerate(recs):
        ct = bytearray(oracle.encrypt(keys[ki], n, ad, pts[i]))
        if i in bad:
            pos = rng.randrange(L + 16) if rng.random() < 0.7 else L + rng.randrange(16)
            ct[pos] ^= 1 << rng.randrange(8)
        cts.append(ct)
    ddesc, din, dout, _ = layout(recs, decrypt=True, in_place=in_place)
    cin = bytearray(din)
    fill(cin, ddesc, cts, "in_off")
    snapshot = bytes(cin)
    d_keys, d_desc = dev(b"".join(keys)), dev(ddesc.view(np.uint8))
    d_in = dev(cin)
    d_out = d_in if in_place else torch.full((dout,), 0x3C, dtype=torch.uint8, device="cuda")
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, nkeys, d_desc, len(recs), d_in, d_out, d_st, None)
    st = host(d_st)
    back = host(d_out)
    for i, (L, *_rest) in enumerate(recs):
        o = int(ddesc[i]["out_off"])
        if i in bad:
            assert st[i] == noise_amd.REC_BAD_MAC, (i, L)
            if in_place:
                assert back[o:o + L + 16] == snapshot[o:o + L + 16], ("in-place failure must keep ct", i, L)
            else:
                assert back[o:o + L] == bytes(L), ("failed copy must be zeroed", i, L)
        else:
            assert st[i] == noise_amd.REC_OK, (i, L, st[i])
            assert back[o:o + L] == pts[i], (i, L)
        if not in_place:
            assert back[o + L:o + L + 16] == b"\x3c" * 16, ("wrote past the record", i, L)


@pytest.mark.parametrize("in_place", [False, True], ids=["copy", "in_place"])
def test_whole_record_classes_tamper(oracle, in_place):
    """Records of exactly 2, 4, 8 and 16 KiB take the whole-record tile
    classes (records_kernels.hip, round 5; 128 KiB super-tiles from 4 KiB up):
    every tag is checked in the wave that holds the record, before its
    plaintext is stored (crypto_aead_read, monocypher.c:2912-2929).  2400
    records (several super-tiles per class and partial last ones), every 7th
    tampered in a ciphertext or tag byte: bit-exact against the oracle,
    REC_BAD_MAC, a failed copy zeroed, a failed in-place record untouched,
    nothing written past a record."""
    rng = random.Random(4096 + in_place)
    nkeys = 9
    keys = [rng.randbytes(32) for _ in range(nkeys)]
    recs = []
    for L in (2048, 4096, 8192, 16384):
        for _ in range(600 - 7 * (L >> 12)):  # class sizes not multiples of a super-tile
            recs.append([L, b"", rng.randrange(nkeys), rng.getrandbits(64) % (2**64 - 2), 0, 0])
    rng.shuffle(recs)
    pts = [rng.randbytes(r[0]) for r in recs]
    cts = [bytearray(oracle.encrypt(keys[r[2]], r[3], b"", pts[i])) for i, r in enumerate(recs)]
    bad = set(range(3, len(recs), 7))
    for i in bad:
        cts[i][rng.randrange(recs[i][0] + 16)] ^= 1 << rng.randrange(8)
    d_keys = dev(b"".join(keys))
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    if in_place:
        desc, nbytes, _, _ = layout(recs, decrypt=True, in_place=True)
        buf = bytearray(nbytes)
        fill(buf, desc, cts, "in_off")
        d_buf = dev(buf)
        noise_amd.decrypt_records(d_keys, nkeys, dev(desc.view(np.uint8)), len(recs), d_buf, d_buf, d_st,
                                  dev(b""))
        res = host(d_buf)
        st = host(d_st)
        for i, (L, _, _, _, _, _) in enumerate(recs):
            o = int(desc[i]["in_off"])
            if i in bad:
                assert st[i] == noise_amd.REC_BAD_MAC, (i, L)
                assert res[o:o + L + 16] == bytes(cts[i]), ("in-place failure must keep ct", i, L)
            else:
                assert st[i] == noise_amd.REC_OK, (i, L, st[i])
                assert res[o:o + L] == pts[i], (i, L)
        return
    desc, din, dout, _ = layout(recs, decrypt=True)
    cin = bytearray(din)
    fill(cin, desc, cts, "in_off")
    d_back = torch.full((dout,), 0x3C, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, nkeys, dev(desc.view(np.uint8)), len(recs), dev(cin), d_back, d_st,
                              dev(b""))
    back = host(d_back)
    st = host(d_st)
    for i, (L, _, _, _, _, _) in enumerate(recs):
        o = int(desc[i]["out_off"])
        if i in bad:
            assert st[i] == noise_amd.REC_BAD_MAC, (i, L)
            assert back[o:o + L] == bytes(L), ("failed copy must be zeroed", i, L)
        else:
            assert st[i] == noise_amd.REC_OK, (i, L, st[i])
            assert back[o:o + L] == pts[i], (i, L)
        assert back[o + L:o + L + 16] == b"\x3c" * 16, ("wrote past the record", i, L)


RAGGED = [1, 33, 64, 65, 100, 127, 129, 191, 193, 255, 257, 300, 480, 511, 513, 700, 961, 1000, 1023, 1025,
          1040, 1400, 1985, 2047, 2049, 3000, 4033, 4095, 4097, 5000, 8129, 8191, 8193, 9000, 12288, 12289,
          16000, 16321,
          16383, 16385, 17000, 32705, 32767, 65456, 65500, 65519]


@pytest.mark.parametrize("in_place", [False, True], ids=["copy", "in_place"])
def test_ragged_classes_tamper(oracle, in_place):
    """Round 6: records of every length class OFF
    the exact tile table -- 1 .. 16383 B take the masked tile classes
    (mtile_kernel.hpp: a record whole in one wave's tile, its tag checked
    there before any plaintext is stored), 16385 .. 65519 B the 1 KiB
    segments with a masked tail unit -- beside exact records in one batch.
    Encrypt bit-exact against the oracle, nothing written past a record's
    ct || tag; then every 5th record tampered (first / last ciphertext byte
    or a tag byte) and decrypted: REC_BAD_MAC, a failed copy zeroed, a
    failed in-place record untouched, nothing written past a record."""
    rng = random.Random(0x52414747 + in_place)
    nkeys = 7
    keys = [rng.randbytes(32) for _ in range(nkeys)]
    recs = []
    for L in RAGGED * 50 + TILE * 10:  # > 2048 records: the classified path
        recs.append([L, b"", rng.randrange(nkeys), rng.getrandbits(64) % (2**64 - 2), 0, 0])
    rng.shuffle(recs)
    pts = [rng.randbytes(r[0]) for r in recs]
    d_keys = dev(b"".join(keys))
    # encrypt (copy layout; the in-place variant encrypts in place too)
    desc, din, dout, _ = layout(recs, decrypt=False, in_place=in_place)
    src = bytearray(din)
    fill(src, desc, pts, "in_off")
    if in_place:
        d_buf = dev(src)
        noise_amd.encrypt_records(d_keys, nkeys, dev(desc.view(np.uint8)), len(recs), d_buf, d_buf, dev(b""))
        ct_img = host(d_buf)
    else:
        d_out = torch.full((dout,), 0x3C, dtype=torch.uint8, device="cuda")
        noise_amd.encrypt_records(d_keys, nkeys, dev(desc.view(np.uint8)), len(recs), dev(src), d_out, dev(b""))
        ct_img = host(d_out)
    cts = []
    for i, (L, _, ki, n, _, _) in enumerate(recs):
        o = int(desc[i]["out_off"])
        want = oracle.encrypt(keys[ki], n, b"", pts[i])
        assert ct_img[o:o + L + 16] == want, ("encrypt", i, L)
        if not in_place:
            assert ct_img[o + L + 16:o + L + 32] == b"\x3c" * 16, ("wrote past the record", i, L)
        cts.append(bytearray(want))
    bad = set(range(2, len(recs), 5))
    for i in bad:
        L = recs[i][0]
        pos = [0, L - 1, L + rng.randrange(16)][i % 3]
        cts[i][pos] ^= 1 << rng.randrange(8)
    d_st = torch.full((len(recs),), 9, dtype=torch.uint8, device="cuda")
    if in_place:
        ddesc, nbytes, _, _ = layout(recs, decrypt=True, in_place=True)
        buf = bytearray(nbytes)
        fill(buf, ddesc, cts, "in_off")
        d_buf = dev(buf)
        noise_amd.decrypt_records(d_keys, nkeys, dev(ddesc.view(np.uint8)), len(recs), d_buf, d_buf, d_st,
                                  dev(b""))
        res, st = host(d_buf), host(d_st)
        for i, (L, _, _, _, _, _) in enumerate(recs):
            o = int(ddesc[i]["in_off"])
            if i in bad:
                assert st[i] == noise_amd.REC_BAD_MAC, (i, L)
                assert res[o:o + L + 16] == bytes(cts[i]), ("in-place failure must keep ct", i, L)
            else:
                assert st[i] == noise_amd.REC_OK, (i, L, st[i])
                assert res[o:o + L] == pts[i], (i, L)
                assert res[o + L:o + L + 16] == bytes(cts[i][L:]), ("in-place decrypt wrote the tag", i, L)
        return
    ddesc, din, dout, _ = layout(recs, decrypt=True)
    cin = bytearray(din)
    fill(cin, ddesc, cts, "in_off")
    d_back = torch.full((dout,), 0x3C, dtype=torch.uint8, device="cuda")
    noise_amd.decrypt_records(d_keys, nkeys, dev(ddesc.view(np.uint8)), len(recs), dev(cin), d_back, d_st,
                              dev(b""))
    back, st = host(d_back), host(d_st)
    for i, (L, _, _, _, _, _) in enumerate(recs):
        o = int(ddesc[i]["out_off"])
        if i in bad:
            assert st[i] == noise_amd.REC_BAD_MAC, (i, L)
            assert back[o:o + L] == bytes(L), ("failed copy must be zeroed", i, L)
        else:
            assert st[i] == noise_amd.REC_OK, (i, L, st[i])
            assert back[o:o + L] == pts[i], (i, L)
        assert back[o + L:o + L + 16] == b"\x3c" * 16, ("wrote past the record", i, L)
