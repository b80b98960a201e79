"""CPU: pin the oracle (oracle/chachapoly_oracle.c) to the reference's own
golden data, the SURVEY known-answer tests, and monocypher itself."""
import hashlib
import os
import random

import pytest

import oracle_lib


def test_golden_counts(golden):
    assert len(golden["transport"]) == 1688
    assert len(golden["handshake"]) == 1828
    assert {len(r["ad"]) for r in golden["handshake"]} == {32, 64}


@pytest.mark.parametrize("kind", ["transport", "handshake"])
def test_oracle_matches_golden(oracle, golden, kind):
    for r in golden[kind]:
        assert oracle.encrypt(r["key"], r["nonce"], r["ad"], r["pt"]) == r["ct"], r["vector"]
        assert oracle.decrypt(r["key"], r["nonce"], r["ad"], r["ct"]) == r["pt"]


def test_oracle_rejects_tampering(oracle, golden):
    rng = random.Random(1)
    for r in golden["handshake"][:300]:
        ct = bytearray(r["ct"])
        ct[rng.randrange(len(ct))] ^= 1 << rng.randrange(8)
        assert oracle.decrypt(r["key"], r["nonce"], r["ad"], bytes(ct)) is None
        if r["ad"]:
            ad = bytearray(r["ad"]); ad[0] ^= 0x80
            assert oracle.decrypt(r["key"], r["nonce"], bytes(ad), r["ct"]) is None
        assert oracle.decrypt(r["key"], r["nonce"] + 1, r["ad"], r["ct"]) is None
    assert oracle.decrypt(bytes(32), 0, b"", b"short") is None  # < 16 bytes


@pytest.mark.parametrize("kat", [oracle_lib.KAT_K1, oracle_lib.KAT_K2, oracle_lib.KAT_K3])
def test_vector_kats(oracle, kat):
    k, n, ad, pt, ct = kat
    assert oracle.encrypt(bytes.fromhex(k), n, bytes.fromhex(ad), bytes.fromhex(pt)).hex() == ct


@pytest.mark.parametrize("n", sorted(oracle_lib.KAT_K5))
def test_k5_1kib_kat(oracle, n):
    head, tag, digest = oracle_lib.KAT_K5[n]
    out = oracle.encrypt(bytes(range(32)), n, b"", oracle_lib.k5_plaintext())
    assert out[:16].hex() == head and out[1024:].hex() == tag
    assert hashlib.blake2b(out[:1024], digest_size=32).hexdigest() == digest


def test_rekey_kat(oracle):
    assert oracle.rekey(bytes(32)).hex() == oracle_lib.KAT_K4_REKEY_ZERO


@pytest.mark.skipif(not os.path.exists(oracle_lib.REF_SO), reason="oracle/_ref not built")
def test_oracle_matches_monocypher(oracle):
    """Random lengths/AD/nonces: the restatement == the reference's monocypher.c."""
    rng = random.Random(7)
    lens = list(range(0, 200)) + [255, 256, 257, 1023, 1024, 1025, 4096, 65519]
    for i, L in enumerate(lens):
        key = rng.randbytes(32)
        n = rng.choice([0, 1, 2**32 - 1, 2**32, 2**63, 2**64 - 3, 2**64 - 1, rng.getrandbits(64)])
        ad = rng.randbytes(rng.choice([0, 0, 1, 16, 17, 32, 64, 100]))
        pt = rng.randbytes(L)
        a = oracle.encrypt(key, n, ad, pt)
        b = oracle.encrypt(key, n, ad, pt, lib=oracle.ref)
        assert a == b, (L, n, len(ad))
        assert oracle.decrypt(key, n, ad, a, lib=oracle.ref) == pt


def test_whole_batch_checkers(oracle):
    """oracle_check_records / oracle_check_uniform (the full-size GPU parity
    checkers): a correct batch passes, every kind of single-record damage is
    counted and located -- ciphertext byte, tag byte, wrong status, a
    plaintext byte behind an OK status, windows (in_base/out_base)."""
    import numpy as np

    import noise_amd
    rng = random.Random(8)
    nrec = 300
    keys = [rng.randbytes(32) for _ in range(5)] + [bytes(32)]  # row 5: no key
    lens = [rng.choice([0, 1, 16, 64, 100, 1024, 1500]) for _ in range(nrec)]
    desc = np.zeros(nrec, dtype=noise_amd.record_dtype())
    inb, outb, ptb = bytearray(), bytearray(), bytearray()
    for i, L in enumerate(lens):
        ki = i % 6 if i % 50 else 9  # every 50th: key index past the table
        ad = rng.randbytes(rng.choice([0, 0, 32]))
        pt = rng.randbytes(L)
        desc[i] = (len(inb), len(outb), rng.getrandbits(64), 0, L, 0, ki, 0)
        ct = oracle.encrypt(keys[ki], int(desc[i]["nonce"]), b"", pt) if ki < 5 else bytes(L + 16)
        inb += pt + bytes(7)
        outb += ct + bytes(3)
        ptb += pt
        del ad
    kt = np.frombuffer(b"".join(keys), dtype=np.uint8).copy()
    ia, oa = np.frombuffer(bytes(inb), dtype=np.uint8).copy(), np.frombuffer(bytes(outb), dtype=np.uint8).copy()
    assert oracle.check_records(0, kt, 6, desc, ia, oa) == (0, -1)
    oa[int(desc[19]["out_off"]) + lens[19] + 3] ^= 1  # a tag byte of record 19
    j = next(i for i in range(40, nrec) if lens[i] and i % 6 < 5 and i % 50)
    oa[int(desc[j]["out_off"])] ^= 0x80                # a ciphertext byte
    assert oracle.check_records(0, kt, 6, desc, ia, oa) == (2, 19)
    # decrypt direction: ct in, plaintext out, statuses
    ddesc = desc.copy()
    ddesc["in_off"], ddesc["out_off"] = desc["out_off"], desc["in_off"]
    st = np.array([0 if (i % 6 < 5 and i % 50) else 2 for i in range(nrec)], dtype=np.uint8)
    st[19] = st[j] = 1
    back = ia.copy()
    assert oracle.check_records(1, kt, 6, ddesc, oa, back, status=st) == (0, -1)
    st[j] = 0
    assert oracle.check_records(1, kt, 6, ddesc, oa, back, status=st)[0] == 1
    st[j] = 1
    k = next(i for i in range(60, nrec) if lens[i] and st[i] == 0)
    back[int(ddesc[k]["out_off"])] ^= 2
    assert oracle.check_records(1, kt, 6, ddesc, oa, back, status=st) == (1, k)
    # windows: records 100.. checked against buffers that start at their offsets
    sub = desc[100:]
    i0, o0 = int(sub[0]["in_off"]), int(sub[0]["out_off"])
    bad, first = oracle.check_records(0, kt, 6, sub, ia[i0:].copy(), oa[o0:].copy(),
                                      in_base=i0, out_base=o0)
    assert bad == (1 if j >= 100 else 0) and first == (j - 100 if j >= 100 else -1)
    # uniform form, strided
    key, L, n0, R = rng.randbytes(32), 256, 2**32 - 5, 64
    pt = np.frombuffer(rng.randbytes(R * L), dtype=np.uint8).copy()
    ct = oracle.encrypt_uniform_np(key, n0, pt, L, L, L + 32, R)
    ct = np.concatenate([ct, np.zeros(16, np.uint8)])
    assert oracle.check_uniform(0, key, n0, pt, L, ct, L + 32, L, R) == (0, -1)
    ct[40 * (L + 32) + 5] ^= 1
    assert oracle.check_uniform(0, key, n0, pt, L, ct, L + 32, L, R) == (1, 40)
    assert oracle.check_uniform(0, key, n0 + 1, pt, L, ct, L + 32, L, R)[0] == R


def test_fullcheck_windows_cpu(oracle):
    """tests/fullcheck.py (the full-size tests' chunked comparison) on CPU
    tensors with tiny chunks: every window boundary is crossed, a damaged
    record is found wherever it sits."""
    import numpy as np
    import torch

    import fullcheck
    import noise_amd
    rng = random.Random(12)
    key = rng.randbytes(32)
    R, L = 97, 192
    pt = np.frombuffer(rng.randbytes(R * L), dtype=np.uint8).copy()
    ct = oracle.encrypt_uniform_np(key, 7, pt, L, L, L + 16, R)
    d_pt, d_ct = torch.from_numpy(pt), torch.from_numpy(ct.copy())
    fullcheck.check_uniform(oracle, torch, key, 7, d_pt, L, d_ct, L + 16, L, R, chunk=1000)
    st = torch.zeros(R, dtype=torch.uint8)
    fullcheck.check_uniform(oracle, torch, key, 7, d_ct, L + 16, d_pt, L, L, R, decrypt=True,
                            d_status=st, chunk=700)
    lens = np.array([rng.choice([1, 64, 300, 1024, 2000]) for _ in range(R)], dtype=np.uint32)
    desc = np.zeros(R, dtype=noise_amd.record_dtype())
    desc["in_off"] = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 5)[:-1]])
    desc["out_off"] = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 16 + 3)[:-1]])
    desc["nonce"] = np.arange(R, dtype=np.uint64) * np.uint64(3)
    desc["len"] = lens
    inb = np.frombuffer(rng.randbytes(int(desc["in_off"][-1]) + int(lens[-1])), np.uint8).copy()
    outb = np.zeros(int(desc["out_off"][-1]) + int(lens[-1]) + 16, dtype=np.uint8)
    for i in range(R):
        o, n = int(desc["in_off"][i]), int(lens[i])
        c = oracle.encrypt(key, int(desc["nonce"][i]), b"", inb[o:o + n].tobytes())
        outb[int(desc["out_off"][i]):int(desc["out_off"][i]) + n + 16] = np.frombuffer(c, np.uint8)
    kt = np.frombuffer(key, np.uint8).copy()
    fullcheck.check_records(oracle, torch, kt, desc, torch.from_numpy(inb),
                            torch.from_numpy(outb), chunk=3000)
    outb[int(desc["out_off"][60]) + int(lens[60]) + 15] ^= 1
    with pytest.raises(AssertionError, match="1 of 97 records differ from the oracle, first 60"):
        fullcheck.check_records(oracle, torch, kt, desc, torch.from_numpy(inb),
                                torch.from_numpy(outb), chunk=3000)


def test_synthetic_generator_offsets(oracle):
    whole = oracle.synthetic(4096, 0x4E4F495345)
    assert oracle.synthetic(1000, 0x4E4F495345, offset=1234) == whole[1234:2234]
