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


def test_synthetic_generator_offsets(oracle):
    whole = oracle.synthetic(4096, 0x4E4F495345)
    assert oracle.synthetic(1000, 0x4E4F495345, offset=1234) == whole[1234:2234]
