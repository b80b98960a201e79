"""Host-side Noise handshake primitives (noise-cpp_amd/host/crypto.cpp) and
pattern table (host/handshake.cpp), no GPU: BLAKE2b and HMAC-BLAKE2b against
Python's hashlib/hmac, the Noise HKDF against its rev34 §4.3 definition,
X25519 against RFC 7748 §5.2 and the independent Python ladder of
tests/golden/make_fixtures.py, and the enum's pattern names against the
reference's HandshakePattern list (noise.h:21-81).  The full replay of the
reference's handshake vectors needs the GPU-backed CipherState:
tests/test_gpu_parity.py::test_handshake_vectors."""
import hashlib
import hmac
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "noise-cpp_amd", "bin", "handshake_test")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def run(*args):
    if not os.path.exists(BIN):
        pytest.fail("handshake_test not built (run __graft_entry__.build())")
    r = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout.split()


@pytest.mark.parametrize("n", [0, 1, 3, 63, 64, 127, 128, 129, 255, 256, 257, 1000])
def test_blake2b(n):
    data = bytes(random.Random(n).getrandbits(8) for _ in range(n))
    assert run("blake2b", data.hex() or "-")[0] == hashlib.blake2b(data).hexdigest()


@pytest.mark.parametrize("klen,n", [(0, 5), (32, 0), (64, 100), (64, 129), (100, 7), (200, 33)])
def test_hmac_blake2b(klen, n):
    rng = random.Random(klen * 1000 + n)
    key = bytes(rng.getrandbits(8) for _ in range(klen))
    data = bytes(rng.getrandbits(8) for _ in range(n))
    got = run("hmac", key.hex() or "-", data.hex() or "-")[0]
    assert got == hmac.new(key, data, hashlib.blake2b).hexdigest()


@pytest.mark.parametrize("n", [0, 32, 64])
def test_noise_hkdf(n):
    rng = random.Random(n + 7)
    ck = bytes(rng.getrandbits(8) for _ in range(64))
    ikm = bytes(rng.getrandbits(8) for _ in range(n))
    tk = hmac.new(ck, ikm, hashlib.blake2b).digest()
    o1 = hmac.new(tk, b"\x01", hashlib.blake2b).digest()
    o2 = hmac.new(tk, o1 + b"\x02", hashlib.blake2b).digest()
    o3 = hmac.new(tk, o2 + b"\x03", hashlib.blake2b).digest()
    assert run("hkdf", ck.hex(), ikm.hex() or "-") == [o1.hex(), o2.hex(), o3.hex()]


@pytest.mark.parametrize("sk,u,out", [
    ("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4",
     "e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c",
     "c3da55379de9c6908e94ea4df28d084f32eccf03491c71f754b4075577a28552"),
    ("4b66e9d4d1b4673c5ad22691957d6af5c11b6421e0ea01d42ca4169e7918ba0d",
     "e5210f12786811d3f4b7959d0538ae2c31dbe7106fc03c3efc4cd549c715a493",
     "95cbde9476e8907d7aade45cb4b873f88b595a68799fa152e6f8f7647aac7957"),
])
def test_x25519_rfc7748(sk, u, out):
    assert run("x25519", sk, u)[0] == out


def test_x25519_vs_python_ladder():
    import make_fixtures  # independent pure-Python X25519 (fixture generator)
    rng = random.Random(25519)
    for _ in range(20):
        sk = bytes(rng.getrandbits(8) for _ in range(32))
        u = bytes(rng.getrandbits(8) for _ in range(32))
        assert run("x25519", sk.hex(), u.hex())[0] == make_fixtures.x25519(sk, u).hex()


def test_pattern_names_match_reference_enum():
    # noise.h:21-81 of the reference, in order
    ref = ("IK IN IX K KK KN KX N NK NN NX XK XN XX NK1 NX1 X X1K XK1 X1K1 X1N X1X XX1 X1X1 "
           "K1N K1K KK1 K1K1 K1X KX1 K1X1 I1N I1K IK1 I1K1 I1X IX1 I1X1 Npsk0 Kpsk0 Xpsk1 "
           "NNpsk0 NNpsk2 NKpsk0 NKpsk2 NXpsk2 XNpsk3 XKpsk3 XXpsk3 KNpsk0 KNpsk2 KKpsk0 "
           "KKpsk2 KXpsk2 INpsk1 INpsk2 IKpsk1 IKpsk2 IXpsk2").split()
    assert run("patterns") == ref


def test_handshake_vector_fixture_present():
    path = os.path.join(ROOT, "tests", "golden", "handshake_vectors.tsv")
    rows = [l.split("\t") for l in open(path).read().splitlines() if l]
    assert len(rows) == 110 and all(len(r) == 13 for r in rows)
    assert all(r[0].endswith("_25519_ChaChaPoly_BLAKE2b") for r in rows)


def _py_xx(si, ei, sr, er):
    """Noise_XX_25519_ChaChaPoly_BLAKE2b, both parties, empty prologue and
    payloads, in plain Python (rev34 §5, hashlib BLAKE2b, the Python X25519
    ladder and AEAD of tests/golden/make_fixtures.py): test infrastructure
    pinning oracle/ref_harness.c:ref_xx_handshake."""
    import make_fixtures as mf

    def hkdf(ck, ikm):
        tk = hmac.new(ck, ikm, hashlib.blake2b).digest()
        o1 = hmac.new(tk, b"\x01", hashlib.blake2b).digest()
        return o1, hmac.new(tk, o1 + b"\x02", hashlib.blake2b).digest()

    class Sym:
        def __init__(self):
            self.h = b"Noise_XX_25519_ChaChaPoly_BLAKE2b".ljust(64, b"\0")
            self.ck, self.k, self.n = self.h, None, 0
            self.mix_hash(b"")

        def mix_hash(self, d):
            self.h = hashlib.blake2b(self.h + d).digest()

        def mix_key(self, ikm):
            self.ck, t = hkdf(self.ck, ikm)
            self.k, self.n = t[:32], 0

        def enc(self, pt):
            ct = pt if self.k is None else mf.aead_encrypt(self.k, self.n, self.h, pt)
            self.n += self.k is not None
            self.mix_hash(ct)
            return ct

        def dec(self, ct):
            pt = ct if self.k is None else mf.aead_decrypt(self.k, self.n, self.h, ct)
            self.n += self.k is not None
            self.mix_hash(ct)
            return pt

    pub = lambda sk: mf.x25519(sk, (9).to_bytes(32, "little"))  # noqa: E731
    I, R = Sym(), Sym()
    m1 = pub(ei)
    I.mix_hash(m1); I.enc(b"")
    R.mix_hash(m1); R.dec(b"")
    epr = pub(er)
    R.mix_hash(epr); R.mix_key(mf.x25519(er, m1))
    m2 = epr + R.enc(pub(sr))
    R.mix_key(mf.x25519(sr, m1)); m2 += R.enc(b"")
    I.mix_hash(m2[:32]); I.mix_key(mf.x25519(ei, m2[:32]))
    rs = I.dec(m2[32:80]); I.mix_key(mf.x25519(ei, rs)); I.dec(m2[80:])
    m3 = I.enc(pub(si)); I.mix_key(mf.x25519(si, m2[:32])); m3 += I.enc(b"")
    rsr = R.dec(m3[:48]); R.mix_key(mf.x25519(er, rsr)); R.dec(m3[48:])
    assert I.h == R.h and rsr == pub(si) and rs == pub(sr)
    k1, k2 = hkdf(I.ck, b"")
    return m1, m2, m3, I.h, k1[:32], k2[:32]


@pytest.mark.parametrize("seed", [1, 2])
def test_reference_primitive_xx_matches_spec(oracle, seed):
    """oracle/ref_harness.c:ref_xx_handshake (the reference's Monocypher
    primitives composed as noise.cpp composes them, spec HasKey) equals an
    independent Python XX: it is then the per-session checker of the batched
    GPU handshake (tests/test_gpu_handshake_batch.py) and the CPU baseline of
    tools/bench_handshake.py."""
    if oracle.ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    rng = random.Random(seed)
    keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(4)]
    assert oracle.ref_xx_handshake(*keys) == _py_xx(*keys)
