"""GPU parity of the batched X25519 kernel (csrc/x25519_kernels.hip,
noise_gpu_x25519) against RFC 7748 (§5.2 and §6.1 test vectors) and the
independent pure-Python ladder of tests/golden/make_fixtures.py, on random
scalars and u-coordinates including non-canonical ones (u >= p, bit 255 set,
u = 0, 1, p-1).  Bit-exact."""
import os
import random
import sys

import numpy as np
import pytest

import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_fixtures  # noqa: E402  (test infrastructure: the Python ladder)

P = 2 ** 255 - 19


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    noise_amd.load()
    torch.cuda.set_device(0)


def gpu_x25519(scalars, points):
    n = len(scalars)
    d_s = torch.from_numpy(np.frombuffer(b"".join(scalars), dtype=np.uint8).copy()).cuda()
    d_p = None
    if points is not None:
        d_p = torch.from_numpy(np.frombuffer(b"".join(points), dtype=np.uint8).copy()).cuda()
    d_o = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    noise_amd.x25519(d_s, d_p, d_o, n)
    torch.cuda.synchronize()
    out = d_o.cpu().numpy().tobytes()
    return [out[32 * i:32 * i + 32] for i in range(n)]


def test_rfc7748_vectors():
    h = bytes.fromhex
    sc = [h("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4"),
          h("4b66e9d4d1b4673c5ad22691957d6af5c11b6421e0ea01d42ca4169e7918ba0d"),
          h("77076d0a7318a57d3c16c17251b26645df4c2f87ebc0992ab177fba51db92c2a"),
          h("5dab087e624a8a4b79e17f8b83800ee66f3bb1292618b6fd1c2f8b27ff88e0eb")]
    pts = [h("e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c"),
           h("e5210f12786811d3f4b7959d0538ae2c31dbe7106fc03c3efc4cd549c715a493"),
           h("de9edb7d7b7dc1b4d35b61c2ece435373f8343c85b78674dadfc7e146f882b4f"),
           h("8520f0098930a754748b7ddcb43ef75a0dbf3a0d26381af4eba4a98eaa9b4e6a")]
    want = ["c3da55379de9c6908e94ea4df28d084f32eccf03491c71f754b4075577a28552",
            "95cbde9476e8907d7aade45cb4b873f88b595a68799fa152e6f8f7647aac7957",
            "4a5d9d5ba4ce2de1728e3bf480350f25e07e21c947d19e3376f09b3c1e161742",
            "4a5d9d5ba4ce2de1728e3bf480350f25e07e21c947d19e3376f09b3c1e161742"]
    assert [o.hex() for o in gpu_x25519(sc, pts)] == want
    # public keys: the base point
    pub = gpu_x25519(sc[2:], None)
    assert [o.hex() for o in pub] == [pts[3].hex(), pts[2].hex()]


def test_random_and_noncanonical_vs_python_ladder():
    rng = random.Random(7748)
    n = 1500
    sc = [rng.randbytes(32) for _ in range(n)]
    pts = [rng.randbytes(32) for _ in range(n)]
    edge = [0, 1, 9, P - 1, P, P + 1, 2 ** 255 - 1, 2 ** 256 - 1]
    for i, u in enumerate(edge):
        pts[i] = u.to_bytes(32, "little")
    got = gpu_x25519(sc, pts)
    for i in range(n):
        assert got[i] == make_fixtures.x25519(sc[i], pts[i]), "lane %d" % i


def test_vs_reference_monocypher():
    """Against the reference's own crypto_x25519 (monocypher.c, compiled into
    oracle/_ref by oracle/Makefile; travels to the GPU box as a built .so)."""
    import ctypes
    path = os.path.join(noise_amd.ROOT, "oracle", "_ref", "libnoise_ref.so")
    if not os.path.exists(path):
        pytest.skip("oracle/_ref not built")
    ref = ctypes.CDLL(path)
    rng = random.Random(1546)
    sc = [rng.randbytes(32) for _ in range(512)]
    pts = [rng.randbytes(32) for _ in range(512)]
    got = gpu_x25519(sc, pts)
    for i in range(512):
        out = ctypes.create_string_buffer(32)
        ref.ref_x25519(out, sc[i], pts[i])
        assert got[i] == out.raw, "lane %d" % i


def test_ragged_count_and_alignment_check():
    rng = random.Random(3)
    sc = [rng.randbytes(32) for _ in range(77)]  # a partial last wave
    got = gpu_x25519(sc, None)
    base = (9).to_bytes(32, "little")
    for i in (0, 63, 64, 76):
        assert got[i] == make_fixtures.x25519(sc[i], base)
    d = torch.zeros(64 + 1, dtype=torch.uint8, device="cuda")
    with pytest.raises(noise_amd.NoiseGpuError):
        noise_amd.load()
        rc = noise_amd._lib.noise_gpu_x25519(d.data_ptr() + 1, None, d.data_ptr(), 1, None)
        noise_amd._check(rc, "noise_gpu_x25519")
