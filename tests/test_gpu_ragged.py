"""GPU parity of the masked ("ragged") tile kernel (csrc/mtile_kernel.hpp):
record lengths OFF the exact tile table, which before round 6 fell to one
lane per record.

Uniform batches (noise_gpu_encrypt_uniform / _decrypt_uniform) with 16-byte
aligned bases and strides and lengths 1 .. 16383 around every class edge
(the power-of-two tiles and the capacities between them: 320 .. 448 B with
one lane per record, 768 .. 5120 B with 3 .. 20 lanes and idle ones): a
lone record, a partial tile and several tiles / super-tiles; three layouts
(tight = strides rounded up to 16, padded = with gaps, in place).  Every
record is compared with the CPU oracle (oracle_check_uniform), the bytes
between records (and past an in-place plaintext: the tag) must be left
untouched, then records are tampered (first / last ciphertext byte, tag byte)
and the batch decrypted: the tampered records fail (in place: left
untouched; copy: zeroed), every other record decrypts to its plaintext.
Reference: crypto_aead_write / crypto_aead_read, monocypher.c:2899-2929;
nonce framing noise.cpp:207-215; any length noise.cpp:202-281."""
import random

import numpy as np
import pytest

import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

LENGTHS = [1, 15, 17, 63, 65, 100, 129, 191, 193, 255, 257, 300, 511, 513, 700, 1000, 1023, 1025,
           1040, 1400, 2047, 2049, 3000, 4095, 4097, 5000, 8191, 8193, 9000, 16000, 16383]
# the capacities between the powers of two (aead_kernels.hip): each full, and
# one byte past it (the next class)
LENGTHS += [320, 321, 384, 448, 449, 768, 769, 1280, 1536, 1792, 1793, 2304, 2560, 3072, 3073, 5120, 5121]
NRECS = [1, 65, 200]
LAYOUTS = ["tight", "padded", "in_place"]
FILL = 0xEE


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    noise_amd.load()
    torch.cuda.set_device(0)


def _np(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def c16(x):
    return (x + 15) // 16 * 16


def strides(layout, L):
    """(plaintext stride, ciphertext stride), both multiples of 16"""
    if layout == "tight":
        return c16(L), c16(L + 16)
    if layout == "padded":
        return c16(L) + 48, c16(L + 16) + 32
    return c16(L + 16), c16(L + 16)


def tamper_list(nrec, L):
    """record -> byte offset: first / last ciphertext byte, a tag byte"""
    if nrec == 1:
        return {0: L + 15}
    return {0: 0, nrec // 3: L - 1, nrec - 1: L + 7, nrec // 2: L}


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("nrec", NRECS)
@pytest.mark.parametrize("L", LENGTHS)
def test_uniform_ragged(oracle, L, nrec, layout):
    rng = random.Random(L * 7907 + nrec * 13 + len(layout))
    key, n0 = rng.randbytes(32), 2**32 - nrec // 2 - 1  # crosses the nonce word carry
    ps, cs = strides(layout, L)
    pt = np.frombuffer(rng.randbytes(nrec * L), dtype=np.uint8)
    src = np.full(ps * nrec, FILL, dtype=np.uint8)
    src.reshape(nrec, ps)[:, :L] = pt.reshape(nrec, L)
    d_in = torch.from_numpy(src.copy()).cuda()
    if layout == "in_place":
        d_ct = d_in
    else:
        d_ct = torch.full((cs * nrec,), FILL, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, n0, d_in, ps, d_ct, cs, L, nrec)
    ct = _np(d_ct).copy()
    assert oracle.check_uniform(0, key, n0, src, ps, ct, cs, L, nrec) == (0, -1)
    gaps = ct.reshape(nrec, cs)[:, L + 16:]
    assert (gaps == FILL).all(), "encrypt wrote past a record's ct || tag"
    # decrypt a tampered copy
    bad = tamper_list(nrec, L)
    for r, off in bad.items():
        ct[r * cs + off] ^= 0x21
    bad = sorted(bad)
    d_c2 = torch.from_numpy(ct.copy()).cuda()
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    if layout == "in_place":
        d_pt = d_c2
        noise_amd.decrypt_uniform(key, n0, d_c2, cs, d_c2, cs, L, d_st, nrec)
    else:
        d_pt = torch.full((ps * nrec,), FILL, dtype=torch.uint8, device="cuda")
        noise_amd.decrypt_uniform(key, n0, d_c2, cs, d_pt, ps, L, d_st, nrec)
    st, back = _np(d_st), _np(d_pt)
    want_st = np.zeros(nrec, dtype=np.uint8)
    want_st[bad] = noise_amd.REC_BAD_MAC
    assert np.array_equal(st, want_st)
    assert oracle.check_uniform(1, key, n0, ct, cs, back, ps, L, nrec, status=st) == (0, -1)
    rows = back.reshape(nrec, ps)
    if layout == "in_place":  # the tag bytes after the plaintext are not written
        assert np.array_equal(rows[:, L:L + 16], ct.reshape(nrec, cs)[:, L:L + 16])
    else:
        assert (rows[:, L:] == FILL).all(), "decrypt wrote past a record's plaintext"
    for r in bad:
        if layout == "in_place":
            assert rows[r, :L].tobytes() == ct[r * cs:r * cs + L].tobytes()  # untouched
        else:
            assert not rows[r, :L].any()  # no unauthenticated plaintext
    ok = np.ones(nrec, dtype=bool)
    ok[bad] = False
    assert np.array_equal(rows[ok, :L], pt.reshape(nrec, L)[ok])


# Unaligned uniform batches of >= 1024 records (aead_kernels.hip stages them
# through an aligned scratch image for the tile kernels): odd strides and base
# offsets, the Noise wire format packed back to back, in place; the oracle on
# every record, gaps untouched, tampered records fail (in place untouched,
# copies zeroed).  Emulated under ASan by `tools/emu/build/emu_uniform unaligned`.
UNALIGNED = [1, 17, 100, 1000, 1040, 3000, 5000, 16383]


@pytest.mark.parametrize("layout", ["odd", "packed", "in_place"])
@pytest.mark.parametrize("L", UNALIGNED)
def test_uniform_unaligned_staged(oracle, L, layout):
    rng = random.Random(L * 131 + len(layout))
    nrec = 1100 if L <= 5000 else 1030
    key, n0 = rng.randbytes(32), rng.getrandbits(40)
    if layout == "odd":
        ps, cs, po, co = L + 3, L + 16 + 5, 1, 7
    elif layout == "packed":
        ps, cs, po, co = L, L + 16, 3, 3
    else:
        ps = cs = L + 16 + 3
        po = co = 5
    pt = np.frombuffer(rng.randbytes(nrec * L), dtype=np.uint8)
    src = np.full(po + ps * nrec + 32, FILL, dtype=np.uint8)
    src[po:po + ps * nrec].reshape(nrec, ps)[:, :L] = pt.reshape(nrec, L)
    d_in = torch.from_numpy(src.copy()).cuda()
    d_ct = d_in if layout == "in_place" else torch.full((co + cs * nrec + 32,), FILL, dtype=torch.uint8,
                                                         device="cuda")
    noise_amd.encrypt_uniform(key, n0, d_in, ps, d_ct, cs, L, nrec, in_offset=po, out_offset=co)
    ct = _np(d_ct).copy()
    assert oracle.check_uniform(0, key, n0, src[po:], ps, ct[co:], cs, L, nrec) == (0, -1)
    if cs > L + 16:
        assert (ct[co:co + cs * nrec].reshape(nrec, cs)[:, L + 16:] == FILL).all()
    assert (ct[:co] == FILL).all() and (ct[co + cs * nrec:] == FILL).all()
    bad = {0: 0, nrec // 3: L - 1, nrec - 1: L + 7, nrec // 2: L}
    for r, off in bad.items():
        ct[co + r * cs + off] ^= 0x21
    bad = sorted(bad)
    d_c2 = torch.from_numpy(ct.copy()).cuda()
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    if layout == "in_place":
        d_pt, so, ss = d_c2, co, cs
    else:
        d_pt = torch.full((po + ps * nrec + 32,), FILL, dtype=torch.uint8, device="cuda")
        so, ss = po, ps
    noise_amd.decrypt_uniform(key, n0, d_c2, cs, d_pt, ss, L, d_st, nrec, in_offset=co, out_offset=so)
    st, back = _np(d_st), _np(d_pt)
    want = np.zeros(nrec, dtype=np.uint8)
    want[bad] = noise_amd.REC_BAD_MAC
    assert np.array_equal(st, want)
    rows = back[so:so + ss * nrec].reshape(nrec, ss)
    ctr = ct[co:co + cs * nrec].reshape(nrec, cs)
    ok = np.ones(nrec, dtype=bool)
    ok[bad] = False
    assert np.array_equal(rows[ok, :L], pt.reshape(nrec, L)[ok])
    for r in bad:
        if layout == "in_place":
            assert rows[r, :L + 16].tobytes() == ctr[r, :L + 16].tobytes()
        else:
            assert not rows[r, :L].any()
    if layout == "in_place":
        assert np.array_equal(rows[:, L:L + 16], ctr[:, L:L + 16])
    elif ss > L:
        assert (rows[:, L:] == FILL).all()
    assert (back[:so] == FILL).all() and (back[so + ss * nrec:] == FILL).all()
