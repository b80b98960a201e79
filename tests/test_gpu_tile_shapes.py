"""GPU parity of EVERY shape the C ABI dispatches to the LDS-staged tile
kernel (tile_kernel.hpp): uniform batches (noise_gpu_encrypt_uniform /
_decrypt_uniform) and many-session batches (noise_gpu_encrypt_sessions /
_decrypt_sessions) at all ten lengths noise_gpu.h promises -- 64, 128, 192,
256, 512, 1024, 2048, 4096, 8192, 16384 B, i.e. G = 1..64 lanes per record
and 64..1 records per tile, including the G = 32 / 64 Poly1305 recombination
with its mid-butterfly renormalisation (tile_kernel.hpp, `if (b == 4)`).

Each case: nrec in {1, 63, 64, 65, 200} (a lone record, partial and full
tiles / super-tiles), three layouts (packed = the contiguous variant, padded
strides and in place = the strided variant), nonces crossing 2^32 (and 2^64
for the 65-record cases), every record compared with the CPU oracle
(oracle_check_uniform / oracle_check_records), then two records tampered
(ciphertext byte, tag byte) and the batch decrypted: the tampered records
fail (in place: left untouched; copy: zeroed), every other record decrypts
to its plaintext.  Sessions cases also carry a key index past the table and
an all-zero key row (nothing written, status BAD_KEY).
Reference: crypto_aead_write / crypto_aead_read, monocypher.c:2899-2929;
nonce framing noise.cpp:207-215."""
import random

import numpy as np
import pytest

import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

LENGTHS = [64, 128, 192, 256, 512, 1024, 2048, 4096, 8192, 16384]
NRECS = [1, 63, 64, 65, 200]
LAYOUTS = ["packed", "padded", "in_place"]
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


def _strides(layout, L):
    """(plaintext stride, ciphertext stride); in place uses one buffer."""
    if layout == "packed":
        return L, L + 16
    if layout == "padded":
        return L + 48, L + 32
    return L + 16, L + 16


def _n0(nrec):
    if nrec == 65:
        return 2**64 - 30          # wraps mod 2^64 inside the batch
    return 2**32 - nrec // 2 - 1   # crosses the nonce word-14 -> 15 carry


def _layout_rows(pt, nrec, L, stride):
    buf = np.zeros(stride * nrec, dtype=np.uint8)
    rows = buf.reshape(nrec, stride)
    rows[:, :L] = pt.reshape(nrec, L)
    return buf


def _tamper(ct, nrec, L, ct_stride):
    """flip a ciphertext byte of one record and a tag byte of another"""
    bad = {0: L + 3} if nrec == 1 else {nrec // 3: L - 1, nrec - 1: L + 7}
    for r, off in bad.items():
        ct[r * ct_stride + off] ^= 0x10
    return sorted(bad)


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("nrec", NRECS)
@pytest.mark.parametrize("L", LENGTHS)
def test_uniform_tile_shapes(oracle, L, nrec, layout):
    rng = random.Random(L * 7919 + nrec * 31 + len(layout))
    key, n0 = rng.randbytes(32), _n0(nrec)
    ps, cs = _strides(layout, L)
    pt = np.frombuffer(rng.randbytes(nrec * L), dtype=np.uint8)
    src = _layout_rows(pt, nrec, L, ps)
    d_in = torch.from_numpy(src.copy()).cuda()
    if layout == "in_place":
        d_ct = d_in
    else:
        d_ct = torch.full((cs * nrec,), FILL, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, n0, d_in, ps, d_ct, cs, L, nrec)
    ct = _np(d_ct).copy()
    assert oracle.check_uniform(0, key, n0, src, ps, ct, cs, L, nrec) == (0, -1)
    # decrypt a tampered copy
    bad = _tamper(ct, nrec, L, cs)
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
    # the oracle agrees record by record (plaintext where the tag verifies)
    assert oracle.check_uniform(1, key, n0, ct, cs, back, ps, L, nrec, status=st) == (0, -1)
    rows = back.reshape(nrec, ps)[:, :L]
    for r in bad:
        if layout == "in_place":
            assert rows[r].tobytes() == ct[r * cs:r * cs + L].tobytes()  # untouched
        else:
            assert not rows[r].any()  # no unauthenticated plaintext
    ok = np.ones(nrec, dtype=bool)
    ok[bad] = False
    assert np.array_equal(rows[ok], pt.reshape(nrec, L)[ok])


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("nrec", NRECS)
@pytest.mark.parametrize("L", LENGTHS)
def test_sessions_tile_shapes(oracle, L, nrec, layout):
    rng = random.Random(L * 104729 + nrec * 17 + len(layout))
    nkeys = min(nrec, 9) + 1
    keys = [rng.randbytes(32) for _ in range(nkeys)]
    zero_row = nkeys - 1
    keys[zero_row] = bytes(32)  # "no key" (a failed handshake's split row)
    kidx = np.array([r % (nkeys - 1) for r in range(nrec)], dtype=np.uint32)
    bad_key = []
    if nrec >= 63:
        kidx[62] = nkeys + 4  # past the table
        kidx[nrec - 2] = zero_row
        bad_key = [62, nrec - 2]
    base = _n0(nrec)
    nonces = np.array([(base + r + (int(kidx[r]) << 40)) % 2**64 for r in range(nrec)],
                      dtype=np.uint64)
    ps, cs = _strides(layout, L)
    pt = np.frombuffer(rng.randbytes(nrec * L), dtype=np.uint8)
    src = _layout_rows(pt, nrec, L, ps)
    ktab = np.frombuffer(b"".join(keys), dtype=np.uint8).copy()
    d_keys = torch.from_numpy(ktab).cuda()
    d_idx = torch.from_numpy(kidx.view(np.uint8).copy()).cuda()
    d_non = torch.from_numpy(nonces.view(np.uint8).copy()).cuda()
    d_in = torch.from_numpy(src.copy()).cuda()
    if layout == "in_place":
        d_ct = d_in
    else:
        d_ct = torch.full((cs * nrec,), FILL, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_sessions(d_keys, nkeys, d_idx, d_non, d_in, ps, d_ct, cs, L, nrec)
    ct = _np(d_ct).copy()
    desc = np.zeros(nrec, dtype=noise_amd.record_dtype())
    r = np.arange(nrec, dtype=np.uint64)
    desc["in_off"], desc["out_off"] = r * np.uint64(ps), r * np.uint64(cs)
    desc["nonce"], desc["len"], desc["key_idx"] = nonces, L, kidx
    assert oracle.check_records(0, ktab, nkeys, desc, src, ct) == (0, -1)
    for b in bad_key:  # nothing written for a record without a usable key
        want = src[b * ps:b * ps + L + 16] if layout == "in_place" else np.full(L + 16, FILL, np.uint8)
        assert np.array_equal(ct[b * cs:b * cs + L + 16], want[:L + 16]), b
    bad = [b for b in _tamper(ct, nrec, L, cs) if b not in bad_key]
    d_c2 = torch.from_numpy(ct.copy()).cuda()
    d_st = torch.full((nrec,), 9, dtype=torch.uint8, device="cuda")
    if layout == "in_place":
        d_pt = d_c2
        noise_amd.decrypt_sessions(d_keys, nkeys, d_idx, d_non, d_c2, cs, d_c2, cs, L, d_st, nrec)
    else:
        d_pt = torch.full((ps * nrec,), FILL, dtype=torch.uint8, device="cuda")
        noise_amd.decrypt_sessions(d_keys, nkeys, d_idx, d_non, d_c2, cs, d_pt, ps, L, d_st, nrec)
    st, back = _np(d_st), _np(d_pt)
    want_st = np.zeros(nrec, dtype=np.uint8)
    want_st[bad] = noise_amd.REC_BAD_MAC
    want_st[bad_key] = noise_amd.REC_BAD_KEY
    assert np.array_equal(st, want_st)
    ddesc = desc.copy()
    ddesc["in_off"], ddesc["out_off"] = desc["out_off"], desc["in_off"]
    assert oracle.check_records(1, ktab, nkeys, ddesc, ct, back, status=st) == (0, -1)
    rows = back.reshape(nrec, ps)[:, :L]
    ok = np.ones(nrec, dtype=bool)
    ok[bad + bad_key] = False
    assert np.array_equal(rows[ok], pt.reshape(nrec, L)[ok])
    for b in bad:
        if layout == "in_place":
            assert rows[b].tobytes() == ct[b * cs:b * cs + L].tobytes()
        else:
            assert not rows[b].any()
