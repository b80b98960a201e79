"""GPU parity at BASELINE full size for configs 3, 4 and 5 (config 2:
test_gpu_parity.py::test_config2_full_size_round_trip), built exactly as
bench.py builds them.  EVERY record of every batch is compared bit for bit
with the CPU oracle, in both directions (tests/fullcheck.py: chunked D2H into
pinned memory, oracle_check_uniform / oracle_check_records on the host
threads), plus the size-independent properties -- every tag verifies,
decrypt(encrypt(x)) == x byte for byte.  Config 4 includes more than 1000
records of 65519 B, the largest Noise message (noise.cpp:886, 982)."""
import sys

import numpy as np
import pytest

import fullcheck
import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = noise_amd.ROOT
sys.path.insert(0, ROOT)
SEED = 0x4E4F495345


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    noise_amd.load()
    torch.cuda.set_device(0)
    yield
    torch.cuda.empty_cache()


def _bytes(t):
    return t.cpu().numpy().tobytes()


def test_config3_full_size_sessions(oracle):
    """65536 sessions x 16 records x 1 KiB through encrypt_sessions /
    decrypt_sessions; record i -> session i mod 65536, nonce (s << 32) + i div
    65536 (nonce word 15 set), keys from splitmix64(0x4B4559)."""
    S, per, L = 65536, 16, 1024
    R = S * per
    d_pt = torch.empty(R * L, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d_pt, R * L, SEED)
    d_keys = torch.empty(S * 32, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d_keys, S * 32, 0x4B4559)
    i = torch.arange(R, dtype=torch.int64, device="cuda")
    d_idx = (i % S).to(torch.int32)
    d_non = ((i % S) << 32) + i // S
    d_ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
    d_back = torch.empty(R * L, dtype=torch.uint8, device="cuda")
    d_st = torch.full((R,), 9, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_sessions(d_keys, S, d_idx, d_non, d_pt, L, d_ct, L + 16, L, R)
    noise_amd.decrypt_sessions(d_keys, S, d_idx, d_non, d_ct, L + 16, d_back, L, L, d_st, R)
    torch.cuda.synchronize()
    assert int((d_st != 0).sum().item()) == 0, "a tag did not verify"
    assert torch.equal(d_pt, d_back)
    keys = d_keys.cpu().numpy()
    desc = np.zeros(R, dtype=noise_amd.record_dtype())
    r = np.arange(R, dtype=np.uint64)
    desc["in_off"], desc["out_off"] = r * np.uint64(L), r * np.uint64(L + 16)
    desc["nonce"] = ((r % np.uint64(S)) << np.uint64(32)) + r // np.uint64(S)
    desc["len"], desc["key_idx"] = L, (r % np.uint64(S)).astype(np.uint32)
    assert np.array_equal(desc["nonce"].view(np.int64), d_non.cpu().numpy())
    fullcheck.check_records(oracle, torch, keys, desc, d_pt, d_ct)
    ddesc = desc.copy()
    ddesc["in_off"], ddesc["out_off"] = desc["out_off"], desc["in_off"]
    fullcheck.check_records(oracle, torch, keys, ddesc, d_ct, d_back, decrypt=True, d_status=d_st)


@pytest.mark.parametrize("jitter", [False, True], ids=["exact", "jitter"])
def test_config4_full_size_zipf(oracle, jitter):
    """The exact bench batch: 2^20 records of 64 * 2^k bytes, P(k) ~ 1/(k+1),
    top bucket 65519, packed at 16-byte aligned offsets, one key, nonces
    0..R-1, through encrypt_records / decrypt_records (classifier, tile
    classes, 1 KiB segments + tails + finalize, generic).  jitter: the same
    buckets with each length lowered by U(0..63) (bench.py --jitter): the
    masked tile classes and the masked tail units (mtile_kernel.hpp)."""
    import bench
    R = 1 << 20
    lens = bench.zipf_lengths(R, jitter)
    in_sz = (lens + np.uint64(15)) // np.uint64(16) * np.uint64(16)
    ct_sz = (lens + np.uint64(31)) // np.uint64(16) * np.uint64(16)
    in_off = np.concatenate([[0], np.cumsum(in_sz)[:-1]]).astype(np.uint64)
    ct_off = np.concatenate([[0], np.cumsum(ct_sz)[:-1]]).astype(np.uint64)
    enc = np.zeros(R, dtype=noise_amd.record_dtype())
    enc["in_off"], enc["out_off"] = in_off, ct_off
    enc["nonce"] = np.arange(R, dtype=np.uint64)
    enc["len"] = lens
    dec = enc.copy()
    dec["in_off"], dec["out_off"] = ct_off, in_off
    tot_in, tot_ct = int(in_sz.sum()), int(ct_sz.sum())
    key = bytes(range(32))
    d_pt = torch.empty(tot_in, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d_pt, tot_in, SEED)
    # zero the alignment padding so the whole buffers compare after the round trip
    padn = (in_sz - lens).astype(np.int64)
    starts = (in_off + lens).astype(np.int64)
    pad_idx = np.repeat(starts, padn) + (np.arange(int(padn.sum())) -
                                         np.repeat(np.cumsum(padn) - padn, padn))
    d_pt[torch.from_numpy(pad_idx).cuda()] = 0
    d_ct = torch.empty(tot_ct, dtype=torch.uint8, device="cuda")
    d_back = torch.zeros(tot_in, dtype=torch.uint8, device="cuda")
    d_st = torch.full((R,), 9, dtype=torch.uint8, device="cuda")
    d_key = torch.frombuffer(bytearray(key), dtype=torch.uint8).cuda()
    noise_amd.encrypt_records(d_key, 1, torch.from_numpy(enc.view(np.uint8).copy()).cuda(), R, d_pt, d_ct)
    noise_amd.decrypt_records(d_key, 1, torch.from_numpy(dec.view(np.uint8).copy()).cuda(), R, d_ct,
                              d_back, d_st)
    torch.cuda.synchronize()
    assert int((d_st != 0).sum().item()) == 0, "a tag did not verify"
    assert torch.equal(d_pt, d_back)
    kt = np.frombuffer(key, dtype=np.uint8).copy()
    fullcheck.check_records(oracle, torch, kt, enc, d_pt, d_ct)
    fullcheck.check_records(oracle, torch, kt, dec, d_ct, d_back, decrypt=True, d_status=d_st)
    assert int((lens == 65519).sum()) > (0 if jitter else 1000)
    if jitter:  # almost every record off the exact tile table, every class used
        assert int(((lens & (lens - np.uint64(1))) == 0).sum()) < R // 20


def test_config5_full_size_shard(oracle):
    """Config 5 at 1 GPU: 8 Mi x 4 KiB, one key, nonce = global index (the
    strong-scaling N = 1 point; ~96 GiB resident), encrypt + decrypt."""
    R, L = 8 << 20, 4096
    key = bytes(range(32))
    d_pt = torch.empty(R * L, dtype=torch.uint8, device="cuda")
    noise_amd.fill_synthetic(d_pt, R * L, SEED)
    d_ct = torch.empty(R * (L + 16), dtype=torch.uint8, device="cuda")
    d_back = torch.empty(R * L, dtype=torch.uint8, device="cuda")
    d_st = torch.full((R,), 9, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_uniform(key, 0, d_pt, L, d_ct, L + 16, L, R)
    noise_amd.decrypt_uniform(key, 0, d_ct, L + 16, d_back, L, L, d_st, R)
    torch.cuda.synchronize()
    assert int((d_st != 0).sum().item()) == 0, "a tag did not verify"
    assert torch.equal(d_pt, d_back)
    fullcheck.check_uniform(oracle, torch, key, 0, d_pt, L, d_ct, L + 16, L, R)
    fullcheck.check_uniform(oracle, torch, key, 0, d_ct, L + 16, d_back, L, L, R, decrypt=True,
                            d_status=d_st)
    for r in (0, R // 2, R - 1):
        assert _bytes(d_pt[r * L:(r + 1) * L]) == oracle.synthetic(L, SEED, offset=r * L)
