"""GPU parity of the batched handshakes (noise_gpu_hs_*: csrc/handshake_batch.hip,
csrc/handshake_kernels.hip; SURVEY.md §8(f) rank 4, mass handshakes).

* the reference's 110 Noise_*_25519_ChaChaPoly_BLAKE2b vectors
  (tests/golden/handshake_vectors.tsv, from /root/reference/tests/vectors)
  through the batched API: every handshake message, the handshake hash and
  the transport records under the split keys, byte-exact;
* random keys / prologues / payloads on 18 patterns against the host
  noise::HandshakeState (itself pinned by those vectors) for sampled sessions,
  both sides' split agreeing for every session, tampered messages failing
  exactly their sessions (tests/cpp/handshake_test.cpp batch_check);
* XX on random keys for every session against the reference's own Monocypher
  primitives (oracle/_ref: ref_xx_handshake), and the split keys feeding the
  sessions transport kernel directly on the device;
* length checks (short messages fail their sessions with HS_BAD_LEN)."""
import os
import subprocess

import numpy as np
import pytest

import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = noise_amd.ROOT
BIN = os.path.join(ROOT, "noise-cpp_amd", "bin", "handshake_test")


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    noise_amd.load()
    torch.cuda.set_device(0)


def run(*args, timeout=120):
    r = subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_batch_vectors():
    out = run("batch_vectors", os.path.join(ROOT, "tests", "golden", "handshake_vectors.tsv"))
    assert "batched vectors 110 in" in out and "failed 0" in out, out


@pytest.mark.parametrize("pattern,n", [
    ("XX", 1000), ("NN", 257), ("NK", 130), ("NX", 64), ("XN", 65), ("XK", 100), ("KN", 63),
    ("KK", 128), ("KX", 70), ("IN", 90), ("IK", 300), ("IX", 129), ("N", 100), ("K", 33),
    ("X", 50), ("XXpsk3", 200), ("NNpsk0+psk2", 77), ("IKpsk2", 66), ("X1X1", 40), ("Npsk0", 21)])
def test_batch_vs_host_handshake(pattern, n):
    out = run("batch_check", pattern, n, n + 11)
    assert "ok" in out, out


def _dev(b):
    return torch.from_numpy(np.frombuffer(bytes(b), dtype=np.uint8).copy()).cuda()


def _xx_batch(n, si, ei, sr, er):
    """Both roles of XX for n sessions with preset keys, empty payloads:
    (msgs [3][n] bytes, hash_i, k1_i, k2_i, k1_r, k2_r, rs_r) as device tensors."""
    I, R = noise_amd.HandshakeBatch("XX", True, n), noise_amd.HandshakeBatch("XX", False, n)
    I.set_key(noise_amd.HS_S, _dev(b"".join(si)))
    I.set_key(noise_amd.HS_E, _dev(b"".join(ei)))
    R.set_key(noise_amd.HS_S, _dev(b"".join(sr)))
    R.set_key(noise_amd.HS_E, _dev(b"".join(er)))
    I.start()
    R.start()
    msgs = []
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for m in range(3):
        w, r = (I, R) if m % 2 == 0 else (R, I)
        ov = w.info().overhead
        buf = torch.zeros(n * 128, dtype=torch.uint8, device="cuda")
        w.write_message(noise_amd.span(buf, stride=128))
        r.read_message(noise_amd.span(buf, stride=128, length=ov), d_status=st)
        torch.cuda.synchronize()
        assert int(st.sum()) == 0
        msgs.append(buf.view(n, 128)[:, :ov].cpu().numpy())
    out = [torch.zeros(n * 32, dtype=torch.uint8, device="cuda") for _ in range(5)]
    h = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    I.split(out[0], out[1], d_hash=h)
    R.split(out[2], out[3], d_rs=out[4])
    torch.cuda.synchronize()
    I.close()
    R.close()
    return msgs, h, out


def test_batch_xx_vs_reference_primitives(oracle):
    """Every session of a 4096-session XX batch against the reference's own
    Monocypher primitives (oracle/_ref ref_xx_handshake): the three messages,
    the handshake hash, both split keys, the responder's view of rs."""
    if oracle.ref is None:
        pytest.skip("oracle/_ref not built")
    n = 4096
    rng = np.random.default_rng(5)
    si, ei, sr, er = ([bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(n)]
                      for _ in range(4))
    msgs, h, (k1, k2, k1r, k2r, rs) = _xx_batch(n, si, ei, sr, er)
    h, k1, k2 = h.cpu().numpy(), k1.cpu().numpy(), k2.cpu().numpy()
    assert np.array_equal(k1, k1r.cpu().numpy()) and np.array_equal(k2, k2r.cpu().numpy())
    rs = rs.cpu().numpy()
    for i in range(n):
        m1, m2, m3, hh, r1, r2 = oracle.ref_xx_handshake(si[i], ei[i], sr[i], er[i])
        assert msgs[0][i].tobytes() == m1 and msgs[1][i].tobytes() == m2 and msgs[2][i].tobytes() == m3, i
        assert h[64 * i:64 * i + 64].tobytes() == hh, i
        assert k1[32 * i:32 * i + 32].tobytes() == r1 and k2[32 * i:32 * i + 32].tobytes() == r2, i
    # the responder learned the initiator's static public key
    pub = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    noise_amd.x25519(_dev(b"".join(si)), None, pub, n)
    torch.cuda.synchronize()
    assert np.array_equal(pub.cpu().numpy(), rs)


def test_batch_split_keys_feed_transport(oracle):
    """The split key tables stay on the device and key the sessions transport
    kernel directly: initiator encrypts with k1, responder decrypts with its
    own k1; records vs the CPU oracle under the same keys."""
    n, L, per = 512, 256, 4
    rng = np.random.default_rng(9)
    keys = [[bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(n)] for _ in range(4)]
    _, _, (k1, k2, k1r, k2r, _) = _xx_batch(n, *keys)
    nrec = n * per
    idx = torch.arange(nrec, dtype=torch.int32, device="cuda") % n
    nonces = (torch.arange(nrec, dtype=torch.int64, device="cuda") // n)
    pt = torch.from_numpy(rng.integers(0, 256, nrec * L, dtype=np.uint8)).cuda()
    ct = torch.zeros(nrec * (L + 16), dtype=torch.uint8, device="cuda")
    back = torch.zeros_like(pt)
    st = torch.ones(nrec, dtype=torch.uint8, device="cuda")
    noise_amd.encrypt_sessions(k1, n, idx, nonces, pt, L, ct, L + 16, L, nrec)
    noise_amd.decrypt_sessions(k1r, n, idx, nonces, ct, L + 16, back, L, L, st, nrec)
    torch.cuda.synchronize()
    assert int(st.sum()) == 0 and torch.equal(pt, back)
    k1h, pth, cth = k1.cpu().numpy(), pt.cpu().numpy(), ct.cpu().numpy()
    for r in list(range(0, nrec, 97)) + [nrec - 1]:
        s, nn = r % n, r // n
        want = oracle.encrypt(k1h[32 * s:32 * s + 32].tobytes(), nn, b"",
                              pth[r * L:(r + 1) * L].tobytes())
        assert cth[r * (L + 16):(r + 1) * (L + 16)].tobytes() == want, r


def test_batch_message_length_checks():
    """Per-session message lengths: a message shorter than the token bytes (or
    > 65535) fails exactly its session with HS_BAD_LEN; the others proceed."""
    n = 256
    I, R = noise_amd.HandshakeBatch("NN", True, n), noise_amd.HandshakeBatch("NN", False, n)
    I.start()
    R.start()
    buf = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    I.write_message(noise_amd.span(buf, stride=64), d_msg_len=lens)
    torch.cuda.synchronize()
    assert int(lens.min()) == 32 == int(lens.max())
    lens[5], lens[77], lens[200] = 31, 0, 70000
    pay = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    plen = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    R.read_message(noise_amd.span(buf, stride=64, lens=lens), noise_amd.span(pay, stride=64),
                   d_payload_len=plen, d_status=st)
    torch.cuda.synchronize()
    bad = {5, 77, 200}
    s = st.cpu().numpy()
    assert all(s[i] == noise_amd.HS_BAD_LEN for i in bad)
    assert all(s[i] == 0 for i in range(n) if i not in bad)
    I.close()
    R.close()


def test_batch_write_payload_length_checks():
    """write_message: a message (token bytes + payload + tag) must fit 65535
    bytes (noise.cpp:886).  A uniform payload length that does not is refused
    on the host; per-session lengths fail exactly their sessions with
    HS_BAD_LEN on the device before any byte of them is written."""
    n = 64
    E = noise_amd.NoiseGpuError
    I = noise_amd.HandshakeBatch("NN", True, n)
    I.start()
    ov = I.info().overhead  # "e" = 32 bytes, no key yet: no tag
    assert ov == 32
    stride = 65536 + 64
    buf = torch.full((n * stride,), 0xAB, dtype=torch.uint8, device="cuda")
    pay = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    with pytest.raises(E):  # uniform: 65535 - 32 + 1 bytes of payload
        I.write_message(noise_amd.span(buf, stride=stride), noise_amd.span(pay, stride=stride,
                                                                           length=65535 - ov + 1))
    plen = torch.full((n,), 10, dtype=torch.int32, device="cuda")
    plen[3], plen[40] = 65535 - ov + 1, 0x7fffffff
    plen[41] = 65535 - ov  # the largest payload that fits
    mlen = torch.zeros(n, dtype=torch.int32, device="cuda")
    I.write_message(noise_amd.span(buf, stride=stride),
                    noise_amd.span(pay, stride=stride, lens=plen), d_msg_len=mlen)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    I.status(st)
    torch.cuda.synchronize()
    s, m = st.cpu().numpy(), mlen.cpu().numpy()
    for i in range(n):
        if i in (3, 40):
            assert s[i] == noise_amd.HS_BAD_LEN, i
            row = buf[i * stride:(i + 1) * stride]
            assert bool((row == 0xAB).all()), ("failed session's message was written", i)
        else:
            assert s[i] == 0, i
            assert m[i] == ov + (65535 - ov if i == 41 else 10), i
    I.close()


def test_batch_api_rules_and_shared_static_key():
    """Host-side rules of the batched API (turn order, keys before start, psk
    count, finished/split order) and a stride-0 static key (one server key for
    every session, derived once and broadcast) giving the same handshakes as
    the same key installed per session."""
    n = 130
    E = noise_amd.NoiseGpuError
    rng = np.random.default_rng(3)
    srv = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    cli = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(n)]
    eph = [[bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(n)] for _ in range(2)]
    results = []
    for shared in (True, False):
        I, R = noise_amd.HandshakeBatch("XX", True, n), noise_amd.HandshakeBatch("XX", False, n)
        I.set_key(noise_amd.HS_S, _dev(b"".join(cli)))
        I.set_key(noise_amd.HS_E, _dev(b"".join(eph[0])))
        if shared:
            R.set_key(noise_amd.HS_S, _dev(srv), stride=0)
        else:
            R.set_key(noise_amd.HS_S, _dev(srv * n))
        R.set_key(noise_amd.HS_E, _dev(b"".join(eph[1])))
        buf = torch.zeros(n * 128, dtype=torch.uint8, device="cuda")
        with pytest.raises(E):  # not started
            I.write_message(noise_amd.span(buf, stride=128))
        I.start()
        R.start()
        with pytest.raises(E):  # keys go in before start
            I.set_key(noise_amd.HS_S, _dev(b"".join(cli)))
        with pytest.raises(E):  # the responder reads first
            R.write_message(noise_amd.span(buf, stride=128))
        with pytest.raises(E):  # not finished
            I.split(*(torch.zeros(32 * n, dtype=torch.uint8, device="cuda") for _ in range(2)))
        msgs = []
        for m in range(3):
            w, r = (I, R) if m % 2 == 0 else (R, I)
            ov = w.info().overhead
            w.write_message(noise_amd.span(buf, stride=128))
            r.read_message(noise_amd.span(buf, stride=128, length=ov))
            msgs.append(buf.view(n, 128)[:, :ov].cpu().numpy().copy())
        assert I.info().finished == 1 and R.info().my_turn == 0
        with pytest.raises(E):  # finished
            I.write_message(noise_amd.span(buf, stride=128))
        k = [torch.zeros(32 * n, dtype=torch.uint8, device="cuda") for _ in range(4)]
        I.split(k[0], k[1])
        R.split(k[2], k[3])
        torch.cuda.synchronize()
        assert torch.equal(k[0], k[2]) and torch.equal(k[1], k[3])
        results.append((msgs, k[0].cpu().numpy()))
        I.close()
        R.close()
    for a, b in zip(results[0][0], results[1][0]):
        assert np.array_equal(a, b)
    assert np.array_equal(results[0][1], results[1][1])
    with pytest.raises(E):  # psk pattern without psks
        P = noise_amd.HandshakeBatch("NNpsk0", True, 4)
        P.start()
