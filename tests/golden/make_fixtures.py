#!/usr/bin/env python3
"""Generate the golden ChaChaPoly record fixtures from the reference's vectors.

Runs ONLY in the build container (it reads /root/reference/tests/vectors,
which does not exist on the GPU box).  Its outputs are committed next to it:

  transport_records.tsv   every post-handshake transport message of every
                          ChaChaPoly vector whose handshake this harness
                          reproduces (k, n, ad = empty, pt, ct||tag)
  handshake_records.tsv   every keyed EncryptAndHash inside those handshakes
                          (k, n, ad = h, pt, ct||tag): the with-AD path of
                          SymmetricState::encrypt_and_hash (noise.cpp:498-504)
  summary.json            counts + which vectors passed

How the tuples are derived.  The vectors (tests/vectors/*.json, fetched by the
reference's dump_tests.py from cacophony/snow) give private keys, prologue,
psks and the exact wire bytes of each message.  The transport keys are not in
the files, so this script replays both sides of each handshake with its own,
independent implementation of the Noise framework (rev 34): X25519/X448 per
RFC 7748, hashlib SHA-256/512 and BLAKE2s/b, HMAC-HKDF, ChaCha20-Poly1305 per
RFC 8439 with the Noise nonce 0^32 || LE64(n).  Every handshake message it
writes must equal the vector's ciphertext byte for byte, and the final
handshake hash must equal `handshake_hash`; only then are the records kept.
So each tuple is pinned by the reference's own golden data, not by this
script's AEAD.

The pattern table below is restated from the Noise specification; the
reference holds the same table at noise.cpp:594-818.
"""
import glob
import hashlib
import hmac
import json
import os
import struct
import sys

VEC_DIR = "/root/reference/tests/vectors"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))

# ----------------------------------------------------------------- X25519/X448
P25519 = 2**255 - 19
P448 = 2**448 - 2**224 - 1


def _ladder(k, u, p, bits, a24):
    x1, x2, z2, x3, z3, swap = u, 1, 0, u, 1, 0
    for t in reversed(range(bits)):
        kt = (k >> t) & 1
        swap ^= kt
        if swap:
            x2, x3, z2, z3 = x3, x2, z3, z2
        swap = kt
        A = (x2 + z2) % p; AA = A * A % p
        B = (x2 - z2) % p; BB = B * B % p
        E = (AA - BB) % p
        C = (x3 + z3) % p; D = (x3 - z3) % p
        DA = D * A % p; CB = C * B % p
        x3 = (DA + CB) ** 2 % p
        z3 = x1 * (DA - CB) ** 2 % p
        x2 = AA * BB % p
        z2 = E * (AA + a24 * E) % p
    if swap:
        x2, z2 = x3, z3
    return x2 * pow(z2, p - 2, p) % p


def x25519(sk, pk):
    k = bytearray(sk); k[0] &= 248; k[31] &= 127; k[31] |= 64
    u = int.from_bytes(pk, "little") & ((1 << 255) - 1)
    r = _ladder(int.from_bytes(k, "little"), u, P25519, 255, 121665)
    return r.to_bytes(32, "little")


def x448(sk, pk):
    k = bytearray(sk); k[0] &= 252; k[55] |= 128
    u = int.from_bytes(pk, "little")
    r = _ladder(int.from_bytes(k, "little"), u, P448, 448, 39081)
    return r.to_bytes(56, "little")


DH = {
    "25519": (32, x25519, (9).to_bytes(32, "little")),
    "448": (56, x448, (5).to_bytes(56, "little")),
}

# ---------------------------------------------------------- ChaCha20-Poly1305
M32 = 0xFFFFFFFF


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & M32


def chacha20_block(key, counter, nonce12):
    s = list(struct.unpack("<4I", b"expand 32-byte k")) + list(
        struct.unpack("<8I", key)) + [counter & M32] + list(
        struct.unpack("<3I", nonce12))
    x = s[:]

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 7)
    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return struct.pack("<16I", *[(x[i] + s[i]) & M32 for i in range(16)])


def poly1305(key32, msg):
    r = int.from_bytes(key32[:16], "little") & 0x0ffffffc0ffffffc0ffffffc0fffffff
    s = int.from_bytes(key32[16:], "little")
    p = (1 << 130) - 5
    h = 0
    for i in range(0, len(msg), 16):
        blk = msg[i:i + 16]
        h = (h + int.from_bytes(blk + b"\x01", "little")) * r % p
    return ((h + s) & ((1 << 128) - 1)).to_bytes(16, "little")


def _pad16(b):
    return b"\x00" * (-len(b) % 16)


def noise_nonce(n):
    return b"\x00" * 4 + struct.pack("<Q", n)


def aead_encrypt(k, n, ad, pt):
    nonce = noise_nonce(n)
    otk = chacha20_block(k, 0, nonce)[:32]
    ks = b"".join(chacha20_block(k, 1 + i, nonce) for i in range((len(pt) + 63) // 64))
    ct = bytes(a ^ b for a, b in zip(pt, ks))
    mac_data = ad + _pad16(ad) + ct + _pad16(ct) + struct.pack("<QQ", len(ad), len(ct))
    return ct + poly1305(otk, mac_data)


def aead_decrypt(k, n, ad, ct_tag):
    ct, tag = ct_tag[:-16], ct_tag[-16:]
    nonce = noise_nonce(n)
    otk = chacha20_block(k, 0, nonce)[:32]
    mac_data = ad + _pad16(ad) + ct + _pad16(ct) + struct.pack("<QQ", len(ad), len(ct))
    if not hmac.compare_digest(poly1305(otk, mac_data), tag):
        raise ValueError("Invalid MAC")
    ks = b"".join(chacha20_block(k, 1 + i, nonce) for i in range((len(ct) + 63) // 64))
    return bytes(a ^ b for a, b in zip(ct, ks))


# ------------------------------------------------------------- Noise framework
HASHES = {
    "SHA256": (hashlib.sha256, 32),
    "SHA512": (hashlib.sha512, 64),
    "BLAKE2s": (hashlib.blake2s, 32),
    "BLAKE2b": (hashlib.blake2b, 64),
}

# Noise rev34 pattern table: (pre-messages initiator, responder), messages.
PATTERNS = {
    "N": ([], ["s"], [["e", "es"]]),
    "K": (["s"], ["s"], [["e", "es", "ss"]]),
    "X": ([], ["s"], [["e", "es", "s", "ss"]]),
    "NN": ([], [], [["e"], ["e", "ee"]]),
    "NK": ([], ["s"], [["e", "es"], ["e", "ee"]]),
    "NX": ([], [], [["e"], ["e", "ee", "s", "es"]]),
    "KN": (["s"], [], [["e"], ["e", "ee", "se"]]),
    "KK": (["s"], ["s"], [["e", "es", "ss"], ["e", "ee", "se"]]),
    "KX": (["s"], [], [["e"], ["e", "ee", "se", "s", "es"]]),
    "XN": ([], [], [["e"], ["e", "ee"], ["s", "se"]]),
    "XK": ([], ["s"], [["e", "es"], ["e", "ee"], ["s", "se"]]),
    "XX": ([], [], [["e"], ["e", "ee", "s", "es"], ["s", "se"]]),
    "IN": ([], [], [["e", "s"], ["e", "ee", "se"]]),
    "IK": ([], ["s"], [["e", "es", "s", "ss"], ["e", "ee", "se"]]),
    "IX": ([], [], [["e", "s"], ["e", "ee", "se", "s", "es"]]),
    "NK1": ([], ["s"], [["e"], ["e", "ee", "es"]]),
    "NX1": ([], [], [["e"], ["e", "ee", "s"], ["es"]]),
    "X1N": ([], [], [["e"], ["e", "ee"], ["s"], ["se"]]),
    "X1K": ([], ["s"], [["e", "es"], ["e", "ee"], ["s"], ["se"]]),
    "XK1": ([], ["s"], [["e"], ["e", "ee", "es"], ["s", "se"]]),
    "X1K1": ([], ["s"], [["e"], ["e", "ee", "es"], ["s"], ["se"]]),
    "X1X": ([], [], [["e"], ["e", "ee", "s", "es"], ["s"], ["se"]]),
    "XX1": ([], [], [["e"], ["e", "ee", "s"], ["es", "s", "se"]]),
    "X1X1": ([], [], [["e"], ["e", "ee", "s"], ["es", "s"], ["se"]]),
    "K1N": (["s"], [], [["e"], ["e", "ee"], ["se"]]),
    "K1K": (["s"], ["s"], [["e", "es"], ["e", "ee"], ["se"]]),
    "KK1": (["s"], ["s"], [["e"], ["e", "ee", "se", "es"]]),
    "K1K1": (["s"], ["s"], [["e"], ["e", "ee", "es"], ["se"]]),
    "K1X": (["s"], [], [["e"], ["e", "ee", "s", "es"], ["se"]]),
    "KX1": (["s"], [], [["e"], ["e", "ee", "se", "s"], ["es"]]),
    "K1X1": (["s"], [], [["e"], ["e", "ee", "s"], ["se", "es"]]),
    "I1N": ([], [], [["e", "s"], ["e", "ee"], ["se"]]),
    "I1K": ([], ["s"], [["e", "es", "s"], ["e", "ee"], ["se"]]),
    "IK1": ([], ["s"], [["e", "s"], ["e", "ee", "se", "es"]]),
    "I1K1": ([], ["s"], [["e", "s"], ["e", "ee", "es"], ["se"]]),
    "I1X": ([], [], [["e", "s"], ["e", "ee", "s", "es"], ["se"]]),
    "IX1": ([], [], [["e", "s"], ["e", "ee", "se", "s"], ["es"]]),
    "I1X1": ([], [], [["e", "s"], ["e", "ee", "s"], ["se", "es"]]),
}


def parse_pattern(name):
    """'XXpsk0+psk2' -> (base pattern, [0, 2])."""
    if "psk" not in name:
        return name, []
    base, mods = name.split("psk", 1)
    return base, [int(m.replace("psk", "")) for m in mods.split("+")]


class CipherState:
    def __init__(self):
        self.k = None
        self.n = 0
        self.log = None  # list collecting (k, n, ad, pt, ct) tuples

    def encrypt_with_ad(self, ad, pt):
        if self.k is None:
            return pt
        ct = aead_encrypt(self.k, self.n, ad, pt)
        if self.log is not None:
            self.log.append((self.k, self.n, ad, pt, ct))
        self.n += 1
        return ct

    def decrypt_with_ad(self, ad, ct):
        if self.k is None:
            return ct
        pt = aead_decrypt(self.k, self.n, ad, ct)
        self.n += 1
        return pt


class SymmetricState:
    def __init__(self, name, hashname):
        self.H, self.HLEN = HASHES[hashname]
        nb = name.encode()
        self.h = nb + b"\x00" * (self.HLEN - len(nb)) if len(nb) <= self.HLEN else self.hash(nb)
        self.ck = self.h
        self.cs = CipherState()

    def hash(self, data):
        return self.H(data).digest()

    def hkdf(self, ikm, n):
        tk = hmac.new(self.ck, ikm, self.H).digest()
        o1 = hmac.new(tk, b"\x01", self.H).digest()
        o2 = hmac.new(tk, o1 + b"\x02", self.H).digest()
        if n == 2:
            return o1, o2
        return o1, o2, hmac.new(tk, o2 + b"\x03", self.H).digest()

    def mix_key(self, ikm):
        self.ck, tk = self.hkdf(ikm, 2)
        self.cs.k, self.cs.n = tk[:32], 0

    def mix_hash(self, data):
        self.h = self.hash(self.h + data)

    def mix_key_and_hash(self, ikm):
        self.ck, th, tk = self.hkdf(ikm, 3)
        self.mix_hash(th)
        self.cs.k, self.cs.n = tk[:32], 0

    def encrypt_and_hash(self, pt):
        ct = self.cs.encrypt_with_ad(self.h, pt)
        self.mix_hash(ct)
        return ct

    def decrypt_and_hash(self, ct):
        pt = self.cs.decrypt_with_ad(self.h, ct)
        self.mix_hash(ct)
        return pt

    def split(self):
        k1, k2 = self.hkdf(b"", 2)
        c1, c2 = CipherState(), CipherState()
        c1.k, c2.k = k1[:32], k2[:32]
        return c1, c2


class Party:
    def __init__(self, vec, initiator, log):
        proto = vec["protocol_name"]
        _, pattern, dhname, cipher, hashname = proto.split("_")
        assert cipher == "ChaChaPoly"
        base, psk_idx = parse_pattern(pattern)
        pre_i, pre_r, msgs = PATTERNS[base]
        msgs = [list(m) for m in msgs]
        for i in psk_idx:
            if i == 0:
                msgs[0].insert(0, "psk")
            else:
                msgs[i - 1].append("psk")
        self.msgs = msgs
        self.dhlen, self.dh, base_pt = DH[dhname]
        self.initiator = initiator
        self.psk_mode = bool(psk_idx)
        pre = "init_" if initiator else "resp_"
        self.ss = SymmetricState(proto, hashname)
        self.ss.cs.log = log
        self.ss.mix_hash(bytes.fromhex(vec[pre + "prologue"]))
        self.psks = [bytes.fromhex(p) for p in vec.get(pre + "psks", [])]

        def kp(field):
            if field not in vec:
                return None
            sk = bytes.fromhex(vec[field])
            return sk, self.dh(sk, base_pt)
        self.s = kp(pre + "static")
        self.e = kp(pre + "ephemeral")
        self.rs = bytes.fromhex(vec[pre + "remote_static"]) if pre + "remote_static" in vec else None
        self.re = None
        # Pre-messages: initiator's first, then responder's (spec 5.3).
        for who, toks in (("i", pre_i), ("r", pre_r)):
            for t in toks:
                assert t == "s"
                mine = (who == "i") == initiator
                self.ss.mix_hash(self.s[1] if mine else self.rs)

    def _dh_token(self, t):
        if t == "ee":
            return self.dh(self.e[0], self.re)
        if t == "ss":
            return self.dh(self.s[0], self.rs)
        if t == "es":
            return self.dh(self.e[0], self.rs) if self.initiator else self.dh(self.s[0], self.re)
        if t == "se":
            return self.dh(self.s[0], self.re) if self.initiator else self.dh(self.e[0], self.rs)
        raise KeyError(t)

    def write(self, idx, payload):
        out = b""
        for t in self.msgs[idx]:
            if t == "e":
                out += self.e[1]
                self.ss.mix_hash(self.e[1])
                if self.psk_mode:
                    self.ss.mix_key(self.e[1])
            elif t == "s":
                out += self.ss.encrypt_and_hash(self.s[1])
            elif t == "psk":
                self.ss.mix_key_and_hash(self.psks.pop(0))
            else:
                self.ss.mix_key(self._dh_token(t))
        return out + self.ss.encrypt_and_hash(payload)

    def read(self, idx, msg):
        for t in self.msgs[idx]:
            if t == "e":
                self.re, msg = msg[:self.dhlen], msg[self.dhlen:]
                self.ss.mix_hash(self.re)
                if self.psk_mode:
                    self.ss.mix_key(self.re)
            elif t == "s":
                n = self.dhlen + (16 if self.ss.cs.k is not None else 0)
                self.rs = self.ss.decrypt_and_hash(msg[:n])
                msg = msg[n:]
            elif t == "psk":
                self.ss.mix_key_and_hash(self.psks.pop(0))
            else:
                self.ss.mix_key(self._dh_token(t))
        return self.ss.decrypt_and_hash(msg)


def run_vector(vec, hs_log):
    """Replay one vector. Returns the list of transport tuples, or raises."""
    ini, res = Party(vec, True, hs_log), Party(vec, False, None)
    nhs = len(ini.msgs)
    # one-way patterns: every transport message goes initiator -> responder
    one_way = parse_pattern(vec["protocol_name"].split("_")[1])[0] in ("N", "K", "X")
    msgs = vec["messages"]
    transport = []
    i_send = i_recv = r_send = r_recv = None
    for m, msg in enumerate(msgs):
        payload, expect = bytes.fromhex(msg["payload"]), bytes.fromhex(msg["ciphertext"])
        init_sends = True if one_way else (m % 2 == 0)
        if m < nhs:
            w, r = (ini, res) if init_sends else (res, ini)
            # the responder's own handshake AEAD calls are logged too
            w.ss.cs.log = hs_log
            wire = w.write(m, payload)
            if wire != expect:
                raise AssertionError("handshake message %d mismatch" % m)
            if r.read(m, wire) != payload:
                raise AssertionError("handshake payload %d mismatch" % m)
            if m == nhs - 1:
                if ini.ss.h != res.ss.h:
                    raise AssertionError("handshake hash differs between parties")
                if "handshake_hash" in vec and ini.ss.h.hex() != vec["handshake_hash"]:
                    raise AssertionError("handshake_hash mismatch")
                i_send, i_recv = ini.ss.split()
                r_recv, r_send = res.ss.split()
        else:
            snd, rcv = (i_send, r_recv) if init_sends else (r_send, i_recv)
            n = snd.n
            ct = snd.encrypt_with_ad(b"", payload)
            if ct != expect:
                raise AssertionError("transport message %d mismatch" % m)
            if rcv.decrypt_with_ad(b"", ct) != payload:
                raise AssertionError("transport decrypt %d mismatch" % m)
            transport.append(("i2r" if init_sends else "r2i", snd.k, n, payload, ct))
    return transport


def main():
    files = sorted(glob.glob(os.path.join(VEC_DIR, "*_ChaChaPoly_*.json")))
    if not files:
        sys.exit("no vectors under %s (this script runs only in the build container)" % VEC_DIR)
    tr_rows, hs_rows, passed, failed = [], [], [], []
    for f in files:
        vec = json.load(open(f))
        hs_log = []
        try:
            recs = run_vector(vec, hs_log)
        except Exception as e:  # noqa: BLE001 - report, keep going
            failed.append((os.path.basename(f), repr(e)))
            continue
        passed.append(os.path.basename(f))
        name = os.path.basename(f)[:-5]
        for d, k, n, pt, ct in recs:
            tr_rows.append("\t".join([name, d, k.hex(), str(n), pt.hex(), ct.hex()]))
        for k, n, ad, pt, ct in hs_log:
            hs_rows.append("\t".join([name, k.hex(), str(n), ad.hex(), pt.hex(), ct.hex()]))
    with open(os.path.join(OUT_DIR, "transport_records.tsv"), "w") as fh:
        fh.write("# vector\tdir\tkey\tnonce\tplaintext\tciphertext_and_tag\n")
        fh.write("\n".join(tr_rows) + "\n")
    with open(os.path.join(OUT_DIR, "handshake_records.tsv"), "w") as fh:
        fh.write("# vector\tkey\tnonce\tad\tplaintext\tciphertext_and_tag\n")
        fh.write("\n".join(hs_rows) + "\n")
    summary = {"vectors": len(files), "passed": len(passed), "failed": failed,
               "transport_records": len(tr_rows), "handshake_records": len(hs_rows)}
    json.dump(summary, open(os.path.join(OUT_DIR, "summary.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "failed"}), "failed:", len(failed))
    for f, e in failed[:10]:
        print("  FAIL", f, e)


if __name__ == "__main__":
    main()
