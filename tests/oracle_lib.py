"""Test-side loaders for the CPU oracle (oracle/liboracle.so), the reference
build (oracle/_ref/libnoise_ref.so) and the golden fixtures (tests/golden/).
Test infrastructure only: the product never imports this."""
import ctypes
import os
import subprocess

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libnoise_ref.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

KAT_K5 = {  # SURVEY.md section 8(c), computed by the reference noise::encrypt
    0: ("1bb25329b2c08be528231531f81d2b4b", "27f85b7f1d11a630ed12ef4d67284e87",
        "fed6b0f4a7c72df81c716d2185ac83ccf78e7e092ae2c4c2f34ca34d801b5481"),
    1: ("9c5de247aa0c822c12f4e70c05cbfceb", "7c8286b62e877a84385fc03829070e26",
        "c6421d28addb68b30ca7b4cfa15132333e973d27e0c1b4c9eb276f48e092ac49"),
    (1 << 64) - 3: ("d28dd4f83a2703ee6d77f38ad5970525", "69ed2ebdfbf1ada97cead15a927d8755",
                    "718bdb56c2c8f02c83d45677ccdfdcbbcfd36e815166af3271dd608e87e5bf3c"),
}
KAT_K4_REKEY_ZERO = "765f5f43857ccfe16f686cb1f02213efb5cad57191351e67b517961142410e93"
KAT_K1 = ("c3afbe61fd5761493bc55a143def98f3c8e12991c8371b0916351bc841727f89", 0, "",
          "4361726c204d656e676572", "fc56eea290b3f3a21aac0c70cd5787b5ee99be37d2f4d751329b55")
KAT_K2 = ("c3afbe61fd5761493bc55a143def98f3c8e12991c8371b0916351bc841727f89", 1, "",
          "457567656e2042f6686d20766f6e2042617765726b",
          "f6199cadb152fb27f82be0a0891ec76a33598ae92a46cab2fb5a8ed5bf48b7f267f8370af7")
KAT_K3 = ("95ce3f98e4774a5eaa1d72a5d8e48864cf266975f8c7820243c8ebb191587fed", 0,
          "dd4d2c6fbfb50025ad792426d0ec2be49c073de8eb106b6e167008e40fdcec8c40897fb47cc8a28b4d95a4"
          "d69904936490fdc2f72fb95612ea08069b2c896ceb",
          "4d757272617920526f746862617264",
          "b42e5b7b74e0e678c4c18ee4543759d015d50f1fe63ee187ff55deb17b6ea7")


def k5_plaintext():
    return bytes((7 * j + 3) % 256 for j in range(1024))


def check_threads():
    """Checker threads: the CPUs this process may run on, at most 16 (a GPU
    box's CPU share; os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)


class Oracle:
    def __init__(self):
        if not os.path.exists(ORACLE_SO):
            _build()
        self.lib = ctypes.CDLL(ORACLE_SO)
        L = self.lib
        L.oracle_noise_encrypt.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                           ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.c_void_p]
        L.oracle_noise_decrypt.argtypes = L.oracle_noise_encrypt.argtypes
        L.oracle_noise_decrypt.restype = ctypes.c_int
        L.oracle_rekey.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
        L.oracle_fill_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_uint64]
        L.oracle_batch_uniform.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_void_p]
        L.oracle_batch_uniform.restype = ctypes.c_double
        L.oracle_batch_records.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.oracle_batch_records.restype = ctypes.c_double
        L.oracle_check_records.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int64)]
        L.oracle_check_records.restype = ctypes.c_int64
        L.oracle_check_uniform.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int64)]
        L.oracle_check_uniform.restype = ctypes.c_int64
        self.ref = None
        if os.path.exists(REF_SO):
            R = ctypes.CDLL(REF_SO)
            R.ref_noise_encrypt.argtypes = L.oracle_noise_encrypt.argtypes
            R.ref_noise_decrypt.argtypes = L.oracle_noise_encrypt.argtypes
            R.ref_noise_decrypt.restype = ctypes.c_int
            R.ref_batch_uniform.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            R.ref_batch_uniform.restype = ctypes.c_double
            R.ref_batch_records.argtypes = L.oracle_batch_records.argtypes
            R.ref_batch_records.restype = ctypes.c_double
            R.ref_xx_handshake.argtypes = [ctypes.c_char_p] * 4 + [ctypes.c_void_p] * 4
            R.ref_xx_handshake.restype = ctypes.c_int
            R.ref_xx_bench.argtypes = [ctypes.c_long, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            R.ref_xx_bench.restype = ctypes.c_double
            self.ref = R

    def ref_xx_handshake(self, si, ei, sr, er):
        """Both parties of Noise_XX_25519_ChaChaPoly_BLAKE2b on the reference's
        Monocypher primitives (oracle/ref_harness.c), empty prologue and
        payloads: (msg1, msg2, msg3, handshake_hash, k1, k2)."""
        msgs, h = ctypes.create_string_buffer(192), ctypes.create_string_buffer(64)
        k1, k2 = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        assert self.ref.ref_xx_handshake(si, ei, sr, er, msgs, h, k1, k2) == 0
        m = msgs.raw
        return m[:32], m[32:128], m[128:192], h.raw, k1.raw, k2.raw

    def encrypt(self, key, n, ad, pt, lib=None):
        lib = lib or self.lib
        out = ctypes.create_string_buffer(len(pt) + 16)
        fn = lib.oracle_noise_encrypt if lib is self.lib else lib.ref_noise_encrypt
        fn(bytes(key), n % (1 << 64), bytes(ad), len(ad), bytes(pt), len(pt), out)
        return out.raw

    def decrypt(self, key, n, ad, ct, lib=None):
        lib = lib or self.lib
        out = ctypes.create_string_buffer(max(len(ct), 1))
        fn = lib.oracle_noise_decrypt if lib is self.lib else lib.ref_noise_decrypt
        rc = fn(bytes(key), n % (1 << 64), bytes(ad), len(ad), bytes(ct), len(ct), out)
        return None if rc else out.raw[:len(ct) - 16]

    def rekey(self, key):
        out = ctypes.create_string_buffer(32)
        self.lib.oracle_rekey(bytes(key), out)
        return out.raw

    def synthetic(self, nbytes, seed, offset=0):
        out = ctypes.create_string_buffer(max(nbytes, 1))
        self.lib.oracle_fill_synthetic(out, offset, nbytes, seed)
        return out.raw[:nbytes]

    def check_records(self, decrypt, keys, nkeys, recs, inb, outb, ad=None, status=None,
                      in_base=0, out_base=0, threads=None):
        """Whole-batch parity: every descriptor of `recs` (numpy noise_gpu_record
        array) recomputed and compared.  keys/inb/outb/ad/status are numpy uint8
        arrays (C-contiguous).  Returns (mismatching records, first mismatching
        index or -1)."""
        first = ctypes.c_int64(-1)

        def ptr(a):
            if a is None:
                return None
            assert a.flags["C_CONTIGUOUS"]
            return a.ctypes.data
        bad = self.lib.oracle_check_records(int(decrypt), ptr(keys), nkeys, ptr(recs), len(recs),
                                            in_base, ptr(inb), out_base, ptr(outb), ptr(ad),
                                            ptr(status), threads or check_threads(),
                                            ctypes.byref(first))
        return int(bad), first.value

    def check_uniform(self, decrypt, key, n0, inb, in_stride, outb, out_stride, length, nrec,
                      status=None, threads=None):
        """Whole-batch parity of a uniform batch (record i: nonce n0 + i)."""
        first = ctypes.c_int64(-1)
        bad = self.lib.oracle_check_uniform(int(decrypt), bytes(key), n0 % (1 << 64),
                                            inb.ctypes.data, in_stride, outb.ctypes.data,
                                            out_stride, length, nrec,
                                            None if status is None else status.ctypes.data,
                                            threads or check_threads(), ctypes.byref(first))
        return int(bad), first.value

    def encrypt_uniform_np(self, key, n0, pt, length, in_stride, out_stride, nrec, threads=8):
        """Uniform batch on numpy buffers (parity tests at moderate sizes)."""
        import numpy as np
        out = np.zeros(out_stride * (nrec - 1) + length + 16, dtype=np.uint8)
        self.lib.oracle_batch_uniform(0, bytes(key), n0, pt.ctypes.data, in_stride, out.ctypes.data,
                                      out_stride, length, nrec, threads, None)
        return out


def load_golden():
    def tsv(name):
        rows = []
        for line in open(os.path.join(GOLDEN, name)):
            if not line.startswith("#") and line.strip():
                rows.append(line.rstrip("\n").split("\t"))
        return rows
    transport = [dict(vector=r[0], dir=r[1], key=bytes.fromhex(r[2]), nonce=int(r[3]), ad=b"",
                      pt=bytes.fromhex(r[4]), ct=bytes.fromhex(r[5]))
                 for r in tsv("transport_records.tsv")]
    handshake = [dict(vector=r[0], key=bytes.fromhex(r[1]), nonce=int(r[2]), ad=bytes.fromhex(r[3]),
                      pt=bytes.fromhex(r[4]), ct=bytes.fromhex(r[5]))
                 for r in tsv("handshake_records.tsv")]
    return {"transport": transport, "handshake": handshake}
