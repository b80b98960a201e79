"""ctypes binding of the MI355X Noise ChaChaPoly engine (include/noise_gpu.h).

The product is the C ABI in noise-cpp_amd/lib/libnoise_amd.so (HIP kernels for
gfx950) and the C++20 noise::CipherState over it.  This module is the thin
Python view used by tests/, bench.py and __graft_entry__.py: it passes device
pointers (torch tensors on the GPU are used only as HBM allocations) and
streams straight through to the C ABI.  There is no Python or CPU compute
path: if the shared library is missing, load() raises.
"""
import ctypes
import os
import re

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
PKG = os.path.join(ROOT, "noise-cpp_amd")
# NOISE_AMD_LIB: load another build of the library (A/B tuning runs only)
LIB_PATH = os.environ.get("NOISE_AMD_LIB") or os.path.join(PKG, "lib", "libnoise_amd.so")
HEADER = os.path.join(ROOT, "include", "noise_gpu.h")

OK, E_NONCE, E_MAC, E_ARG, E_HIP, E_NODEV = 0, 1, 2, 3, 4, 5
REC_OK, REC_BAD_MAC, REC_BAD_KEY = 0, 1, 2
NONCE_LIMIT = (1 << 64) - 2  # noise.cpp:398 refuses n == 2^64-2


class Record(ctypes.Structure):
    """noise_gpu_record (include/noise_gpu.h)."""
    _fields_ = [("in_off", ctypes.c_uint64), ("out_off", ctypes.c_uint64),
                ("nonce", ctypes.c_uint64), ("ad_off", ctypes.c_uint64),
                ("len", ctypes.c_uint32), ("ad_len", ctypes.c_uint32),
                ("key_idx", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


RECORD_DTYPE = None  # numpy structured dtype, built lazily


def record_dtype():
    global RECORD_DTYPE
    if RECORD_DTYPE is None:
        import numpy as np
        RECORD_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"),
                                 ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4"),
                                 ("key_idx", "<u4"), ("reserved", "<u4")])
        assert RECORD_DTYPE.itemsize == ctypes.sizeof(Record) == 48
    return RECORD_DTYPE


class Span(ctypes.Structure):
    """noise_gpu_span (include/noise_gpu.h): per-session byte ranges."""
    _fields_ = [("base", ctypes.c_void_p), ("off", ctypes.c_void_p), ("stride", ctypes.c_uint64),
                ("len", ctypes.c_void_p), ("len_all", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class HsInfo(ctypes.Structure):
    """noise_gpu_hs_info (include/noise_gpu.h)."""
    _fields_ = [("message_index", ctypes.c_uint32), ("message_count", ctypes.c_uint32),
                ("my_turn", ctypes.c_int32), ("finished", ctypes.c_int32),
                ("overhead", ctypes.c_uint32), ("psk_count", ctypes.c_uint32)]


HS_S, HS_E, HS_RS, HS_RE = 0, 1, 2, 3
HS_OK, HS_BAD_MAC, HS_BAD_LEN = 0, 1, 3


class NoiseGpuError(RuntimeError):
    def __init__(self, code, what):
        super().__init__("%s (status %d): %s" % (what, code, _lib.noise_gpu_last_error().decode()
                                                if _lib else ""))
        self.code = code


_lib = None
u8p, u64, u32, vp = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p


def declared_symbols():
    """Function names declared in include/noise_gpu.h."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char \*)\s*(noise_gpu_\w+)\s*\(", text, re.M)))


def load(path=LIB_PATH):
    """Load the engine library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError("libnoise_amd.so not built (%s); run __graft_entry__.build()" % path)
    lib = ctypes.CDLL(path)
    sig = {
        "noise_gpu_version": (ctypes.c_char_p, []),
        "noise_gpu_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "noise_gpu_last_error": (ctypes.c_char_p, []),
        "noise_gpu_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "noise_gpu_encrypt_uniform": (ctypes.c_int, [ctypes.c_char_p, u64, u8p, u64, u8p, u64, u32,
                                                     u8p, u64, u32, u64, vp]),
        "noise_gpu_decrypt_uniform": (ctypes.c_int, [ctypes.c_char_p, u64, u8p, u64, u8p, u64, u32,
                                                     u8p, u64, u32, u8p, u64, vp]),
        "noise_gpu_encrypt_records": (ctypes.c_int, [u8p, u32, u8p, u64, u8p, u8p, u8p, vp]),
        "noise_gpu_decrypt_records": (ctypes.c_int, [u8p, u32, u8p, u64, u8p, u8p, u8p, u8p, vp]),
        "noise_gpu_rekey_keys": (ctypes.c_int, [u8p, u64, vp]),
        "noise_gpu_x25519": (ctypes.c_int, [u8p, u8p, u8p, u64, vp]),
        "noise_gpu_encrypt_sessions": (ctypes.c_int, [u8p, u32, u8p, u8p, u8p, u64, u8p, u64, u32,
                                                      u64, vp]),
        "noise_gpu_decrypt_sessions": (ctypes.c_int, [u8p, u32, u8p, u8p, u8p, u64, u8p, u64, u32,
                                                      u8p, u64, vp]),
        "noise_gpu_encrypt_host": (ctypes.c_int, [ctypes.c_char_p, u64, u8p, ctypes.c_size_t,
                                                  u8p, ctypes.c_size_t]),
        "noise_gpu_decrypt_host": (ctypes.c_int, [ctypes.c_char_p, u64, u8p, ctypes.c_size_t,
                                                  u8p, ctypes.c_size_t]),
        "noise_gpu_rekey_host": (ctypes.c_int, [u8p]),
        "noise_gpu_encrypt_records_host": (ctypes.c_int, [u8p, u32, u8p, u64, u8p, u64, u8p, u64,
                                                          u8p, u64]),
        "noise_gpu_decrypt_records_host": (ctypes.c_int, [u8p, u32, u8p, u64, u8p, u64, u8p, u64,
                                                          u8p, u64, u8p]),
        "noise_gpu_encrypt_uniform_host": (ctypes.c_int, [ctypes.c_char_p, u64, u8p, u64, u8p, u64,
                                                          u32, u64, ctypes.POINTER(ctypes.c_double)]),
        "noise_gpu_decrypt_uniform_host": (ctypes.c_int, [ctypes.c_char_p, u64, u8p, u64, u8p, u64,
                                                          u32, u8p, u64,
                                                          ctypes.POINTER(ctypes.c_double)]),
        "noise_gpu_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
        "noise_gpu_ctx_destroy": (ctypes.c_int, [vp]),
        "noise_gpu_ctx_device": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int)]),
        "noise_gpu_ctx_encrypt_host": (ctypes.c_int, [vp, ctypes.c_char_p, u64, u8p, ctypes.c_size_t,
                                                      u8p, ctypes.c_size_t]),
        "noise_gpu_ctx_decrypt_host": (ctypes.c_int, [vp, ctypes.c_char_p, u64, u8p, ctypes.c_size_t,
                                                      u8p, ctypes.c_size_t]),
        "noise_gpu_ctx_rekey_host": (ctypes.c_int, [vp, u8p]),
        "noise_gpu_ctx_encrypt_records_host": (ctypes.c_int, [vp, u8p, u32, u8p, u64, u8p, u64, u8p,
                                                              u64, u8p, u64]),
        "noise_gpu_ctx_decrypt_records_host": (ctypes.c_int, [vp, u8p, u32, u8p, u64, u8p, u64, u8p,
                                                              u64, u8p, u64, u8p]),
        "noise_gpu_ctx_encrypt_uniform_host": (ctypes.c_int, [vp, ctypes.c_char_p, u64, u8p, u64, u8p,
                                                              u64, u32, u64,
                                                              ctypes.POINTER(ctypes.c_double)]),
        "noise_gpu_ctx_decrypt_uniform_host": (ctypes.c_int, [vp, ctypes.c_char_p, u64, u8p, u64, u8p,
                                                              u64, u32, u8p, u64,
                                                              ctypes.POINTER(ctypes.c_double)]),
        "noise_gpu_set_resident": (ctypes.c_int, [ctypes.c_int, u32]),
        "noise_gpu_ctx_set_resident": (ctypes.c_int, [vp, ctypes.c_int, u32]),
        "noise_gpu_thread_release": (ctypes.c_int, []),
        "noise_gpu_fill_synthetic": (ctypes.c_int, [u8p, u64, u64, u64, vp]),
        "noise_gpu_scratch_wipe": (ctypes.c_int, [vp]),
        "noise_gpu_scratch_release": (ctypes.c_int, [vp]),
        "noise_gpu_hs_create": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, u64,
                                               ctypes.POINTER(ctypes.c_void_p)]),
        "noise_gpu_hs_destroy": (ctypes.c_int, [vp]),
        "noise_gpu_hs_info_get": (ctypes.c_int, [vp, ctypes.POINTER(HsInfo)]),
        "noise_gpu_hs_set_key": (ctypes.c_int, [vp, ctypes.c_int, u8p, u64, vp]),
        "noise_gpu_hs_set_psks": (ctypes.c_int, [vp, u8p, vp]),
        "noise_gpu_hs_start": (ctypes.c_int, [vp, ctypes.POINTER(Span), vp]),
        "noise_gpu_hs_write_message": (ctypes.c_int, [vp, ctypes.POINTER(Span), ctypes.POINTER(Span),
                                                      u8p, vp]),
        "noise_gpu_hs_read_message": (ctypes.c_int, [vp, ctypes.POINTER(Span), ctypes.POINTER(Span),
                                                     u8p, u8p, vp]),
        "noise_gpu_hs_status": (ctypes.c_int, [vp, u8p, vp]),
        "noise_gpu_hs_split": (ctypes.c_int, [vp, u8p, u8p, u8p, u8p, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    _lib = lib
    return lib


def _check(rc, what):
    if rc != OK:
        raise NoiseGpuError(rc, what)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _key(key):
    key = bytes(key)
    if len(key) != 32:
        raise ValueError("key must be 32 bytes")
    return key


# ---- device-resident batches (torch uint8 CUDA tensors as HBM buffers) ----
def encrypt_uniform(key, nonce0, d_in, in_stride, d_out, out_stride, length, nrec,
                    d_ad=None, ad_stride=0, ad_len=0, stream=None, in_offset=0, out_offset=0):
    lib = load()
    rc = lib.noise_gpu_encrypt_uniform(_key(key), nonce0 % (1 << 64),
                                       ctypes.c_void_p(d_in.data_ptr() + in_offset), in_stride,
                                       ctypes.c_void_p(d_out.data_ptr() + out_offset), out_stride,
                                       length, _ptr(d_ad), ad_stride, ad_len, nrec, _stream(stream))
    _check(rc, "noise_gpu_encrypt_uniform")


def decrypt_uniform(key, nonce0, d_in, in_stride, d_out, out_stride, length, d_status, nrec,
                    d_ad=None, ad_stride=0, ad_len=0, stream=None, in_offset=0, out_offset=0):
    lib = load()
    rc = lib.noise_gpu_decrypt_uniform(_key(key), nonce0 % (1 << 64),
                                       ctypes.c_void_p(d_in.data_ptr() + in_offset), in_stride,
                                       ctypes.c_void_p(d_out.data_ptr() + out_offset), out_stride,
                                       length, _ptr(d_ad), ad_stride, ad_len, _ptr(d_status), nrec,
                                       _stream(stream))
    _check(rc, "noise_gpu_decrypt_uniform")


def encrypt_records(d_keys, nkeys, d_recs, nrec, d_in, d_out, d_ad=None, stream=None):
    rc = load().noise_gpu_encrypt_records(_ptr(d_keys), nkeys, _ptr(d_recs), nrec, _ptr(d_in),
                                          _ptr(d_out), _ptr(d_ad), _stream(stream))
    _check(rc, "noise_gpu_encrypt_records")


def decrypt_records(d_keys, nkeys, d_recs, nrec, d_in, d_out, d_status, d_ad=None, stream=None):
    rc = load().noise_gpu_decrypt_records(_ptr(d_keys), nkeys, _ptr(d_recs), nrec, _ptr(d_in),
                                          _ptr(d_out), _ptr(d_ad), _ptr(d_status), _stream(stream))
    _check(rc, "noise_gpu_decrypt_records")


def encrypt_sessions(d_keys, nkeys, d_key_idx, d_nonces, d_in, in_stride, d_out, out_stride,
                     length, nrec, stream=None):
    rc = load().noise_gpu_encrypt_sessions(_ptr(d_keys), nkeys, _ptr(d_key_idx), _ptr(d_nonces),
                                           _ptr(d_in), in_stride, _ptr(d_out), out_stride, length,
                                           nrec, _stream(stream))
    _check(rc, "noise_gpu_encrypt_sessions")


def decrypt_sessions(d_keys, nkeys, d_key_idx, d_nonces, d_in, in_stride, d_out, out_stride,
                     length, d_status, nrec, stream=None):
    rc = load().noise_gpu_decrypt_sessions(_ptr(d_keys), nkeys, _ptr(d_key_idx), _ptr(d_nonces),
                                           _ptr(d_in), in_stride, _ptr(d_out), out_stride, length,
                                           _ptr(d_status), nrec, _stream(stream))
    _check(rc, "noise_gpu_decrypt_sessions")


def rekey_keys(d_keys, nkeys, stream=None):
    _check(load().noise_gpu_rekey_keys(_ptr(d_keys), nkeys, _stream(stream)), "noise_gpu_rekey_keys")


def x25519(d_scalars, d_points, d_out, n, stream=None):
    """d_out[i] = X25519(d_scalars[i], d_points[i] or 9): n x 32-byte device arrays."""
    _check(load().noise_gpu_x25519(_ptr(d_scalars), _ptr(d_points) if d_points is not None else None,
                                   _ptr(d_out), n, _stream(stream)), "noise_gpu_x25519")


def fill_synthetic(d_dst, nbytes, seed, offset=0, stream=None, dst_offset=0):
    rc = load().noise_gpu_fill_synthetic(ctypes.c_void_p(d_dst.data_ptr() + dst_offset), offset,
                                         nbytes, seed, _stream(stream))
    _check(rc, "noise_gpu_fill_synthetic")


def span(base, stride=0, length=0, off=None, lens=None):
    """A noise_gpu_span over torch device tensors (base: uint8, off: int64
    offsets, lens: int32 lengths; None = uniform stride / length)."""
    return Span(base.data_ptr(), None if off is None else off.data_ptr(), stride,
                None if lens is None else lens.data_ptr(), length, 0)


class HandshakeBatch:
    """n sessions of one handshake pattern in one role on the GPU
    (noise_gpu_hs_*): the batched form of noise::HandshakeState."""

    def __init__(self, pattern, initiator, n):
        self.lib, self.n = load(), n
        h = ctypes.c_void_p()
        _check(self.lib.noise_gpu_hs_create(pattern.encode(), 1 if initiator else 0, n,
                                            ctypes.byref(h)), "noise_gpu_hs_create")
        self.h = h

    def close(self):
        if self.h:
            _check(self.lib.noise_gpu_hs_destroy(self.h), "noise_gpu_hs_destroy")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        i = HsInfo()
        _check(self.lib.noise_gpu_hs_info_get(self.h, ctypes.byref(i)), "noise_gpu_hs_info_get")
        return i

    def set_key(self, which, d_keys, stride=32, stream=None):
        _check(self.lib.noise_gpu_hs_set_key(self.h, which, _ptr(d_keys), stride, _stream(stream)),
               "noise_gpu_hs_set_key")

    def set_psks(self, d_psks, stream=None):
        _check(self.lib.noise_gpu_hs_set_psks(self.h, _ptr(d_psks), _stream(stream)),
               "noise_gpu_hs_set_psks")

    def start(self, prologue=None, stream=None):
        _check(self.lib.noise_gpu_hs_start(self.h, ctypes.byref(prologue) if prologue else None,
                                           _stream(stream)), "noise_gpu_hs_start")

    def write_message(self, msg, payload=None, d_msg_len=None, stream=None):
        _check(self.lib.noise_gpu_hs_write_message(
            self.h, ctypes.byref(payload) if payload else None, ctypes.byref(msg), _ptr(d_msg_len),
            _stream(stream)), "noise_gpu_hs_write_message")

    def read_message(self, msg, payload=None, d_payload_len=None, d_status=None, stream=None):
        _check(self.lib.noise_gpu_hs_read_message(
            self.h, ctypes.byref(msg), ctypes.byref(payload) if payload else None,
            _ptr(d_payload_len), _ptr(d_status), _stream(stream)), "noise_gpu_hs_read_message")

    def status(self, d_status, stream=None):
        _check(self.lib.noise_gpu_hs_status(self.h, _ptr(d_status), _stream(stream)),
               "noise_gpu_hs_status")

    def split(self, d_k1, d_k2, d_hash=None, d_rs=None, stream=None):
        _check(self.lib.noise_gpu_hs_split(self.h, _ptr(d_k1), _ptr(d_k2), _ptr(d_hash), _ptr(d_rs),
                                           _stream(stream)), "noise_gpu_hs_split")


# ---- host-buffer entry points (CipherState single-record path) ------------
def encrypt_host(key, nonce, ad, plaintext):
    """ENCRYPT(k, n, ad, pt) through the GPU; returns ct || tag (bytes)."""
    buf = ctypes.create_string_buffer(bytes(plaintext), len(plaintext) + 16)
    adb = bytes(ad)
    rc = load().noise_gpu_encrypt_host(_key(key), nonce, adb or None, len(adb), buf, len(plaintext))
    _check(rc, "noise_gpu_encrypt_host")
    return buf.raw


def decrypt_host(key, nonce, ad, ciphertext):
    """DECRYPT through the GPU; returns plaintext or raises NoiseGpuError(E_MAC)."""
    ct = bytes(ciphertext)
    buf = ctypes.create_string_buffer(ct, max(len(ct), 1))
    adb = bytes(ad)
    rc = load().noise_gpu_decrypt_host(_key(key), nonce, adb or None, len(adb), buf, len(ct))
    _check(rc, "noise_gpu_decrypt_host")
    return buf.raw[:len(ct) - 16]


def rekey_host(key):
    buf = ctypes.create_string_buffer(_key(key), 32)
    _check(load().noise_gpu_rekey_host(buf), "noise_gpu_rekey_host")
    return buf.raw


def set_resident(on, idle_us=0):
    """Resident latency mode of the calling thread's single-record path
    (noise_gpu_set_resident): one workgroup stays on the GPU while on."""
    _check(load().noise_gpu_set_resident(1 if on else 0, idle_us), "noise_gpu_set_resident")


def thread_release():
    _check(load().noise_gpu_thread_release(), "noise_gpu_thread_release")


def version():
    return load().noise_gpu_version().decode()
