"""CPU: the C-ABI library builds, loads, exports every symbol include/noise_gpu.h
declares, validates arguments before touching a device, and fails loudly
(no CPU fallback) when no gfx950 device is present."""
import ctypes
import os
import subprocess

import pytest

import noise_amd

ROOT = noise_amd.ROOT


def test_library_exports_every_declared_symbol():
    lib = noise_amd.load()
    names = noise_amd.declared_symbols()
    assert len(names) >= 17
    for name in names:
        assert hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", noise_amd.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T " in line}
    assert set(names) <= exported


def test_library_does_not_link_the_oracle():
    out = subprocess.run(["ldd", noise_amd.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out and "noise_ref" not in out
    nm = subprocess.run(["nm", "-D", noise_amd.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in nm and "crypto_aead" not in nm


def test_status_strings():
    lib = noise_amd.load()
    assert lib.noise_gpu_strerror(noise_amd.E_MAC) == b"Invalid MAC"
    assert lib.noise_gpu_strerror(noise_amd.E_NONCE) == b"Nonce limit has been exceeded!"
    assert lib.noise_gpu_version().startswith(b"noise-mi355x")


def test_argument_validation_precedes_device():
    lib = noise_amd.load()
    key = bytes(range(1, 33))
    buf = ctypes.c_void_p(0x10000)
    # null buffers
    assert lib.noise_gpu_encrypt_uniform(key, 0, None, 64, buf, 80, 64, None, 0, 0, 4, None) == noise_amd.E_ARG
    # output stride smaller than len + 16
    assert lib.noise_gpu_encrypt_uniform(key, 0, buf, 64, ctypes.c_void_p(0x90000), 64, 64, None, 0, 0, 4,
                                         None) == noise_amd.E_ARG
    # in-place with unequal strides
    assert lib.noise_gpu_encrypt_uniform(key, 0, buf, 80, buf, 96, 64, None, 0, 0, 4, None) == noise_amd.E_ARG
    # ad_len without ad
    assert lib.noise_gpu_encrypt_uniform(key, 0, buf, 64, ctypes.c_void_p(0x90000), 80, 64, None, 0, 8, 4,
                                         None) == noise_amd.E_ARG
    # decrypt without status
    assert lib.noise_gpu_decrypt_uniform(key, 0, buf, 80, ctypes.c_void_p(0x90000), 64, 64, None, 0, 0,
                                         None, 4, None) == noise_amd.E_ARG
    # empty batches are no-ops, even without a device
    assert lib.noise_gpu_encrypt_uniform(key, 0, None, 0, None, 0, 0, None, 0, 0, 0, None) == noise_amd.OK
    # an all-zero key is "no key" (Noise HasKey() false): refused, never used
    zero = bytes(32)
    assert lib.noise_gpu_encrypt_uniform(zero, 0, buf, 64, ctypes.c_void_p(0x90000), 80, 64, None, 0, 0, 4,
                                         None) == noise_amd.E_ARG
    assert lib.noise_gpu_decrypt_uniform(zero, 0, buf, 80, ctypes.c_void_p(0x90000), 64, 64, None, 0, 0,
                                         buf, 4, None) == noise_amd.E_ARG
    hbuf = ctypes.create_string_buffer(64)
    assert lib.noise_gpu_encrypt_host(zero, 0, None, 0, hbuf, 16) == noise_amd.E_ARG
    assert lib.noise_gpu_decrypt_host(zero, 0, None, 0, hbuf, 32) == noise_amd.E_ARG
    # descriptor offsets near 2^64 must not wrap past the host bounds check
    rec = noise_amd.Record(in_off=(1 << 64) - 8, out_off=0, nonce=0, ad_off=0, len=64, ad_len=0,
                           key_idx=0, reserved=0)
    out = ctypes.create_string_buffer(256)
    src = ctypes.create_string_buffer(256)
    assert lib.noise_gpu_encrypt_records_host(key, 1, ctypes.byref(rec), 1, src, 256, out, 256,
                                              None, 0) == noise_amd.E_ARG
    rec = noise_amd.Record(in_off=0, out_off=(1 << 64) - 16, nonce=0, ad_off=0, len=64, ad_len=0,
                           key_idx=0, reserved=0)
    assert lib.noise_gpu_encrypt_records_host(key, 1, ctypes.byref(rec), 1, src, 256, out, 256,
                                              None, 0) == noise_amd.E_ARG
    rec = noise_amd.Record(in_off=0, out_off=0, nonce=0, ad_off=(1 << 64) - 4, len=64, ad_len=8,
                           key_idx=0, reserved=0)
    assert lib.noise_gpu_encrypt_records_host(key, 1, ctypes.byref(rec), 1, src, 256, out, 256,
                                              src, 16) == noise_amd.E_ARG


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_no_device_fails_loudly():
    with pytest.raises(noise_amd.NoiseGpuError) as e:
        noise_amd.encrypt_host(bytes(range(32)), 0, b"", b"hello")
    assert e.value.code == noise_amd.E_NODEV
    lib = noise_amd.load()
    assert lib.noise_gpu_rekey_host(ctypes.create_string_buffer(32)) == noise_amd.E_NODEV


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_context_api_without_device():
    lib = noise_amd.load()
    h = ctypes.c_void_p()
    assert lib.noise_gpu_ctx_create(0, ctypes.byref(h)) == noise_amd.E_NODEV and not h.value
    assert lib.noise_gpu_ctx_create(0, None) == noise_amd.E_ARG
    assert lib.noise_gpu_ctx_destroy(None) == noise_amd.OK
    buf = ctypes.create_string_buffer(64)
    assert lib.noise_gpu_ctx_encrypt_host(None, bytes(range(32)), 0, None, 0, buf, 16) == noise_amd.E_ARG
    assert lib.noise_gpu_ctx_rekey_host(None, buf) == noise_amd.E_ARG


def test_cipherstate_host_rules():
    """noise::CipherState rules that run before any device call: spec
    has_key, the 2^64-2 nonce limit (noise.cpp:398), 40-byte layout."""
    exe = os.path.join(ROOT, "noise-cpp_amd", "bin", "cipherstate_test")
    assert os.path.exists(exe), "build() first"
    r = subprocess.run([exe, "--host-only"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout


def test_handshake_batch_argument_validation():
    """noise_gpu_hs_*: names and counts are checked before any device call;
    NULL handles are refused; destroy(NULL) is a no-op."""
    lib = noise_amd.load()
    h = ctypes.c_void_p()
    assert lib.noise_gpu_hs_create(b"XY", 1, 16, ctypes.byref(h)) == noise_amd.E_ARG
    assert b"unknown handshake pattern" in lib.noise_gpu_last_error()
    assert lib.noise_gpu_hs_create(b"XXpsk9", 1, 16, ctypes.byref(h)) == noise_amd.E_ARG
    assert lib.noise_gpu_hs_create(b"XX", 1, 0, ctypes.byref(h)) == noise_amd.E_ARG
    assert lib.noise_gpu_hs_create(None, 1, 16, ctypes.byref(h)) == noise_amd.E_ARG
    assert lib.noise_gpu_hs_destroy(None) == noise_amd.OK
    info = noise_amd.HsInfo()
    assert lib.noise_gpu_hs_info_get(None, ctypes.byref(info)) == noise_amd.E_ARG
    assert lib.noise_gpu_hs_start(None, None, None) == noise_amd.E_ARG
    assert lib.noise_gpu_hs_split(None, None, None, None, None, None) == noise_amd.E_ARG
    assert ctypes.sizeof(noise_amd.Span) == 40 and ctypes.sizeof(noise_amd.HsInfo) == 24


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_handshake_batch_needs_a_device():
    h = ctypes.c_void_p()
    assert noise_amd.load().noise_gpu_hs_create(b"XX", 1, 16, ctypes.byref(h)) == noise_amd.E_NODEV
    assert not h.value


def test_reference_free_function_signatures(tmp_path):
    """the reference's exported free functions
    noise::encrypt / noise::decrypt (noise.cpp:202-204, 254-256: `T` symbols
    of its library) resolve against libnoise_amd.so.  A translation unit that
    declares only the reference's signatures (tests/cpp/ref_signatures.cpp,
    nothing from this build's headers) is compiled; every noise:: symbol it
    leaves undefined must be a defined text symbol of the library, and the
    linked program runs: without a device the engine refuses loudly
    (runtime_error), it never falls back to a host AEAD."""
    src = os.path.join(ROOT, "tests", "cpp", "ref_signatures.cpp")
    obj, exe = str(tmp_path / "ref_signatures.o"), str(tmp_path / "ref_signatures")
    subprocess.run(["g++", "-std=c++20", "-O1", "-c", src, "-o", obj], check=True)
    undef = subprocess.run(["nm", "-u", obj], capture_output=True, text=True, check=True).stdout.split()
    want = sorted(s for s in undef if s.startswith("_ZN5noise"))
    assert want == ["_ZN5noise7decryptERSt5arrayIhLm32EEmSt8optionalISt6vectorIhSaIhEEERS6_",
                    "_ZN5noise7encryptERSt5arrayIhLm32EEmSt8optionalISt6vectorIhSaIhEEERS6_"]
    nm = subprocess.run(["nm", "-D", "--defined-only", noise_amd.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T " in line}
    assert set(want) <= exported
    libdir = os.path.dirname(noise_amd.LIB_PATH)
    subprocess.run(["g++", obj, "-o", exe, "-L" + libdir, "-lnoise_amd", "-Wl,-rpath," + libdir], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    if r.returncode == 3:  # no gfx950 device here: refused, not computed on the host
        assert "no gfx950 device" in r.stdout
    else:
        assert r.returncode == 0 and "round trip ok" in r.stdout, r.stdout + r.stderr


def test_resident_request_tag_survives_tears(tmp_path):
    """the resident request line's per-chunk check
    (launchers.hpp req_chunk_tag) is non-linear -- a chunk torn into a new
    seq word over stale (zero or previous) payload words does not decode to
    the new seq for structured lengths / nonces (tests/cpp/req_tag_test.cpp,
    host-only)."""
    exe = str(tmp_path / "req_tag_test")
    subprocess.run(["g++", "-std=c++20", "-O1", "-pthread", "-I", os.path.join(ROOT, "tools", "emu", "include"),
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "noise-cpp_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "req_tag_test.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "decode to the new seq" in r.stdout and ", 0 decode" in r.stdout
