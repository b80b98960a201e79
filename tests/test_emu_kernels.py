"""CPU-side check of the kernels' indexing: the unmodified records-path
kernels (classification, tile / long-record segments / lane-per-record) compiled as host C++
against the HIP stand-in in tools/emu, run under AddressSanitizer on
BASELINE config-4 shaped batches and compared with the oracle.  The emulation
build classifies batches from 64 records (the product: 2048) and caps the
grid at 3 workgroups so every workgroup loops over several super-tiles /
batches; the gap puts records past 2^31 bytes into their buffers (64-bit
offsets whose low word has bit 31 set); "ragged" lengths 1..70000 give odd
segment tails and > 65535-byte records (generic class); a 300-segment
scratch cap forces the segment-overflow path.  Test infrastructure only: the
product runs these kernels on the GPU (tests/test_gpu_records_mixed.py).
The batched-handshake kernels run the same way (emu_handshake)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tools", "emu")
JOBS = "-j%d" % max(1, min(8, os.cpu_count() or 1))  # the ASan objects build in parallel
BIN = os.path.join(EMU, "build", "emu_records")


# The emulated runs are independent processes that each keep about one core
# busy (a block's threads take turns at the wave barriers), so the module
# builds every binary once and then starts all runs together on a small pool;
# each test waits for its own.  That keeps the CPU suite's wall time near the
# longest single run instead of the sum.
RECORDS_CASES = [
    ("cfg4", 700, 4, 0),
    ("cfg4", 2500, 8, 0),   # >= 1000 records (emulation build): the chunked decrypt pipeline
    ("inplace", 500, 5, (2 << 30) + 4096),
    ("ragged", 300, 6, 0),
    # round 6: config-4 buckets minus U(0..63) -- the masked tile classes and
    # the masked tail units of the long records, copy and in place
    ("jitter", 700, 4, 0),
    ("jitterinplace", 500, 5, 0),
]
TRANSPORT_CASES = [
    ["pipeline", "10", "300", "2"],                       # launcher thread, tiny slots
    ["pipeline", "10", "300", "3"],                       # flush() issues its own work
    ["pipeline_batch", "20", "600", "4"],                 # copy pool, ragged batches
    # parallel bookkeeping (>= 4096 messages per call), byte cut; no 65519-B messages
    ["pipeline_batch", "30", "4500", "6", "8192", str(512 << 10), "300", "20000", "4", "0"],
    ["keyrace", "4096"],                                  # key rows uploaded on another slot's stream
    # 96 copy threads, 64 KiB slots of ~85 messages: the byte cut leaves fewer
    # messages than threads (empty chunks must keep their own index)
    ["pipeline_batch", "40", "4500", "8", "8192", str(64 << 10), "1500", "20000", "96", "0"],
]
BUILD = os.path.join(EMU, "build")
ASAN_NOLEAK = "detect_leaks=0:allocator_may_return_null=1"


def _make(*args):
    r = subprocess.run(["make", JOBS, "-C", EMU, *args], capture_output=True, text=True, timeout=1200)
    if r.returncode != 0:
        pytest.fail("emulation build failed:\n" + r.stdout[-2000:] + r.stderr[-4000:])


def _job_list():
    jobs = {}
    for mode, nrec, seed, gap in RECORDS_CASES:
        jobs["records-%s-%d" % (mode, nrec)] = (
            [BIN, mode, str(nrec), str(seed), str(gap)], ASAN_NOLEAK, 900)
    jobs["records-overflow"] = ([BIN + "_seg300ull", "cfg4", "700", "7", "0"], ASAN_NOLEAK, 900)
    # the uniform entry off the exact tile table: the masked tile kernel
    jobs["uniform"] = ([os.path.join(BUILD, "emu_uniform"), "5"], ASAN_NOLEAK, 900)
    # leak detection on: noise_gpu_ctx_destroy and noise_gpu_thread_release
    # must free everything the engine allocated (the run ends with both)
    jobs["api"] = ([os.path.join(BUILD, "emu_api")], "detect_leaks=1", 1500)
    for i, args in enumerate(TRANSPORT_CASES):
        # case 5 (96 copy threads) takes ~190 s alone, mostly kernel thread
        # creation (sys time); beside the pool's other jobs on 8 cores it
        # took 600+ s once in round 6 (and passed the run before): 900 s
        jobs["transport-%d" % i] = ([os.path.join(BUILD, "emu_transport"), *args], "detect_leaks=1",
                                    900 if i == 5 else 600)
    jobs["handshake"] = ([os.path.join(BUILD, "emu_handshake"),
                          os.path.join(ROOT, "tests", "golden", "handshake_vectors.tsv")], "detect_leaks=0", 900)
    jobs["x25519"] = ([os.path.join(BUILD, "emu_x25519"), "300", "11"], "detect_leaks=0", 300)
    return jobs


@pytest.fixture(scope="module")
def emu():
    """Build every emulation binary, start every run; name -> future of its
    CompletedProcess (slowest first, so the pool drains evenly)."""
    import concurrent.futures
    _make("GRID_CAP=3u")
    _make("GRID_CAP=3u", "SEG_CAP=300ull")
    _make("GRID_CAP=3u", "api")
    _make("GRID_CAP=3u", "uniform")
    _make("GRID_CAP=3u", "transport")
    _make("handshake")
    jobs = _job_list()

    logs = os.path.join(BUILD, "logs")
    os.makedirs(logs, exist_ok=True)

    def run(name):
        argv, asan, timeout = jobs[name]
        # the whole output stays in build/logs/<name>.log (the assertion
        # messages carry only its tail; emu_api's watchdog lines and phase
        # times go there)
        with open(os.path.join(logs, name + ".log"), "w") as f:
            r = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                               timeout=timeout, env=dict(os.environ, ASAN_OPTIONS=asan))
            f.write(r.stdout)
            f.write(r.stderr)
        return r
    # slowest first, so the pool drains evenly: emu_api (~170 s alone; every
    # emulated launch of the 256-thread latency kernel costs ~0.2-0.6 s of
    # thread starts and barrier rounds, ~2.5x that beside the other runs)
    order = ["api", "transport-5", "handshake", "records-ragged-300", "records-cfg4-2500"]
    order += [k for k in jobs if k not in order]
    workers = max(2, min(6, (os.cpu_count() or 2) - 1))
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=workers)
    futs = {name: pool.submit(run, name) for name in order}
    yield futs
    pool.shutdown(wait=True)


def _result(emu, name):
    return emu[name].result()


@pytest.mark.parametrize("mode,nrec,seed,gap", RECORDS_CASES)
def test_records_path_emulated(emu, mode, nrec, seed, gap):
    """...and verify-before-write (crypto_aead_read, monocypher.c:2912-2929):
    every 16-byte store of the decrypt is watched (tools/emu store hook); no
    store puts a non-zero byte into the output range of a record whose tag
    fails, nor lands at all in one decrypted in place -- the segmented path
    (>= 1 KiB records) included: its Poly1305 pass and the finalize check
    every tag before the keystream pass writes any plaintext."""
    r = _result(emu, "records-%s-%d" % (mode, nrec))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "ok (0 failures)" in r.stdout
    assert ": 0 stores of unverified plaintext" in r.stdout
    assert "watched 0 failed" not in r.stdout  # the batch holds tampered long records


def test_uniform_ragged_lengths_emulated(emu):
    """noise_gpu_{en,de}crypt_uniform at 33 lengths off the exact tile table
    (1 .. 16383, every class edge), 16-byte aligned strides, copy and in
    place: the masked tile kernel (csrc/mtile_kernel.hpp) bit-exact against
    the oracle under AddressSanitizer, no store outside a record's output
    (ct || tag / plaintext), and -- with tampered tags, first and last
    ciphertext bytes -- no store of unverified plaintext (monocypher.c:
    2912-2929)."""
    r = _result(emu, "uniform")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "0 stores outside, 0 stores of unverified plaintext" in r.stdout
    assert "ok (0 failures)" in r.stdout


def test_host_entry_points_emulated_and_wiped(emu):
    """The C ABI's host-buffer entry points (noise_gpu_api.hip: the latency
    kernel for single records, the staged lane walk for AD > 8 KiB, rekey, the
    records path with its scratch, the uniform host pipeline) on the CPU under
    AddressSanitizer, bit-exact against the oracle, and after EVERY call every
    buffer the engine allocated is zero: no key, plaintext, ciphertext or
    one-time key is left in staging or scratch (monocypher.c:163-167)."""
    r = _result(emu, "api")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "emu_api ok" in r.stdout


def test_resident_wait_is_bounded_emulated(emu):
    """OneCtx::wait (noise_gpu_api.hip) returns NOISE_GPU_E_HIP for a request
    line the resident instance never takes (its check word corrupted by an
    emulation-only hook): with instances that leave at once (relaunch cap)
    and with one long-lived instance that keeps polling (the 10-s limit,
    checked before the relaunch branch) -- and the next call works.  The
    reference's encrypt_with_ad returns or throws, never spins
    (noise.cpp:393-427)."""
    r = _result(emu, "api")
    for what in ("synchronous instances", "asynchronous instance"):
        line = [l for l in r.stdout.splitlines() if l.startswith("refused request (%s)" % what)]
        assert line, r.stdout[-3000:]
        assert "rc 4 after" in line[0], line[0]
        assert float(line[0].split("after ")[1].split(" s")[0]) < 15.0, line[0]


@pytest.mark.parametrize("idx", range(len(TRANSPORT_CASES)))
def test_transport_pipeline_emulated(emu, idx):
    """noise::transport::Pipeline (host/transport.cpp: copy pool, launcher
    thread, parallel submit_batch bookkeeping, key-table uploads) over the
    emulated C ABI, under AddressSanitizer with leak detection: ciphertexts vs
    the oracle, nonce accounting, tampered records, and every slot stream's
    records scratch and companion stream released with the Pipeline."""
    r = _result(emu, "transport-%d" % idx)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "ok (0 failures)" in r.stdout


def test_records_segment_overflow_emulated(emu):
    # long records past the 300-segment scratch fall back to the generic kernel
    r = _result(emu, "records-overflow")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "ok (0 failures)" in r.stdout


def test_emulated_batched_handshakes(emu):
    """The batched-handshake kernels (csrc/handshake_kernels.hip) and their
    host driver (csrc/handshake_batch.hip), unmodified, on the CPU under ASan:
    the reference's 110 vectors through noise_gpu_hs_* -- messages, handshake
    hashes, split keys, transport records under them vs the oracle."""
    r = _result(emu, "handshake")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "vectors 110, failed 0" in r.stdout and "transport records 211" in r.stdout, r.stdout


def test_emulated_fixed_base_public_keys(emu):
    """x25519_device.hpp's fixed-base path (edwards25519 radix-16 table,
    constant-time selects) on the CPU under ASan: RFC 7748 §6.1 and random /
    extreme scalars against the device ladder with u = 9 and the host X25519."""
    r = _result(emu, "x25519")
    assert r.returncode == 0 and "0 failures: ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_base_table_generator_is_current():
    """noise-cpp_amd/csrc/ed25519_base_table.inc is what tools/gen_base_table.py
    (exact big-integer edwards25519 arithmetic, self-checked) generates."""
    import importlib.util
    import tempfile
    spec = importlib.util.spec_from_file_location("gen_base_table",
                                                  os.path.join(ROOT, "tools", "gen_base_table.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with tempfile.TemporaryDirectory() as d:
        mod.OUT = os.path.join(d, "t.inc")
        mod.main()
        fresh = open(mod.OUT).read()
    assert fresh == open(os.path.join(ROOT, "noise-cpp_amd", "csrc", "ed25519_base_table.inc")).read()
