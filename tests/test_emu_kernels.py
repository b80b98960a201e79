"""CPU-side check of the kernels' indexing: the unmodified records-path
kernels (classification, tile / wave / lane-per-record) compiled as host C++
against the HIP stand-in in tools/emu, run under AddressSanitizer on
BASELINE config-4 shaped batches and compared with the oracle.  The grid is
capped at 3 workgroups so every workgroup loops over several super-tiles /
batches; the gap puts records past 2^31 bytes into their buffers (64-bit
offsets whose low word has bit 31 set).  Test infrastructure only: the
product runs these kernels on the GPU (tests/test_gpu_records_mixed.py)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tools", "emu")
BIN = os.path.join(EMU, "build", "emu_records")


@pytest.fixture(scope="module")
def emu_bin():
    r = subprocess.run(["make", "-C", EMU, "GRID_CAP=3u"], capture_output=True, text=True,
                       timeout=900)
    if r.returncode != 0:
        pytest.fail("emulation build failed:\n" + r.stdout[-2000:] + r.stderr[-4000:])
    return BIN


@pytest.mark.parametrize("mode,nrec,seed,gap", [
    ("cfg4", 2300, 4, 0),
    ("inplace", 2100, 5, (2 << 30) + 4096),
])
def test_records_path_emulated(emu_bin, mode, nrec, seed, gap):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:allocator_may_return_null=1")
    r = subprocess.run([emu_bin, mode, str(nrec), str(seed), str(gap)], capture_output=True,
                       text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "ok (0 failures)" in r.stdout
