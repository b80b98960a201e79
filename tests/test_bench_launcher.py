"""CPU: the real `python bench.py --gpus N` launcher (no WORLD_SIZE in the
environment) spawns N ranks, each rank gets its own nonce range, the ranks
meet over gloo for the barrier / max-over-ranks / shard table, and exactly one
JSON line comes out with n_gpus = N.  The workload is the --stub host
stand-in (no GPU here); the launcher, the rank environment and the reductions
are the ones the GPU run uses."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def run_bench(*extra, gpus=2, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--gpus", str(gpus),
                        "--steps", "3", "--warmup", "1", "--min-warmup-s", "0", *extra],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    return p


@pytest.mark.parametrize("gpus", [2, 3])
def test_launcher_spawns_ranks_one_json_line(gpus):
    p = run_bench("--records", "100", gpus=gpus)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == gpus and d["steps"] == 3 and d["scaling"] == "weak"
    shards = sorted(d["shards"], key=lambda s: s["rank"])
    assert [s["rank"] for s in shards] == list(range(gpus))
    # disjoint nonce ranges, one per rank, each of the rank's own records
    assert [(s["nonce_lo"], s["nonce_hi"]) for s in shards] == \
        [(100 * r, 100 * (r + 1)) for r in range(gpus)]
    # every rank logged itself
    for r in range(gpus):
        assert "rank %d/%d" % (r, gpus) in p.stderr
    # value counts every rank's records
    assert d["value"] > 0 and d["config"]["records_per_gpu"] == 100


def test_launcher_eight_ranks_per_rank_fields():
    """The driver's 8-GPU shape, rehearsed on the CPU: 8 ranks over gloo, one
    JSON line with n_gpus = 8, and each shard entry carries the rank's own
    encrypt / decrypt / step times and device, so the 8-GPU line shows every
    GPU's balance beside the max-over-ranks wall rate."""
    p = run_bench("--records", "256", gpus=8, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8
    shards = sorted(d["shards"], key=lambda s: s["rank"])
    assert [s["rank"] for s in shards] == list(range(8))
    for s in shards:
        assert s["enc_ms"] > 0 and s["dec_ms"] > 0 and s["step_ms"] > 0
        assert "device" in s and "name" in s["device"]
    # the line's wall time is the max over ranks
    assert d["ms_per_step"] >= max(s["step_ms"] for s in shards) * 0.999


def test_launcher_config5_eight_ranks_one_nonce_range():
    """Config 5 (strong scaling) at N = 8: one 8 Mi-record nonce range split
    contiguously, rank r holds 1 Mi records at nonce base r * 2^20 (SURVEY
    8(e); bench.py shard / rank_nonce_base, the same code the GPU run uses)."""
    p = run_bench("--config", "5", gpus=8, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 8 and d["scaling"] == "strong"
    shards = sorted(d["shards"], key=lambda s: s["rank"])
    assert [(s["nonce_lo"], s["nonce_hi"], s["records"]) for s in shards] == \
        [(r << 20, (r + 1) << 20, 1 << 20) for r in range(8)]


def test_single_gpu_path_does_not_launch():
    p = run_bench("--records", "64", gpus=1)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 1 and len(d["shards"]) == 1


def test_check_shards_flags_overlap():
    sys.path.insert(0, ROOT)
    import bench
    ok = [{"rank": 0, "nonce_lo": 0, "nonce_hi": 10}, {"rank": 1, "nonce_lo": 10, "nonce_hi": 20}]
    assert bench.check_shards(ok) is None
    bad = [{"rank": 0, "nonce_lo": 0, "nonce_hi": 11}, {"rank": 1, "nonce_lo": 10, "nonce_hi": 20}]
    assert "share" in bench.check_shards(bad)
    # strong scaling (cfg 5): contiguous slices of one range cover it exactly
    spans = [bench.shard(8 << 20, r, 8) for r in range(8)]
    assert spans[0][0] == 0 and spans[-1][1] == 8 << 20
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_roofline_fields_from_committed_profiles(cfg):
    """bench.py's roofline block is recomputable from profiles/: the kernel
    symbol the driver's run launches, HBM traffic from the committed PMC
    passes (gfx950 FETCH_SIZE correction), both HBM fractions and the VALU
    issue fraction from SQ_INSTS_VALU."""
    sys.path.insert(0, ROOT)
    import bench
    L = {2: 1024, 3: 1024, 5: 4096}[cfg]
    mode = 1 if cfg == 3 else 0
    R = (8 << 20) if cfg == 5 else (1 << 20)  # as profiled (cfg 5: the whole 8 Mi x 4 KiB)
    ms = 19.0 if cfg == 5 else 0.61
    # as profiled, then one rank's shard of an 8-GPU run (cfg 5: 1 Mi of the
    # 8 Mi records, at ~1/8 of the time): the per-launch PMC counts scale with
    # the records launched, the per-wave and utilisation figures do not
    for R, t in ((R, ms), (R // 8, ms / 8)):
        wl = {"R": R, "enc_bytes": R * (2 * L + 16), "dec_bytes": R * (2 * L + 17),
              "read_bytes": (R * L, R * (L + 16)),
              "knames": ((bench.tile_symbol(False, L, True, mode),), (bench.tile_symbol(True, L, True, mode),))}
        roof = bench.roofline(cfg, wl, t, t - 0.001)
        assert roof["kernel"].startswith("noise_amd::k_aead_tile<false, %d, true, %d" % (L, mode))
        assert roof["pmc_source"] and roof["pmc_source"].startswith("profiles/")
        assert roof["traffic"] and 0.95 < roof["traffic"] / wl["enc_bytes"] < 1.2
        assert 0 < roof["hbm_frac_read"] < roof["hbm_frac_rw"] < 1
        v = roof["valu"]
        assert v["insts_per_wave"] > 10000 and 0 < v["frac"] <= 1.2 and 0 < v["issue_util_profiled"] <= 1.05
        # the VALU-implied cap on the HBM fraction: above the achieved one
        # (the kernel cannot beat its own instruction count), below 1, and
        # the achieved fraction over it is the VALU issue fraction
        cap = roof["valu_cap_hbm_frac"]
        assert roof["hbm_frac_rw"] < cap < 1.0
        assert abs(roof["hbm_frac_rw"] / cap - v["frac"]) < 0.01


def test_two_ranks_on_one_device_refused():
    """an N-rank line whose ranks report the same
    device (PCI address) is refused -- non-zero exit, no JSON line -- unless
    the ranks were told to share the GPU (--share-device, the 1-GPU-box test
    hook), in which case the line is printed and says so."""
    p = run_bench("--records", "64", "--stub-same-device", gpus=2)
    assert p.returncode != 0
    assert "same device" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    p = run_bench("--records", "64", "--stub-same-device", "--share-device", gpus=2)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 2 and "share-device" in d["note"]
    # the per-rank spread of the launch times is in the line
    for f in ("enc_ms", "dec_ms", "step_ms"):
        sp = d["rank_spread"][f]
        assert sp["max"] >= sp["min"] > 0 and sp["max_over_min"] >= 1.0


def test_check_shards_device_aliasing():
    sys.path.insert(0, ROOT)
    import bench
    dev = lambda bus: {"index": 0, "name": "x", "pci_domain_id": 0, "pci_bus_id": bus, "pci_device_id": 0}
    two = [{"rank": 0, "nonce_lo": 0, "nonce_hi": 10, "device": dev(5)},
           {"rank": 1, "nonce_lo": 10, "nonce_hi": 20, "device": dev(5)}]
    assert "same device" in bench.check_shards(two)
    assert bench.check_shards(two, share_device=True) is None
    two[1]["device"] = dev(6)
    assert bench.check_shards(two) is None
    # no PCI address reported: nothing to compare
    two[0]["device"] = two[1]["device"] = {"index": 0, "name": "x"}
    assert bench.check_shards(two) is None
