"""The multi-GPU bench path on a GPU box: bench.py --gpus 2 through its own
launcher (two rank processes, gloo control plane, per-rank disjoint nonce
ranges, barrier + max-over-ranks timing), the ranks sharing the box's GPU
(--share-device).  One JSON line with n_gpus 2, disjoint shards, exit 0 --
the command the driver's multi-GPU run uses, minus the device count.
SURVEY.md 8(e): records shard per GPU with no collective.

With --check-oracle every rank then compares its WHOLE shard with the CPU
oracle (tests/fullcheck.check_bench_shard) at its global nonce base and data
offset: rank 1's records are bit-exact against noise::encrypt / decrypt at
nonces rank 1 owns (noise.cpp:207-215; monocypher.c:2891-2929), which a
self round trip cannot show (a nonce-base or data-offset error that is the
same in both directions round-trips and self-authenticates)."""
import json
import os
import subprocess
import sys

import pytest

import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _run(extra, timeout=300):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    cmd = [sys.executable, os.path.join(noise_amd.ROOT, "bench.py"), "--gpus", "2", "--share-device",
           "--no-cpu-baseline", "--steps", "3", "--warmup", "2", "--min-warmup-s", "0"] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert "rank 1/2" in p.stderr and "rank 0/2" in p.stderr
    return line, sorted(line["shards"], key=lambda s: s["rank"])


def test_bench_two_ranks_share_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    line, shards = _run(["--records", "65536"])
    assert [s["rank"] for s in shards] == [0, 1]
    assert all(s["records"] == 65536 for s in shards)
    assert shards[0]["nonce_hi"] <= shards[1]["nonce_lo"], shards


# (config, records per rank or total, expected nonce base of rank 1)
SHARDED = [
    (2, 65536, 65536),     # weak: each rank its own 65536 nonces
    (5, 262144, 131072),   # strong: one 262144-record range cut in two
    (4, 65536, 65536),     # weak: Zipf mix, classifier + segments + tails
    (3, 0, 1 << 20),       # weak: 65536 sessions x 16 per rank, rank-offset keys and data
]


@pytest.mark.parametrize("cfg,records,base1", SHARDED, ids=["cfg2", "cfg5", "cfg4", "cfg3"])
def test_bench_two_ranks_oracle_exact(cfg, records, base1):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    line, shards = _run(["--config", str(cfg), "--records", str(records), "--check-oracle"])
    assert [s["rank"] for s in shards] == [0, 1]
    assert shards[1]["nonce_lo"] == base1 and shards[0]["nonce_lo"] == 0, shards
    for s in shards:
        oc = s["oracle_check"]
        assert oc["nonce_base"] == s["nonce_lo"]
        n = s["records"]
        assert oc["encrypt"]["records"] == n and oc["encrypt"]["mismatches"] == 0, oc
        assert oc["decrypt"]["records"] == n and oc["decrypt"]["mismatches"] == 0, oc
        assert oc["synthetic"]["bytes"] > 0
    if cfg == 5:
        assert sum(s["records"] for s in shards) == records
