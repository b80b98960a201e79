"""The multi-GPU bench path on a GPU box: bench.py --gpus 2 through its own
launcher (two rank processes, gloo control plane, per-rank disjoint nonce
ranges, barrier + max-over-ranks timing), the ranks sharing the box's GPU
(--share-device).  One JSON line with n_gpus 2, disjoint shards, exit 0 --
the command the driver's multi-GPU run uses, minus the device count.
SURVEY.md 8(e): records shard per GPU with no collective."""
import json
import os
import subprocess
import sys

import pytest

import noise_amd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def test_bench_two_ranks_share_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    cmd = [sys.executable, os.path.join(noise_amd.ROOT, "bench.py"), "--gpus", "2", "--share-device",
           "--records", "65536", "--no-cpu-baseline", "--steps", "3", "--warmup", "2",
           "--min-warmup-s", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    shards = sorted(line["shards"], key=lambda s: s["rank"])
    assert [s["rank"] for s in shards] == [0, 1]
    assert all(s["records"] == 65536 for s in shards)
    assert shards[0]["nonce_hi"] <= shards[1]["nonce_lo"], shards
    assert "rank 1/2" in p.stderr and "rank 0/2" in p.stderr
