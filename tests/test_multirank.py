"""CPU, world_size 2 over gloo: the multi-GPU bookkeeping of bench.py.
Records shard per rank with no data-path collective; the only collectives
are the barrier and the max/sum reductions of the timing."""
import os
import socket
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    R = 1000
    # weak scaling: disjoint nonce ranges, one per rank
    base = bench.rank_nonce_base(2, rank, world, R, R * world)
    # strong scaling: one range of 1003 split contiguously
    lo, hi = bench.shard(1003, rank, world)
    base5 = bench.rank_nonce_base(5, rank, world, hi - lo, 1003)
    elapsed, total = bench.reduce_over_ranks(dist, 0.5 + rank, R + rank, "cpu")
    dist.barrier()
    q.put((rank, base, lo, hi, base5, elapsed, total))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharding_and_reductions(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    bases = [r[1] for r in res]
    assert bases == [0, 1000]  # disjoint weak-scaling nonce ranges
    spans = [(r[2], r[3]) for r in res]
    assert spans[0][0] == 0 and spans[-1][1] == 1003
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))  # contiguous, no overlap
    assert [r[4] for r in res] == [s[0] for s in spans]
    assert all(r[5] == 1.5 for r in res)          # max over ranks
    assert all(r[6] == 2001 for r in res)         # sum of records
