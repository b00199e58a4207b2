"""world_size-2 gloo tests of the multi-GPU plumbing (CPU, no GPU needed).

Covers herdsman_amd.dist: shard assignment (disjoint, complete, herdsman's
floor/+1 rule), the evaluation-key broadcast (the only collective) and the
max-over-ranks timing reduction used by bench.py.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from herdsman_amd.dist import broadcast_key, max_over_ranks, shard_range


def test_shard_range_rule():
    for total in (0, 1, 7, 8, 8192, 8193):
        for w in (1, 2, 3, 8):
            spans = [shard_range(total, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                assert a1 == b0
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
            assert sizes == sorted(sizes, reverse=True)
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # key: rank 0 holds the real words, the others garbage until the broadcast
        key = torch.arange(3 * 2 * 16 * 64, dtype=torch.int64) * 7 if rank == 0 else torch.full((3 * 2 * 16 * 64,), -1)
        broadcast_key(key, src=0)
        ok_key = bool(torch.equal(key, torch.arange(3 * 2 * 16 * 64, dtype=torch.int64) * 7))
        m = max_over_ranks(float(rank + 1) * 0.5)
        b, e = shard_range(8192, world, rank)
        q.put((rank, ok_key, m, b, e))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_key_broadcast_and_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), "key broadcast mismatch"
    assert all(r[2] == 1.0 for r in res), "max over ranks"
    assert res[0][3:] == (0, 4096) and res[1][3:] == (4096, 8192)
