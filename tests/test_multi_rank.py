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


# ---------------------------------------------------------------- reduce tree
Q_TEST = 2147483647  # small modulus: the int64 stand-in combine below cannot overflow
K_MIX = 1000003


def _mix(a, b):
    """Non-commutative stand-in for a ciphertext combine (a <- a*K + b mod q): the
    result pins WHICH partial results were combined in WHICH order."""
    a.mul_(K_MIX).add_(b).remainder_(Q_TEST)


def _simulate(world, root, init):
    """Expected root value, level by level: at level s the rank at offset rel
    (rel % 2s == 0) absorbs the one at rel + s, which finished its own levels."""
    vals = {rel: init((rel + root) % world) for rel in range(world)}
    s = 1
    while s < world:
        for rel in range(0, world, 2 * s):
            if rel + s < world:
                vals[rel] = (vals[rel] * K_MIX + vals[rel + s]) % Q_TEST
        s *= 2
    return vals[0]


def _init(rank):
    return (rank + 1) * 7919 + 13


def _reduce_worker(rank, world, root, port, q):
    import torch.distributed as dist
    from herdsman_amd.dist import reduce_ranks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ct = torch.full((2, 3, 16), _init(rank), dtype=torch.int64)
        scratch = torch.empty_like(ct)
        reduce_ranks(ct, _mix, scratch, root=root)
        q.put((rank, int(ct[0, 0, 0]), bool((ct == ct[0, 0, 0]).all())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,root", [(2, 0), (3, 0), (4, 1)])
def test_gloo_reduce_ranks_tree(world, root):
    """The cross-rank join of per-rank partial results delivers
    exactly the binomial-tree combination to root."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reduce_worker, args=(r, world, root, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (v, uni)) for r, v, uni in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[root][1]
    assert res[root][0] == _simulate(world, root, _init)


def test_reduce_schedule_is_a_tree():
    """Every non-root rank sends exactly once, to a rank that receives from it."""
    from herdsman_amd.dist import reduce_schedule
    for world in range(1, 17):
        for root in range(world):
            sched = {r: reduce_schedule(r, world, root) for r in range(world)}
            sends = {r: [p for k, p in s if k == "send"] for r, s in sched.items()}
            assert sends[root] == []
            for r in range(world):
                if r == root:
                    continue
                assert len(sends[r]) == 1 and sched[r][-1][0] == "send"
                assert ("recv", r) in sched[sends[r][0]]
            assert sum(len(s) for s in sched.values()) == 2 * (world - 1)


# ------------------------------------------------------- bench.py multi-rank launcher
def test_bench_launcher_spawns_ranks_dry_run():
    """`bench.py --gpus 2` outside torchrun spawns 2 fresh rank processes (the
    parent never touches a GPU); the ranks form a gloo group, split the C5 batch
    of 8192 with herdsman's rule and time with max-over-ranks (--dry-run: the
    control flow without GPU work)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["ranks"] == 2
    shards = sorted(line["shards"])
    assert [s[1] for s in shards] == [4096, 4096] and all(s[1] == s[2] for s in shards)
    assert len({s[3] for s in shards}) == 2  # two processes
    assert line["elapsed"] >= 0.02  # the slower rank's time


def test_bench_driver_argv_eight_ranks_dry_run():
    """The driver's exact 8-GPU launch (torch.distributed.run, --nproc-per-node 8,
    127.0.0.1) with --dry-run appended: 8 ranks, shards of 1024 by herdsman's
    partition rule, n_gpus and the per-rank list cover all 8."""
    import json
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "8", "--steps", "5", "--warmup", "2", "--dry-run"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["ranks"] == 8 and line["n_gpus"] == 8
    assert sorted(sh[1] for sh in line["shards"]) == [1024] * 8
    assert all(sh[1] == sh[2] for sh in line["shards"])  # each rank's wave plan covers its shard once
    assert len(line["per_rank_ct_mult_per_s"]) == 8 and line["steps"] == 5 and line["warmup"] == 2
    assert len({sh[3] for sh in line["shards"]}) == 8  # eight processes


def test_wave_plan_covers_each_shard_once():
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for G, world, batch, streams, pool in [(8192, 1, 128, 4, 1024), (8192, 8, 128, 4, 1024), (8192, 3, 128, 4, 1024),
                                           (1000, 7, 64, 3, 100), (5, 8, 128, 4, 1024)]:
        total = 0
        for rank in range(world):
            my, B, S, waves, P, Bs, plan = bench.wave_plan(G, batch, streams, pool, world, rank)
            assert sum(hi - lo for _, lo, hi in plan) == my
            assert all(0 <= lo < hi <= P and 0 <= i < S and hi - lo <= Bs for i, lo, hi in plan)
            assert P % B == 0 and P <= max(pool, B) * 1 + B
            total += my
        assert total == G
