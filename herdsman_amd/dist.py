"""Multi-GPU plumbing for the ciphertext-batch path.

One process per GPU.  Ciphertexts are independent, so a batch shards with no
data-path collective; the only collective is ONE broadcast of the evaluation
key from rank 0 (RCCL over xGMI when the backend is "nccl").  This mirrors
herdsman's own partition sharding (/root/reference/src/service/
execution_service.cpp:545-548: one task per partition; partition p holds
floor(rows/P) rows, +1 for p < rows mod P, storage_service.cpp:121-129).
"""
from __future__ import annotations

import os
from typing import Callable, List, Tuple


def world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard_range(total: int, world_size: int, rank: int) -> Tuple[int, int]:
    """[begin, end) of `rank`'s items: floor(total/W) each, +1 for rank < total mod W
    (the same rule herdsman uses to split rows over partitions)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError("bad rank / world size")
    base, extra = divmod(total, world_size)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def _host_staged() -> bool:
    """gloo moves host tensors only: device tensors are staged through host memory."""
    import torch.distributed as dist
    return dist.get_backend() == "gloo"


def broadcast_key(key, src: int = 0) -> None:
    """Broadcast an evaluation key tensor in place (the only collective)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if key.is_cuda and _host_staged():
            tmp = key.cpu()
            dist.broadcast(tmp, src=src)
            key.copy_(tmp)
        else:
            dist.broadcast(key, src=src)


def max_over_ranks(x: float, device=None) -> float:
    """Max of a host float over ranks (timing: the job ends when the slowest rank ends)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=None if _host_staged() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_schedule(rank: int, world_size: int, root: int = 0) -> List[Tuple[str, int]]:
    """Binomial tree towards `root` (the schedule of fhe_reduce_ranks): at level
    s = 1, 2, 4, ... a rank whose offset from root is an odd multiple of s sends
    its partial result to offset - s and stops; one at an even multiple receives
    from offset + s (when that rank exists) and combines."""
    if world_size < 1 or not (0 <= rank < world_size and 0 <= root < world_size):
        raise ValueError("bad rank / world / root")
    rel, steps, s = (rank - root) % world_size, [], 1
    while s < world_size:
        if rel % (2 * s) == s:
            steps.append(("send", (rel - s + root) % world_size))
            break
        if rel % (2 * s) == 0 and rel + s < world_size:
            steps.append(("recv", (rel + s + root) % world_size))
        s *= 2
    return steps


def reduce_ranks(ct, combine: Callable, scratch, root: int = 0) -> None:
    """Join per-rank partial results with torch.distributed
    point-to-point transfers (RCCL on GPU tensors, gloo on CPU ones):
    combine(ct, scratch) folds a received ciphertext into ct, e.g. a batched
    mod-q add (ctx.add) or mul+relin on the GPU.  The result is in ct on root.
    The C ABI's fhe_reduce_ranks runs the same tree with ncclSend/ncclRecv."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    rank, world_size = dist.get_rank(), dist.get_world_size()
    for kind, peer in reduce_schedule(rank, world_size, root):
        if kind == "recv":
            dist.recv(scratch, src=peer)
            combine(ct, scratch)
        else:
            dist.send(ct, dst=peer)
