"""One rank of the RCCL parity check (tests/test_multi_gpu.py); run as a script.

    python tests/rccl_ranks.py        (RANK, WORLD_SIZE, MASTER_ADDR/PORT in the env)

Every rank binds GPU `rank`, joins a torch.distributed "nccl" (RCCL) group and
takes PyTorch's communicator (the librccl instance libherdsman_fhe.so binds to):
  * fhe_bcast_key: rank 0 holds the oracle's key, the others garbage; after the
    broadcast every rank's key equals the oracle's bit for bit;
  * fhe_reduce_ranks ADD and MUL_RELIN: rank r holds ciphertext r; root's result
    equals the oracle's evaluation of the same binomial tree.
Prints "rank <r> ok" on success.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import herdsman_amd.backend as hb  # noqa: E402
from oracle_ffi import Oracle, SCHEME_CKKS  # noqa: E402


def expected_tree(o, cts, op, rlk, world, root=0):
    """The binomial tree of fhe_reduce_ranks evaluated with the oracle's ops."""
    vals = {r: cts[r][None] for r in range(world)}
    s = 1
    while s < world:
        for rel in range(0, world, 2 * s):
            if rel + s < world:
                a, b = vals[(rel + root) % world], vals[(rel + s + root) % world]
                vals[(rel + root) % world] = o.ct_add(a, b) if op == hb.REDUCE_ADD else o.mul_relin(a, b, rlk)
        s *= 2
    return vals[root][0]


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", device_id=dev)
    comm = int(dist.group.WORLD._get_backend(dev)._comm_ptr())
    assert comm, "no RCCL communicator pointer from torch"
    log_n, L, K, dnum = 13, 4, 2, 2
    o = Oracle(SCHEME_CKKS, log_n, L, K, dnum)
    c = hb.Context(SCHEME_CKKS, log_n, L, K, dnum, moduli=o.moduli, device=rank)
    c.set_stream(torch.cuda.current_stream(dev))
    key = o.uniform(o.key_shape(), seed=500)
    dk = hb.to_device(key, dev) if rank == 0 else hb.empty(o.key_shape(), device=dev).fill_(-1)
    c.bcast_key(dk, comm, root=0)
    torch.cuda.synchronize(dev)
    assert np.array_equal(hb.to_host(dk), key), "fhe_bcast_key"
    cts = [o.uniform((1, 2, L, 1 << log_n), seed=600 + r)[0] for r in range(world)]
    lib = hb.load_library()
    for op in (hb.REDUCE_ADD, hb.REDUCE_MUL_RELIN):
        ct = hb.to_device(cts[rank][None], dev)
        tmp = hb.empty(ct.shape, device=dev)
        rc = lib.fhe_reduce_ranks(c.h, ct.data_ptr(), op, dk.data_ptr(), comm, 0, tmp.data_ptr())
        assert rc == 0, lib.fhe_last_error(c.h)
        torch.cuda.synchronize(dev)
        if rank == 0:
            assert np.array_equal(hb.to_host(ct)[0], expected_tree(o, cts, op, key, world)), f"reduce op {op}"
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    main()
