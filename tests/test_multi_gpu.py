"""RCCL entry points across ranks, bit-exact against the oracle (GPU).

fhe_bcast_key (the one collective of the multi-GPU path) and
fhe_reduce_ranks (the cross-rank ReduceTask join, §8f-3) are driven on the
communicator of PyTorch's RCCL process group -- the one bench.py hands to
fhe_bcast_key.  World 1 runs on any GPU box; world 2 needs two GPUs and skips
otherwise (RCCL refuses two ranks on one device).  Each rank is its own
process (tests/rccl_ranks.py).
"""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "rccl_ranks.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for r, (rc, out) in enumerate(outs):
        assert rc == 0 and f"rank {r} ok" in out, out[-3000:]


def test_rccl_world1_torch_communicator():
    import torch
    assert torch.cuda.device_count() >= 1
    _run(1)


def test_rccl_world2_bcast_and_reduce_ranks():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    _run(2)
