"""Rehearsal of the sharded C5 bench on one GPU, with the HIP path.

`bench.py --gpus N` under HERD_BENCH_DIST=gloo runs N ranks that share the one
device of the box and exchange host-staged tensors over gloo (RCCL refuses two
ranks on one device).  Everything else is the driver's multi-GPU path: the
spawned ranks, herdsman's partition rule for the shards, the key broadcast from
rank 0, the waves over the lanes, max-over-ranks timing and, per rank, the
self-check of every lane context against the committed metric digest
(tests/golden/digests.json) with the key that rank received.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(world, G, batch, streams, pool):
    env = dict(os.environ, HERD_BENCH_DIST="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--global-batch", str(G),
           "--batch", str(batch), "--streams", str(streams), "--pool", str(pool), "--steps", "2", "--warmup", "1",
           "--no-cpu", "--no-secondary", "--ntt-reps", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_bench_rehearsal_checks_every_rank(world):
    from herdsman_amd.dist import shard_range

    G = 24 * world + 3  # ragged: the first G mod world ranks own one more
    line = _run(world, G, batch=16, streams=2, pool=16)
    assert line["config"]["ranks"] == world
    assert line["config"]["global_batch"] == G
    assert line["config"]["batch_per_gpu"] == shard_range(G, world, 0)[1]
    assert line["per_rank_bitexact"] == [True] * world
    assert all(lanes == [True, True] for lanes in line["per_rank_check"]["lanes"])
    assert len(line["per_rank_ct_mult_per_s"]) == world and min(line["per_rank_ct_mult_per_s"]) > 0
    assert line["key_identical_on_all_ranks"] is True
    assert line["n_gpus"] == 1  # the ranks share the box's one device
    assert line["value"] > 0
