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


def _run(world, G, batch, streams, pool, timeout=400):
    env = dict(os.environ, HERD_BENCH_DIST="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--global-batch", str(G),
           "--batch", str(batch), "--streams", str(streams), "--pool", str(pool), "--steps", "2", "--warmup", "1",
           "--no-cpu", "--no-secondary", "--ntt-reps", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_line(line, world, G, streams):
    from herdsman_amd.dist import shard_range

    cfg = line["config"]
    assert cfg["ranks"] == world
    assert cfg["global_batch"] == G
    assert cfg["batch_per_gpu"] == shard_range(G, world, 0)[1]
    # every rank's shard is herdsman's partition rule (storage_service.cpp:121-129),
    # and the waves each rank issued cover its shard exactly
    sh = [shard_range(G, world, r) for r in range(world)]  # (first row, end row)
    assert cfg["batch_per_rank"] == [e - b for b, e in sh]
    assert cfg["shard_first_per_rank"] == [b for b, _ in sh]
    assert cfg["issued_per_step_per_rank"] == cfg["batch_per_rank"]
    assert sum(cfg["batch_per_rank"]) == G and cfg["shards_cover_batch"] is True
    assert line["per_rank_bitexact"] == [True] * world
    assert line["per_rank_check"]["lanes"] == [[True] * streams] * world


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_bench_rehearsal_checks_every_rank(world):
    G = 24 * world + 3  # ragged: the first G mod world ranks own one more
    line = _run(world, G, batch=16, streams=2, pool=16)
    _check_line(line, world, G, 2)
    assert len(line["per_rank_ct_mult_per_s"]) == world and min(line["per_rank_ct_mult_per_s"]) > 0
    assert line["key_identical_on_all_ranks"] is True
    assert line["n_gpus"] == 1  # the ranks share the box's one device
    assert line["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_sharded_bench_rehearsal_driver_shape_eight_ranks():
    """The driver's N = 8 shape: 8 ranks, 4 lanes each, on the
    box's one device over gloo, a ragged batch (8 * 16 + 5: five ranks own 17).
    Every rank's shard, issued work and all 4 lane digests are checked."""
    world, G = 8, 8 * 16 + 5
    line = _run(world, G, batch=16, streams=4, pool=16, timeout=560)
    _check_line(line, world, G, 4)
    assert len(line["per_rank_ct_mult_per_s"]) == world and min(line["per_rank_ct_mult_per_s"]) > 0
    assert len(line["ntt_fwd_limb_per_s_per_rank"]) == world
    assert line["key_identical_on_all_ranks"] is True
    assert line["n_gpus"] == 1
