#!/usr/bin/env python3
"""Headline benchmark: CKKS ct-mult+relin/s at N=2^16, L=12 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch G] [--batch B]

Workload (BASELINE.json configs[4], "C5"): a batch of G = 8192 independent
ct-mult+relin at N=2^16, L=12 primes of 60 bits, K=4 special primes of 61 bits,
dnum=3 hybrid key switching.  The batch is sharded over the ranks with
herdsman's partition rule (dist.shard_range: floor(G/N) each, +1 for the first
G mod N ranks; /root/reference/src/service/storage_service.cpp:121-129), one
process per GPU; every rank processes its shard in waves of B ct-mults, each
wave split over S concurrent contexts (one HIP stream each).  One step = the
whole G-ct batch; "scaling" is "strong" (total work fixed as N grows).

Memory: 8192 ciphertext pairs plus outputs are 288 GiB, more than one GPU's
HBM, so each rank keeps a resident pool of up to --pool distinct input pairs
and output slots (36 GiB at 1024) generated ON THE DEVICE, and its waves walk
through the pool (at N=8 a rank's 1024 ct-mults all have distinct inputs).
Inputs are resident in HBM before the timed region; nothing is skipped inside it.

Multi-GPU: `--gpus N` without a torchrun environment spawns N fresh worker
processes (one per GPU, MASTER_ADDR 127.0.0.1) before anything touches the GPU;
under torchrun (RANK/WORLD_SIZE set) the process is one rank.  Rank 0 generates
the relinearisation key and broadcasts it once with fhe_bcast_key on PyTorch's
RCCL communicator (the same librccl instance the backend binds to) -- the only
collective; afterwards each rank works alone.  value = G * steps / max-rank time.

Extra fields:
  roofline     -- the dominant kernel group, the forward NTT (column + row pass
                  kernels, one fhe_ntt_fwd launch over B*3*L limbs), timed with
                  HIP events on the stream the kernels run on; algorithmic bytes
                  = 2 * N * 8 per limb-NTT.  frac_rocprof recomputes the same
                  fraction from the committed rocprofv3 kernel averages, and
                  traffic is the PMC-counted HBM bytes (profiles/, see "profile").
  cpu_baseline -- the CPU oracle (oracle/fhe_oracle.c, OpenMP, threads pinned) on
                  a bounded sample of the same workload, in a child process on
                  the host's cores (rank 0, N=1 only); also C2/C3/C4 samples.
  secondary    -- per-GPU throughput of the other BASELINE configs (C4 rotate,
                  C3 BFV mul+relin by BEHZ and by HPS, C2 NTT) and the metric
                  config on OpenFHE-style primes (generic Montgomery path).
  step         -- the headline op's own roofline: rocprofv3-counted HBM bytes per
                  ct-mult (profiles/step_traffic.json), the fraction of peak the
                  measured rate moves with them, the dominant kernel of a wave.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "ct-mult+relin/sec at N=2^16 L=12; achieved HBM GB/s vs 8 TB/s peak"
LOG_N, L, K, DNUM = 16, 12, 4, 3
HBM_PEAK_GBS = 8000.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--global-batch", type=int, default=8192, help="ct-mults per step over all ranks (C5)")
    ap.add_argument("--batch", type=int, default=128, help="ct-mults per wave per GPU")
    ap.add_argument("--pool", type=int, default=1024, help="distinct resident input pairs per GPU")
    ap.add_argument("--no-stagger", action="store_true", help="lanes start in phase (see wave_plan)")
    ap.add_argument("--streams", type=int, default=4,
                    help="contexts (one HIP stream each) that share a wave and run concurrently")
    ap.add_argument("--ntt-reps", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline duration (metric)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every core this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary measurements (C4 rotate, C3 BFV, C2 NTT, generic moduli)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the timed NTT loop (for rocprofv3 runs of the dominant kernel)")
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / sharding / timing control flow only, on CPU (gloo), no GPU work")
    ap.add_argument("--profile-json", default=os.path.join(ROOT, "profiles", "ntt_traffic.json"))
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def launch(args) -> int:
    """Parent of an N-GPU run started without torchrun: spawn one fresh process
    per GPU (this process never initialises the GPU), wait, relay the exit code.
    If a rank fails, the others are stopped (they would wait in a collective)."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in procs:
                    q.terminate()
        time.sleep(0.2)
    return rc


def _rccl_comm(dev):
    """(ncclComm_t of PyTorch's RCCL process group on `dev`, error text): the
    backend's fhe_bcast_key must use a communicator of the librccl instance it
    is bound to, which in a torch process is torch's own.
    A failed hand-off is returned as an error string, never swallowed: the
    bench line reports it (key_bcast_error) and stderr says so."""
    import torch.distributed as dist
    try:
        be = dist.group.WORLD._get_backend(dev)
        if not hasattr(be, "_comm_ptr"):
            return 0, f"{type(be).__name__} has no _comm_ptr (torch {__import__('torch').__version__})"
        comm = int(be._comm_ptr())
        return comm, None if comm else "_comm_ptr() returned 0"
    except Exception as e:  # reported, not hidden
        return 0, f"{type(e).__name__}: {e}"


def _key_digest(key, dev):
    """Per-rank checksum of the key words (a torch reduction on the device), so
    the line can state that every rank holds the same key after the broadcast."""
    import torch
    w = key.view(torch.int64)
    return int(torch.bitwise_xor(w[0::2], w[1::2]).sum().item()) & ((1 << 64) - 1)


# -------------------------------------------------------------------- ranks
def main():
    args = parse()
    if args.cpu_baseline_child:
        print(json.dumps(cpu_baseline_child(args)), flush=True)
        return 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args)
    if args.dry_run:
        return dry_run(args)

    import torch
    import torch.distributed as dist

    import herdsman_amd.backend as hb
    from herdsman_amd.dist import broadcast_key, max_over_ranks, shard_range
    from herdsman_amd.dist import world as dist_world

    rank, local, world = dist_world()
    # HERD_BENCH_DIST=gloo rehearses the multi-rank control flow with several ranks
    # sharing the GPUs there are (the real runs use RCCL, one rank per GPU)
    backend = os.environ.get("HERD_BENCH_DIST", "nccl")
    gpu = local % torch.cuda.device_count() if backend == "gloo" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    devices = [gpu]
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, gpu)
    n_gpus = len(set(devices))

    # ---- shard of the C5 batch and its wave / pool geometry
    G = args.global_batch
    my, B, S, waves, P, Bs, plan = wave_plan(G, args.batch, args.streams, args.pool, world, rank,
                                              not args.no_stagger)
    full_secondary = world == 1 and not (args.roofline_only or args.no_secondary)

    n = 1 << LOG_N
    ctx = hb.Context(hb.SCHEME_CKKS, LOG_N, L, K, DNUM, device=gpu)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream)
    ctx.reserve(B if full_secondary else Bs)  # the secondary calls run whole waves on lane 0
    lanes = [(ctx, stream)]
    for _ in range(S - 1):
        c_i = hb.Context(hb.SCHEME_CKKS, LOG_N, L, K, DNUM, device=gpu)
        s_i = torch.cuda.Stream(dev)
        c_i.set_stream(s_i)
        c_i.reserve(Bs)
        lanes.append((c_i, s_i))

    # ---- relinearisation key: rank 0 makes it, one RCCL broadcast to the others
    # (seeded like the committed metric digest case, so that every rank can
    # check its own outputs against that digest with the key it RECEIVED)
    rlk = hb.empty(ctx.key_shape(), device=dev)
    if rank == 0:
        ctx.fill_uniform(rlk, seed=SELF_CHECK["seed_key"])
    torch.cuda.synchronize(dev)
    bcast, bcast_err, key_ok = "none (1 rank)", None, True
    if world > 1:
        dist.barrier()
    t_b = time.perf_counter()
    if world > 1:
        comm, bcast_err = _rccl_comm(dev) if backend == "nccl" else (0, None)
        if comm:
            ctx.bcast_key(rlk, comm, root=0)  # fhe_bcast_key: ncclBroadcast over xGMI
            bcast = "fhe_bcast_key (RCCL)"
        else:
            if bcast_err:
                print(f"bench.py: RCCL communicator hand-off failed ({bcast_err}); "
                      "broadcasting the key through torch.distributed instead", file=sys.stderr, flush=True)
            broadcast_key(rlk, src=0)
            bcast = f"torch.distributed.broadcast ({backend})"
    torch.cuda.synchronize(dev)
    key_bcast_ms = (time.perf_counter() - t_b) * 1e3
    if world > 1:
        digests = [None] * world
        dist.all_gather_object(digests, _key_digest(rlk, dev))
        key_ok = len(set(digests)) == 1
        if not key_ok:
            print(f"bench.py: key digests differ across ranks after the broadcast: {digests}", file=sys.stderr)
            return 3

    a = hb.empty((P, 2, L, n), device=dev)
    b = hb.empty((P, 2, L, n), device=dev)
    out = hb.empty((P, 2, L, n), device=dev)
    ctx.fill_uniform(a, seed=0x48455244 ^ (rank << 32) ^ 1)
    ctx.fill_uniform(b, seed=0x48455244 ^ (rank << 32) ^ 2)
    torch.cuda.synchronize(dev)  # inputs were filled on the first context's stream

    def step():
        for i, lo, hi in plan:
            lanes[i][0].mul_relin(a[lo:hi], b[lo:hi], rlk, out[lo:hi])

    steps = 0 if args.roofline_only else args.steps
    for _ in range(0 if args.roofline_only else args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    mine = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = max_over_ranks(mine, device=dev)
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, (my * steps / mine) if mine > 0 else 0.0)
    else:
        per_rank = [(my * steps / mine) if mine > 0 else 0.0]
    value = G * steps / elapsed if steps else 0.0
    # every rank's shard (first row, size) and the ct-mults its step actually
    # issued: the line shows each rank's share, and a plan that does not cover
    # the global batch exactly once fails the run (exit 5)
    shard = {"first": shard_range(G, world, rank)[0], "size": my, "issued": sum(hi - lo for _, lo, hi in plan)}
    shards = [shard]
    if world > 1:
        shards = [None] * world
        dist.all_gather_object(shards, shard)
    shards_ok = (sum(s_["issued"] for s_ in shards) == G and all(s_["issued"] == s_["size"] for s_ in shards)
                 and all(shards[r]["first"] + shards[r]["size"] == (shards[r + 1]["first"] if r + 1 < world else G)
                         for r in range(world)))

    # ---- dominant kernel group: forward NTT over the ModUp-sized wave (36 limbs per ct),
    # right after the timed steps: the timed launches follow the warm-up ones with no
    # idle gap at 1 rank (an idle GPU re-ramps its clock: +1.5% on the launch time)
    limbs = B * 3 * L
    x = hb.empty((B * 3, L, n), device=dev)
    ctx.fill_uniform(x, seed=99)
    if world > 1:
        # every rank's NTT loop runs at the same time (the N-GPU NTT/s); the barrier
        # comes BEFORE the warm-up launches, so no rank idles (and re-ramps its clock)
        # between them and the timed ones
        torch.cuda.synchronize(dev)
        dist.barrier()
    for _ in range(3):
        ctx.ntt_fwd(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)  # the stream the NTT kernels are launched on (ctx.set_stream above)
    reps = max(1, args.ntt_reps)
    for _ in range(reps):
        ctx.ntt_fwd(x)
    e1.record(stream)
    e1.synchronize()
    ntt_ms = e0.elapsed_time(e1) / reps
    del x
    ntt_rates = [limbs / (ntt_ms * 1e-3)]
    if world > 1:
        ntt_rates = [None] * world
        dist.all_gather_object(ntt_rates, limbs / (ntt_ms * 1e-3))
    # ---- per-rank output check: every lane context of every rank recomputes the
    # committed metric digest case with the broadcast key (after the timed regions)
    mine_ok = rank_self_check(hb, lanes, rlk, dev)
    per_rank_ok = [mine_ok]
    if world > 1:
        per_rank_ok = [None] * world
        dist.all_gather_object(per_rank_ok, mine_ok)

    algo_per_limb = 2 * n * 8
    algo_bytes = limbs * algo_per_limb
    achieved = algo_bytes / (ntt_ms * 1e-3) / 1e9
    roof = {
        "kernel": "ntt_fwd (ntt_pass col + row), N=2^16",
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None,
        "algorithmic_bytes": algo_bytes,
        "launch_ms": round(ntt_ms, 4),
    }
    roof.update(profile_fields(args.profile_json, limbs, algo_per_limb))
    roof.update(copy_cap_fields(roof["frac"]))

    secondary = None
    if full_secondary:
        secondary = secondary_configs(hb, ctx, rlk, a, b, out, dev, stream, B, max(2, 2 * args.steps))

    cpu = None
    if rank == 0 and world == 1 and not (args.no_cpu or args.roofline_only):
        cpu = run_cpu_baseline(args)
        if "digest_2ct" in cpu:
            cpu["gpu_bitexact_2ct"] = gpu_digest_2ct(hb, ctx, dev) == cpu["digest_2ct"]

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "ct-mult/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(steps, 1) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: uniform residues mod q (on-device SplitMix64), uniform relin key",
            "config": {
                "workload": f"C5: {G} independent CKKS ct-mult+relin per step, sharded over {world} rank(s)",
                "log_n": LOG_N, "L": L, "K": K, "dnum": DNUM,
                "q_bits": 60, "p_bits": 61,
                "global_batch": G, "batch_per_gpu": my, "batch_per_rank": [s_["size"] for s_ in shards],
                "shard_first_per_rank": [s_["first"] for s_ in shards],
                "issued_per_step_per_rank": [s_["issued"] for s_ in shards], "shards_cover_batch": shards_ok,
                "wave": B, "waves_per_step": waves,
                "resident_pool": P, "streams_per_gpu": S,
                "parallelism": f"shard{world}", "ranks": world,
            },
            "roofline": roof,
            "ntt_fwd_limb_per_s": round(limbs / (ntt_ms * 1e-3), 1),
            # all ranks' NTT loops at once (N=2^16 limb-NTTs per second over the node)
            "ntt_fwd_limb_per_s_all_gpus": round(sum(ntt_rates), 1),
            "ntt_fwd_limb_per_s_per_rank": [round(v, 1) for v in ntt_rates],
            "per_rank_ct_mult_per_s": [round(v, 1) for v in per_rank],
            "key_bcast_ms": round(key_bcast_ms, 3),
            "key_bcast_via": bcast,
            "key_bcast_error": bcast_err,
            "key_identical_on_all_ranks": key_ok,
            "per_rank_bitexact": [bool(v["ok"]) for v in per_rank_ok],
            "per_rank_check": {"case": SELF_CHECK["case"], "lanes": [v["lanes"] for v in per_rank_ok],
                               "source": "tests/golden/digests.json (CPU oracle, make_digests.py)"},
            "algorithmic_GBps_ct_mult": round(value / n_gpus * 6 * L * n * 8 / 1e9, 1),
            "step": step_fields(value / n_gpus, 6 * L * n * 8),
            "cpu_baseline": cpu,
            "secondary": secondary,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not shards_ok:
        if rank == 0:
            print(f"bench.py: the ranks' shards do not cover the global batch {G} exactly once: {shards}",
                  file=sys.stderr, flush=True)
        return 5
    if not all(v["ok"] for v in per_rank_ok):
        if rank == 0:
            print(f"bench.py: output digest mismatch on rank(s) "
                  f"{[r for r, v in enumerate(per_rank_ok) if not v['ok']]}", file=sys.stderr, flush=True)
        return 4
    return 0


def _load_self_check():
    """The metric digest case of tests/golden (committed SHA-256 of the CPU
    oracle's output on SplitMix64 inputs with fixed seeds)."""
    case = "metric_ckks_mul_relin_n65536_l12"
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))[case]
    # the seeds of tests/golden/full_size_cases.py (SEED_A, SEED_B, SEED_KEY)
    return {"case": case, "sha256": d["sha256"], "moduli": d["moduli"],
            "seed_a": 0x48455244, "seed_b": 0x48455245, "seed_key": 0x4B4559}


SELF_CHECK = _load_self_check()


def rank_self_check(hb, lanes, rlk, dev):
    """{"ok", "lanes"}: each lane context's product of the digest case's inputs
    (generated on the device) with this rank's copy of the key hashes to the
    committed digest.  A wrong-but-fast rank, a lane whose context diverged or a
    corrupted key broadcast fails the run (exit 4)."""
    import hashlib

    import torch
    n = 1 << LOG_N
    res = []
    for c, s in lanes:
        if [int(q) for q in c.moduli] != SELF_CHECK["moduli"]:
            res.append(False)
            continue
        a = c.fill_uniform(hb.empty((1, 2, L, n), device=dev), seed=SELF_CHECK["seed_a"])
        b = c.fill_uniform(hb.empty((1, 2, L, n), device=dev), seed=SELF_CHECK["seed_b"])
        y = hb.empty((1, 2, L, n), device=dev)
        c.mul_relin(a, b, rlk, y)
        torch.cuda.synchronize(dev)
        res.append(hashlib.sha256(hb.to_host(y).tobytes()).hexdigest() == SELF_CHECK["sha256"])
    return {"ok": bool(res) and all(res), "lanes": res}


def wave_plan(G, batch, streams, pool, world, rank, stagger=True):
    """This rank's shard of a G-ct batch (herdsman's partition rule) as waves of
    `batch` ct-mults over `streams` lanes, on a resident pool of P slots (a
    multiple of the wave).  Returns (my, B, S, waves, P, Bs, plan) with plan =
    [(lane, lo, hi)] pool slices in issue order.

    Each lane owns P/S pool slots and a near-equal share of the shard, which it
    runs in calls of Bs = B/S ciphertexts.  With `stagger`, lane i's first call
    is (i+1)/S of a full one: the lanes run the same kernel sequence, so
    without an offset their NTT passes (VALU-bound) and their conversions and
    products (HBM-bound) would run at the same time on every stream; offset by
    a quarter of a call each, different kernel types overlap on the GPU."""
    from herdsman_amd.dist import shard_range

    b0, b1 = shard_range(G, world, rank)
    my = b1 - b0
    B = max(1, min(batch, my)) if my else 1
    S = max(1, min(streams, B))
    waves = math.ceil(my / B) if my else 0
    P = min(max(pool // B, 1), max(waves, 1)) * B
    Bs = math.ceil(B / S)
    PL = P // S  # pool slots per lane (>= Bs: P is a multiple of B)
    lanes = []
    for i in range(S):
        l0, l1 = shard_range(my, S, i)
        total, calls = l1 - l0, []
        first = max(1, (Bs * (i + 1)) // S) if stagger else Bs
        o = 0
        while total > 0:
            c = min(first if not calls else Bs, total)
            if o + c > PL:
                o = 0
            calls.append((i, i * PL + o, i * PL + o + c))
            o += c
            total -= c
        lanes.append(calls)
    plan = []
    for k in range(max((len(c) for c in lanes), default=0)):
        for calls in lanes:
            if k < len(calls):
                plan.append(calls[k])
    return my, B, S, waves, P, Bs, plan


def dry_run(args):
    """The multi-rank control flow without a GPU (tests/test_multi_rank.py): process
    group (gloo), shard / wave plan, barriers, max-over-ranks timing, rank-0 line."""
    import torch.distributed as dist

    from herdsman_amd.dist import max_over_ranks
    from herdsman_amd.dist import world as dist_world

    rank, local, world = dist_world()
    if world > 1:
        dist.init_process_group("gloo")
    my, B, S, waves, P, Bs, plan = wave_plan(args.global_batch, args.batch, args.streams, args.pool, world, rank)
    covered = sum(hi - lo for _, lo, hi in plan)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    elapsed = max_over_ranks(time.perf_counter() - t0)
    shards = [(rank, my, covered, os.getpid(), local)]
    if world > 1:
        shards = [None] * world
        dist.all_gather_object(shards, (rank, my, covered, os.getpid(), local))
    per_rank = [s[1] / elapsed if elapsed > 0 else 0.0 for s in sorted(shards)]
    if rank == 0:
        print(json.dumps({"dry_run": True, "ranks": world, "shards": shards, "wave": B, "waves": waves,
                          "pool": P, "lanes": S, "elapsed": elapsed, "steps": args.steps, "warmup": args.warmup,
                          "n_gpus": len({s[4] for s in shards}), "per_rank_ct_mult_per_s": per_rank,
                          "value": args.global_batch / elapsed if elapsed > 0 else 0.0}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def profile_fields(path, limbs, algo_per_limb):
    """The committed rocprofv3 evidence for the roofline kernels (tools/collect_profile.py):
    the kernel-trace average launch time -> frac_rocprof, the PMC bytes -> traffic."""
    try:
        pj = json.load(open(path))
    except (OSError, ValueError):
        return {"profile": None}
    res = {"profile": pj.get("source")}
    per_limb = pj.get("hbm_bytes_per_limb_ntt")
    if per_limb:
        res["traffic"] = round(per_limb * limbs)
        res["traffic_per_limb_ntt"] = round(per_limb)
        # not measured in this run: the PMC bytes per limb-NTT of the committed
        # rocprofv3 passes (FETCH_SIZE x2 + WRITE_SIZE) times this call's limbs
        res["traffic_source"] = f"{os.path.relpath(path, ROOT)} (rocprofv3 --pmc, committed)"
    launch_ns, plimbs = pj.get("ntt_fwd_launch_ns"), pj.get("limbs_per_launch")
    if launch_ns and plimbs:
        res["rocprof_launch_ms"] = round(launch_ns / 1e6, 4)
        res["frac_rocprof"] = round(plimbs * algo_per_limb / (launch_ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
    if pj.get("valu_busy") is not None:
        res["valu_busy"] = pj["valu_busy"]
    return res


def copy_cap_fields(frac):
    """What the roofline kernel can reach with its access pattern: a two-pass NTT
    moves every word through HBM twice, and a pure copy with the column-pass and
    row-pass patterns (profiles/copy_cap.json, committed microbenchmark) bounds
    each pass.  cap_frac = algorithmic bytes / (both copy times) / peak."""
    try:
        cc = json.load(open(os.path.join(ROOT, "profiles", "copy_cap.json")))
    except (OSError, ValueError):
        return {}
    algo = cc["limbs"] * 2 * (1 << LOG_N) * 8
    cap = algo / ((cc["col_pass_copy_ms"] + cc["row_pass_copy_ms"]) * 1e-3) / 1e9 / HBM_PEAK_GBS
    return {"cap_frac": round(cap, 4), "frac_of_cap": round(frac / cap, 4),
            "bound_note": "HBM with the two-pass access pattern (column pass of 128 B row segments, then row "
                          "pass): cap_frac is a pure copy with those patterns; VALU co-bound (valu_busy)",
            "cap_source": "profiles/copy_cap.json (" + cc["source"] + ")"}


def step_fields(per_gpu_value, algo_bytes_per_ct):
    """The headline op's own roofline: HBM bytes per ct-mult
    counted by rocprofv3 (FETCH_SIZE x2 + WRITE_SIZE over every kernel of a
    128-ct mul+relin wave, profiles/step_traffic.json, tools/step_summary.py),
    the fraction of peak the measured headline rate moves with those bytes and
    with the algorithmic ones, and the dominant kernel of the wave."""
    res = {"algorithmic_bytes_per_ct_mult": algo_bytes_per_ct,
           "headline_frac_algorithmic": round(per_gpu_value * algo_bytes_per_ct / 1e9 / HBM_PEAK_GBS, 4)}
    try:
        st = json.load(open(os.path.join(ROOT, "profiles", "step_traffic.json")))
    except (OSError, ValueError):
        return res
    b = st["hbm_bytes_per_ct_mult"]
    res.update({"hbm_bytes_per_ct_mult": b,
                "headline_GBps_counted_bytes": round(per_gpu_value * b / 1e9, 1),
                "headline_frac_counted_bytes": round(per_gpu_value * b / 1e9 / HBM_PEAK_GBS, 4),
                "wave_kernel_ms": st["kernel_ms_per_wave"], "wave_kernel_TBps": st["kernel_TBps"],
                "dominant_kernel": st["dominant"], "source": st["source"] + " (rocprofv3, committed)"})
    return res


def _timed(fn, reps, stream):
    import torch
    fn()  # warm (workspace, caches)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def secondary_configs(hb, ctx, gk, a, b, out, dev, stream, B, reps):
    """Per-GPU throughput of the other BASELINE.json configs (same synthetic-data rules):
    C4 CKKS rotate + hybrid KS at the metric parameters (B ciphertexts per call) and
    4 hoisted rotations of the same batch (fhe_rotate_hoisted, one ModUp of c1) and the
    double-hoisted sum of 16 rotations (fhe_rotate_sum_hoisted, one ModUp and one ModDown),
    C3 BFV mul+relin at N=2^15 L=8 (BEHZ), C2 forward+inverse NTT at N=2^14 L=4, and
    the metric op on OpenFHE-style primes (q = 1 mod 2N, generic Montgomery path)
    next to the same single-context call on the default primes."""
    from herdsman_amd.params import openfhe_style_primes

    res = {}
    g = ctx.galois_elt(1)
    ct, o = a[:B], out[:B]
    t = _timed(lambda: ctx.rotate(ct, g, gk, o), reps, stream)
    res["C4_ckks_rotate_per_s"] = round(B / t, 1)
    # hoisted: 4 Galois elements over the same B ciphertexts, one ModUp of c1
    # (rotations per second = 4 B / t; the same key stands in for the 4 keys)
    gs = [ctx.galois_elt(s) for s in (1, 2, -1, 5)]
    hos = [hb.empty((B, 2, L, 1 << LOG_N), device=dev) for _ in gs]
    t = _timed(lambda: ctx.rotate_hoisted(ct, gs, [gk] * len(gs), hos), reps, stream)
    res["C4_ckks_rotate_hoisted4_rot_per_s"] = round(len(gs) * B / t, 1)
    del hos
    # double-hoisted sum of 16 rotations (one ModUp, one ModDown): rotations per second summed
    g16 = [ctx.galois_elt(s_) for s_ in range(1, 17)]
    t = _timed(lambda: ctx.rotate_sum_hoisted(ct, g16, [gk] * len(g16), o), reps, stream)
    res["C4_ckks_rotate_sum16_rot_per_s"] = round(len(g16) * B / t, 1)
    t = _timed(lambda: ctx.mul_relin(ct, b[:B], gk, o), reps, stream)
    res["C5_mul_relin_1ctx_per_s"] = round(B / t, 1)
    # the CKKS multiply as a circuit runs it: mul+relin then rescale (12 -> 11 limbs),
    # and the same product one level down (mul_relin_at on 11-limb ciphertexts)
    r11 = hb.empty((B, 2, L - 1, 1 << LOG_N), device=dev)
    t = _timed(lambda: (ctx.mul_relin(ct, b[:B], gk, o), ctx.rescale(o, r11, L)), reps, stream)
    res["C5_mul_relin_rescale_1ctx_per_s"] = round(B / t, 1)
    a11 = r11.clone()
    t = _timed(lambda: ctx.mul_relin_at(a11, r11, gk, a11, L - 1), reps, stream)
    res["C5_mul_relin_level11_1ctx_per_s"] = round(B / t, 1)
    del r11, a11
    mods = openfhe_style_primes([(60, L), (61, K)], LOG_N)
    gen = hb.Context(hb.SCHEME_CKKS, LOG_N, L, K, DNUM, moduli=mods, device=dev.index)
    gen.set_stream(stream)
    gen.reserve(B)
    ga = gen.fill_uniform(hb.empty((B, 2, L, 1 << LOG_N), device=dev), seed=41)
    gb = gen.fill_uniform(hb.empty((B, 2, L, 1 << LOG_N), device=dev), seed=42)
    gkey = gen.fill_uniform(hb.empty(gen.key_shape(), device=dev), seed=43)
    t = _timed(lambda: gen.mul_relin(ga, gb, gkey, o), reps, stream)
    res["C5_mul_relin_openfhe_primes_1ctx_per_s"] = round(B / t, 1)
    del ga, gb, gkey
    gen.close()
    bfv = hb.Context(hb.SCHEME_BFV, 15, 8, 4, 2, t=65537, device=dev.index)
    bfv.set_stream(stream)
    n3 = 1 << 15
    a3 = bfv.fill_uniform(hb.empty((B, 2, 8, n3), device=dev), seed=31)
    b3 = bfv.fill_uniform(hb.empty((B, 2, 8, n3), device=dev), seed=32)
    k3 = bfv.fill_uniform(hb.empty(bfv.key_shape(), device=dev), seed=33)
    o3 = hb.empty((B, 2, 8, n3), device=dev)
    t = _timed(lambda: bfv.mul_relin(a3, b3, k3, o3), reps, stream)
    res["C3_bfv_mul_relin_per_s"] = round(B / t, 1)
    bfv.close()
    hps = hb.Context(hb.SCHEME_BFV, 15, 8, 4, 2, t=65537, device=dev.index, bfv_mult="hps")
    hps.set_stream(stream)
    t = _timed(lambda: hps.mul_relin(a3, b3, k3, o3), reps, stream)
    res["C3_bfv_hps_mul_relin_per_s"] = round(B / t, 1)
    del a3, b3, k3, o3
    hps.close()
    c2 = hb.Context(hb.SCHEME_CKKS, 14, 4, device=dev.index)
    c2.set_stream(stream)
    polys = 256
    x2 = c2.fill_uniform(hb.empty((polys, 4, 1 << 14), device=dev), seed=21)
    t = _timed(lambda: (c2.ntt_fwd(x2), c2.ntt_inv(x2)), reps, stream)
    res["C2_ntt_fwd_inv_poly_per_s"] = round(polys / t, 1)
    res["C2_limb_ntt_per_s"] = round(2 * 4 * polys / t, 1)
    c2.close()
    return res


# --------------------------------------------------------------- CPU baseline
def _host_cores():
    """(cores this process may use, nproc, cgroup CPU quota or None, CPU model)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    return cores, aff, quota, model


def gpu_digest_2ct(hb, ctx, dev):
    """SHA-256 of the GPU's first two products of the CPU baseline's sample (the
    same SplitMix64 seeds, generated on the device): equal to the child's digest
    iff the two outputs agree bit for bit."""
    import hashlib

    import torch
    n = 1 << LOG_N
    a = ctx.fill_uniform(hb.empty((2, 2, L, n), device=dev), seed=1)
    b = ctx.fill_uniform(hb.empty((2, 2, L, n), device=dev), seed=2)
    k = ctx.fill_uniform(hb.empty(ctx.key_shape(), device=dev), seed=3)
    out = hb.empty((2, 2, L, n), device=dev)
    ctx.mul_relin(a, b, k, out)
    torch.cuda.synchronize(dev)
    return hashlib.sha256(hb.to_host(out).tobytes()).hexdigest()


def run_cpu_baseline(args):
    """The oracle in a child process (no GPU, no torch) so that its OpenMP threads
    can be pinned (OMP_PROC_BIND / OMP_PLACES are read when libgomp starts)."""
    cores, aff, quota, model = _host_cores()
    threads = args.cpu_threads or cores
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores")
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--cpu-threads", str(threads),
           "--cpu-seconds", str(args.cpu_seconds)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res.update({"cores": threads, "nproc": aff, "cgroup_cpu_quota": quota, "cpu_model": model,
                "pinning": "OMP_PROC_BIND=close OMP_PLACES=cores"})
    return res


def cpu_baseline_child(args):
    """CPU oracle (test infrastructure) on bounded samples of the bench workloads."""
    import hashlib

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_ffi import Oracle, SCHEME_BFV, SCHEME_CKKS

    threads = max(1, args.cpu_threads)

    def timed(fn, per_call, seconds):
        done, t0 = 0, time.perf_counter()
        while True:
            fn()
            done += per_call
            dt = time.perf_counter() - t0
            if dt >= seconds and done >= 2 * per_call:
                return done, dt

    o = Oracle(SCHEME_CKKS, LOG_N, L, K, DNUM)
    o.lib.orc_set_threads(threads)
    a = o.uniform((threads, 2, L, 1 << LOG_N), seed=1)
    b = o.uniform((threads, 2, L, 1 << LOG_N), seed=2)
    k = o.uniform(o.key_shape(), seed=3)
    done, dt = timed(lambda: o.mul_relin(a, b, k), threads, args.cpu_seconds)
    res = {
        "value": round(done / dt, 3),
        "unit": "ct-mult/s",
        "kind": "port",
        "sample": f"{done} CKKS ct-mult+relin at N=2^16 L=12 K=4 dnum=3 in {dt:.1f} s "
                  f"(batches of {threads}, OpenMP one ciphertext per thread)",
        # the CPU and GPU outputs of the same inputs are compared in
        # the same run; the GPU side recomputes the first two products (main())
        "digest_2ct": hashlib.sha256(np.ascontiguousarray(o.mul_relin(a[:2], b[:2], k)).tobytes()).hexdigest(),
    }
    sec = {}
    g = o.galois_elt(1)
    done, dt = timed(lambda: o.rotate(a, g, k), threads, 3.0)
    sec["C4_ckks_rotate_per_s"] = round(done / dt, 3)
    gs = [o.galois_elt(s_) for s_ in (1, 2, -1, 5)]
    k4 = np.stack([k] * len(gs))
    done, dt = timed(lambda: o.rotate_hoisted(a, gs, k4), len(gs) * threads, 3.0)
    sec["C4_ckks_rotate_hoisted4_rot_per_s"] = round(done / dt, 3)
    del k4
    g16 = [o.galois_elt(s_) for s_ in range(1, 17)]
    k16 = np.stack([k] * len(g16))
    done, dt = timed(lambda: o.rotate_sum_hoisted(a, g16, k16), len(g16) * threads, 3.0)
    sec["C4_ckks_rotate_sum16_rot_per_s"] = round(done / dt, 3)
    del k16
    del a, b, k
    o3 = Oracle(SCHEME_BFV, 15, 8, 4, 2, t=65537)
    a3 = o3.uniform((threads, 2, 8, 1 << 15), seed=31)
    b3 = o3.uniform((threads, 2, 8, 1 << 15), seed=32)
    k3 = o3.uniform(o3.key_shape(), seed=33)
    done, dt = timed(lambda: o3.mul_relin(a3, b3, k3), threads, 3.0)
    sec["C3_bfv_mul_relin_per_s"] = round(done / dt, 3)
    del a3, b3, k3
    o2 = Oracle(SCHEME_CKKS, 14, 4)
    polys = 4 * threads
    x2 = o2.uniform((polys, 4, 1 << 14), seed=21)
    done, dt = timed(lambda: o2.ntt_inv(o2.ntt_fwd(x2)), polys, 3.0)
    sec["C2_ntt_fwd_inv_poly_per_s"] = round(done / dt, 3)
    res["secondary"] = sec
    return res


if __name__ == "__main__":
    sys.exit(main())
