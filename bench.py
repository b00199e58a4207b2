#!/usr/bin/env python3
"""Headline benchmark: CKKS ct-mult+relin/s at N=2^16, L=12 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

One step = one fhe_mul_relin call over B independent ciphertext pairs per GPU
(N=2^16, L=12 primes of 60 bits, K=4 special primes of 61 bits, dnum=3 hybrid
key switching), inputs already resident in HBM (generated on device with the
backend's SplitMix64 fill).  Multi-GPU: one process per GPU (torchrun), the
relinearisation key is generated on rank 0 and broadcast once over RCCL
(the only collective), then every rank works on its own shard with no
communication ("scaling": "weak").  value = ct-mults of all ranks / max-rank time.

Extra fields:
  roofline     -- the dominant kernel group, the forward NTT (column + row pass
                  kernels, one fhe_ntt_fwd launch over the batch's limbs),
                  timed with HIP events on the backend's stream; algorithmic
                  bytes = 2 * N * 8 per limb-NTT (read + write the residue once).
  cpu_baseline -- the CPU oracle (oracle/fhe_oracle.c, OpenMP over ciphertexts)
                  on a bounded sample of the same workload, rank 0 at N=1 only.
  secondary    -- per-GPU throughput of the other BASELINE configs: C4 rotate,
                  C3 BFV mul+relin, C2 NTT (not part of `value`).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "ct-mult+relin/sec at N=2^16 L=12; achieved HBM GB/s vs 8 TB/s peak"
LOG_N, L, K, DNUM = 16, 12, 4, 3
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128, help="ct-mults per GPU per step")
    ap.add_argument("--ntt-reps", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=4096, help="max ct-mults in the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline duration")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--graph", type=int, default=0, help="1: replay the step from a captured HIP graph")
    ap.add_argument("--streams", type=int, default=4,
                    help="contexts (one HIP stream each) that share a step's batch and run concurrently")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary measurements (C4 rotate, C3 BFV mul+relin, C2 NTT)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the timed NTT loop (for rocprofv3 runs of the dominant kernel)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "ntt_traffic.json"))
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import herdsman_amd.backend as hb
    from herdsman_amd.dist import broadcast_key, max_over_ranks
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

    ctx = hb.Context(hb.SCHEME_CKKS, LOG_N, L, K, DNUM, device=gpu)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream)
    n = 1 << LOG_N
    B = args.batch
    # S concurrent contexts, one HIP stream each, split the step's batch: kernels of
    # different stages (VALU-bound NTT passes, HBM-bound conversions) overlap across
    # the GPU's hardware queues (4 x 32 vs 1 x 128: +5%)
    S = 1 if args.graph else max(1, min(args.streams, B))
    if B % S:
        raise SystemExit(f"--batch {B} is not a multiple of --streams {S}")
    Bs = B // S
    ctx.reserve(B)
    lanes = [(ctx, stream)]
    for _ in range(S - 1):
        c_i = hb.Context(hb.SCHEME_CKKS, LOG_N, L, K, DNUM, device=gpu)
        s_i = torch.cuda.Stream(dev)
        c_i.set_stream(s_i)
        c_i.reserve(Bs)
        lanes.append((c_i, s_i))

    # relinearisation key: rank 0 makes it, RCCL broadcast to everyone else
    rlk = hb.empty(ctx.key_shape(), device=dev)
    if rank == 0:
        ctx.fill_uniform(rlk, seed=0x524C4B)
    torch.cuda.synchronize(dev)
    t_b = time.perf_counter()
    broadcast_key(rlk, src=0)  # the only collective: RCCL over xGMI
    torch.cuda.synchronize(dev)
    key_bcast_ms = (time.perf_counter() - t_b) * 1e3

    a = hb.empty((B, 2, L, n), device=dev)
    b = hb.empty((B, 2, L, n), device=dev)
    out = hb.empty((B, 2, L, n), device=dev)
    ctx.fill_uniform(a, seed=0x48455244 ^ (rank << 32) ^ 1)
    ctx.fill_uniform(b, seed=0x48455244 ^ (rank << 32) ^ 2)

    torch.cuda.synchronize(dev)  # inputs were filled on the first context's stream

    def step():
        for i, (c_i, _) in enumerate(lanes):
            c_i.mul_relin(a[i * Bs:(i + 1) * Bs], b[i * Bs:(i + 1) * Bs], rlk, out[i * Bs:(i + 1) * Bs])

    if args.graph and not args.roofline_only:
        # capture one step (~25 kernel launches) into a HIP graph and replay it:
        # the workspace was pre-sized by ctx.reserve, so nothing allocates
        ctx.mul_relin(a, b, rlk, out)  # warm
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            ctx.set_stream(torch.cuda.current_stream(dev))
            ctx.mul_relin(a, b, rlk, out)
        ctx.set_stream(stream)
        step = graph.replay

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
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = max_over_ranks(time.perf_counter() - t0, device=dev)
    total = world * B * steps
    value = total / elapsed if steps else 0.0

    # ---- dominant kernel group: forward NTT over the ModUp-sized batch (36 limbs per ct)
    limbs = B * 3 * L  # the converted limbs of one batch's ModUp
    x = hb.empty((limbs, 1, n), device=dev)
    ctx.fill_uniform(x.view(B * 3, L, n), seed=99)
    for _ in range(3):
        ctx.ntt_fwd(x.view(B * 3, L, n))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    reps = max(1, args.ntt_reps)
    for _ in range(reps):
        ctx.ntt_fwd(x.view(B * 3, L, n))
    e1.record(stream)
    e1.synchronize()
    ntt_ms = e0.elapsed_time(e1) / reps
    algo_bytes = limbs * 2 * n * 8
    achieved = algo_bytes / (ntt_ms * 1e-3) / 1e9
    traffic = valu_busy = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get("hbm_bytes_per_limb_ntt")
            valu_busy = tj.get("valu_busy")
            if traffic is not None:
                traffic = traffic * limbs
        except Exception:
            traffic = None
    ntt_limb_per_s = limbs / (ntt_ms * 1e-3)

    secondary = None
    if not (args.roofline_only or args.no_secondary):
        secondary = secondary_configs(hb, ctx, rlk, a, out, dev, stream, B, max(2, args.steps // 2))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, ctx)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "ct-mult/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(steps, 1) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: uniform residues mod q (on-device SplitMix64), uniform relin key",
            "config": {
                "workload": "ckks_mul_relin",
                "log_n": LOG_N, "L": L, "K": K, "dnum": DNUM,
                "q_bits": 60, "p_bits": 61,
                "batch_per_gpu": B, "global_batch": B * world,
                "parallelism": f"shard{world}", "streams_per_gpu": S,
            },
            "roofline": {
                "kernel": "ntt_fwd (ntt_pass col + row), N=2^16",
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes": algo_bytes,
                "launch_ms": round(ntt_ms, 4),
                # the NTT is integer-VALU bound, not HBM bound: share of the
                # SIMDs' issue slots running VALU work (PMC, profiles/)
                "valu_busy": valu_busy,
            },
            "ntt_fwd_limb_per_s": round(ntt_limb_per_s, 1),
            "key_bcast_ms": round(key_bcast_ms, 3),
            "algorithmic_GBps_ct_mult": round(value / world * 6 * L * n * 8 / 1e9, 1),
            "cpu_baseline": cpu,
            "secondary": secondary,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


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


def secondary_configs(hb, ctx, gk, ct, out, dev, stream, B, reps):
    """Per-GPU throughput of the other BASELINE.json configs (same synthetic-data rules):
    C4 CKKS rotate + hybrid KS at the metric parameters (B ciphertexts per call),
    C3 BFV mul+relin at N=2^15 L=8 (BEHZ), C2 forward+inverse NTT at N=2^14 L=4."""
    res = {}
    g = ctx.galois_elt(1)
    t = _timed(lambda: ctx.rotate(ct, g, gk, out), reps, stream)
    res["C4_ckks_rotate_per_s"] = round(B / t, 1)
    bfv = hb.Context(hb.SCHEME_BFV, 15, 8, 4, 2, t=65537, device=dev.index)
    bfv.set_stream(stream)
    n3 = 1 << 15
    a3 = bfv.fill_uniform(hb.empty((B, 2, 8, n3), device=dev), seed=31)
    b3 = bfv.fill_uniform(hb.empty((B, 2, 8, n3), device=dev), seed=32)
    k3 = bfv.fill_uniform(hb.empty(bfv.key_shape(), device=dev), seed=33)
    o3 = hb.empty((B, 2, 8, n3), device=dev)
    t = _timed(lambda: bfv.mul_relin(a3, b3, k3, o3), reps, stream)
    res["C3_bfv_mul_relin_per_s"] = round(B / t, 1)
    del a3, b3, k3, o3
    bfv.close()
    c2 = hb.Context(hb.SCHEME_CKKS, 14, 4, device=dev.index)
    c2.set_stream(stream)
    polys = 256
    x2 = c2.fill_uniform(hb.empty((polys, 4, 1 << 14), device=dev), seed=21)
    t = _timed(lambda: (c2.ntt_fwd(x2), c2.ntt_inv(x2)), reps, stream)
    res["C2_ntt_fwd_inv_poly_per_s"] = round(polys / t, 1)
    res["C2_limb_ntt_per_s"] = round(2 * 4 * polys / t, 1)
    c2.close()
    return res


def cpu_baseline(args, ctx):
    """CPU oracle (test infrastructure) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_ffi import Oracle, SCHEME_CKKS

    o = Oracle(SCHEME_CKKS, LOG_N, L, K, DNUM, moduli=ctx.moduli)
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    o.lib.orc_set_threads(threads)
    s = max(threads, 1)
    a = o.uniform((s, 2, L, 1 << LOG_N), seed=1)
    b = o.uniform((s, 2, L, 1 << LOG_N), seed=2)
    k = o.uniform(o.key_shape(), seed=3)
    done, t0 = 0, time.perf_counter()
    while True:  # ~args.cpu_seconds of CPU work, at least two rounds
        o.mul_relin(a, b, k)
        done += s
        dt = time.perf_counter() - t0
        if (dt >= args.cpu_seconds and done >= 2 * s) or done >= args.cpu_sample:
            break
    return {
        "value": round(done / dt, 3),
        "unit": "ct-mult/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} CKKS ct-mult+relin at N=2^16 L=12 K=4 dnum=3 in {dt:.1f} s "
                  f"(batches of {s}, OpenMP one ciphertext per thread)",
    }


if __name__ == "__main__":
    main()
