"""Throughput of S concurrent contexts/streams (one process), each running
ct-mult+relin on its own batch: does concurrent kernel execution help?

    python tools/streams_probe.py --streams 2 --batch 128 --steps 10
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import herdsman_amd.backend as hb

    dev = torch.device("cuda", 0)
    ctxs, bufs = [], []
    rlk = None
    for s in range(args.streams):
        c = hb.Context(hb.SCHEME_CKKS, 16, 12, 4, 3, device=0)
        st = torch.cuda.Stream(dev)
        c.set_stream(st)
        c.reserve(args.batch)
        if rlk is None:
            rlk = hb.empty(c.key_shape(), device=dev)
            c.fill_uniform(rlk, seed=1)
        shape = (args.batch, 2, 12, 1 << 16)
        a = c.fill_uniform(hb.empty(shape, device=dev), seed=2 + s)
        b = c.fill_uniform(hb.empty(shape, device=dev), seed=3 + s)
        ctxs.append((c, st))
        bufs.append((a, b, hb.empty(shape, device=dev)))
    torch.cuda.synchronize(dev)

    def step():
        for (c, st), (a, b, o) in zip(ctxs, bufs):
            c.mul_relin(a, b, rlk, o)

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    print(f"streams {args.streams} batch {args.batch}: {args.streams * args.batch * args.steps / dt:.1f} ct-mult/s")


if __name__ == "__main__":
    main()
