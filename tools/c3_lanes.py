"""C3 BFV mul+relin throughput (N=2^15, L=8, BEHZ) with the batch split over S
concurrent contexts, one stream each (the C5 headline's lane structure): the
latency-bound BEHZ kernels of one lane overlap the VALU-bound transforms of
another.  Prints ct-mult/s per (lanes, per-lane batch).

    python tools/c3_lanes.py [--reps 20] [--hps]
"""
import argparse
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--hps", action="store_true")
    args = ap.parse_args()
    import torch
    import herdsman_amd.backend as hb

    dev = torch.device("cuda:0")
    kw = dict(t=65537, device=0, **({"bfv_mult": "hps"} if args.hps else {}))
    n3 = 1 << 15
    for S, Bs in ((1, 128), (2, 64), (4, 32), (2, 128), (4, 64)):
        lanes = []
        for i in range(S):
            c = hb.Context(hb.SCHEME_BFV, 15, 8, 4, 2, **kw)
            s = torch.cuda.current_stream(dev) if i == 0 else torch.cuda.Stream(dev)
            c.set_stream(s)
            a = c.fill_uniform(hb.empty((Bs, 2, 8, n3), device=dev), seed=31 + i)
            b = c.fill_uniform(hb.empty((Bs, 2, 8, n3), device=dev), seed=41 + i)
            k = c.fill_uniform(hb.empty(c.key_shape(), device=dev), seed=33)
            o = hb.empty((Bs, 2, 8, n3), device=dev)
            lanes.append((c, s, a, b, k, o))
        for c, s, a, b, k, o in lanes:  # warm (workspaces)
            c.mul_relin(a, b, k, o)
        torch.cuda.synchronize(dev)
        main_s = lanes[0][1]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        for _, s, *_ in lanes[1:]:
            s.wait_event(e0)
        for _ in range(args.reps):
            for c, s, a, b, k, o in lanes:
                c.mul_relin(a, b, k, o)
        for _, s, *_ in lanes[1:]:
            ev = torch.cuda.Event()
            ev.record(s)
            main_s.wait_event(ev)
        e1.record(main_s)
        e1.synchronize()
        dt = e0.elapsed_time(e1) * 1e-3
        print(f"lanes {S} x {Bs}: {S * Bs * args.reps / dt:.1f} ct-mult/s ({dt / args.reps * 1e3:.3f} ms per step of {S * Bs})",
              flush=True)
        for c, *_ in lanes:
            c.close()
        del lanes
        torch.cuda.synchronize(dev)


if __name__ == "__main__":
    main()
