"""Probe: does running the two-pass N=2^16 forward NTT over chunks of limbs
(column pass then row pass per chunk, so a chunk's intermediate can stay in the
256 MiB Infinity Cache) beat one launch pair over all limbs?

    python tools/ntt_chunk_probe.py [--limbs 4608]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--limbs", type=int, default=4608)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import herdsman_amd.backend as hb

    L, n = 12, 1 << 16
    ctx = hb.Context(hb.SCHEME_CKKS, 16, L)
    s = torch.cuda.current_stream()
    ctx.set_stream(s)
    polys = args.limbs // L
    x = hb.empty((polys, L, n))
    ctx.fill_uniform(x, seed=1)
    for chunk_polys in (polys, 64, 32, 16, 8, 4):
        def run():
            for p0 in range(0, polys, chunk_polys):
                ctx.ntt_fwd(x[p0:p0 + chunk_polys])
        for _ in range(2):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.reps):
            run()
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        mib = chunk_polys * L * n * 8 / 2**20
        print(f"chunk {chunk_polys * L:5d} limbs ({mib:6.0f} MiB): {ms:.3f} ms per {args.limbs} limbs, "
              f"frac {args.limbs * 2 * n * 8 / (ms * 1e-3) / 8e12:.4f}", flush=True)


if __name__ == "__main__":
    main()
