"""Micro-benchmark of the NTT passes and KS kernels (GPU box).

    python tools/ntt_bench.py [--log-n 16] [--limbs 1152] [--openfhe-primes]
Prints limb-NTT/s for forward and inverse transforms and the achieved
algorithmic bandwidth (2 * N * 8 bytes per limb-NTT).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, nargs="+", default=[14, 16])
    ap.add_argument("--limbs", type=int, default=1152)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--openfhe-primes", action="store_true", help="q = 1 mod 2N (generic Montgomery path)")
    args = ap.parse_args()
    import torch
    import herdsman_amd.backend as hb

    for log_n in args.log_n:
        n = 1 << log_n
        L = 12
        mods = None
        if args.openfhe_primes:
            from herdsman_amd.params import openfhe_style_primes
            mods = openfhe_style_primes([(60, L)], log_n)
        ctx = hb.Context(hb.SCHEME_CKKS, log_n, L, moduli=mods)
        s = torch.cuda.current_stream()
        ctx.set_stream(s)
        polys = max(1, args.limbs // L)
        x = hb.empty((polys, L, n))
        ctx.fill_uniform(x, seed=1)
        for name, fn in (("fwd", ctx.ntt_fwd), ("inv", ctx.ntt_inv)):
            for _ in range(3):
                fn(x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                fn(x)
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            limbs = polys * L
            rate = limbs / (ms * 1e-3)
            gbs = limbs * 2 * n * 8 / (ms * 1e-3) / 1e9
            print(f"log_n={log_n} {name}: {ms:.3f} ms for {limbs} limbs -> {rate/1e6:.3f} M limb-NTT/s, "
                  f"{gbs:.0f} GB/s algorithmic ({gbs/8000*100:.1f}% of 8 TB/s)")


if __name__ == "__main__":
    main()
