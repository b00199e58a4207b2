"""Time one ciphertext op at a BASELINE config (GPU box), for rocprofv3 runs.

    python tools/op_bench.py bfv_mul|ckks_mul|ckks_rot|ckks_hrot|bfv_rot|bfv_hrot [--batch 32] [--reps 10]
                             [--openfhe-primes]

*_hrot: --rot (default 4) hoisted rotations of the batch (fhe_rotate_hoisted); the rate counts rotations.
*_rsum: the sum of --rot rotations with one ModDown (fhe_rotate_sum_hoisted); the rate counts rotations.
ckks_lin: the hoisted linear transform of --rot plaintext-weighted rotations (fhe_linear_hoisted).

--openfhe-primes: the CKKS ops on OpenFHE-style primes (q = 1 mod 2N, generic
Montgomery path) instead of the default q = 1 (mod 2^32) family.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("op", choices=["bfv_mul", "bfv_hps_mul", "ckks_mul", "ckks_rot", "ckks_hrot", "bfv_rot", "bfv_hrot",
                                       "ckks_rsum", "bfv_rsum", "ckks_lin"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--openfhe-primes", action="store_true")
    ap.add_argument("--rot", type=int, default=4, help="Galois elements per hoisted call (*_hrot)")
    args = ap.parse_args()
    import torch
    import herdsman_amd.backend as hb

    if args.op.startswith("bfv"):
        # bfv_hps_*: the HPS multiplication (fhe_params FHE_FLAG_BFV_HPS)
        kw = {"bfv_mult": "hps"} if args.op.startswith("bfv_hps") else {}
        c = hb.Context(hb.SCHEME_BFV, 15, 8, 4, 2, t=65537, **kw)
        if args.op.startswith("bfv_hps"):
            args.op = "bfv" + args.op[len("bfv_hps"):]
    else:
        mods = None
        if args.openfhe_primes:
            from herdsman_amd.params import openfhe_style_primes
            mods = openfhe_style_primes([(60, 12), (61, 4)], 16)
        c = hb.Context(hb.SCHEME_CKKS, 16, 12, 4, 3, moduli=mods)
    s = torch.cuda.current_stream()
    c.set_stream(s)
    shape = (args.batch, 2, c.L, c.n)
    a = c.fill_uniform(hb.empty(shape), seed=1)
    b = c.fill_uniform(hb.empty(shape), seed=2)
    k = c.fill_uniform(hb.empty(c.key_shape()), seed=3)
    out = hb.empty(shape)
    g = c.galois_elt(1)
    gs = [c.galois_elt(s_) for s_ in range(1, args.rot + 1)]
    outs = [hb.empty(shape) for _ in gs] if args.op.endswith("hrot") else []
    per = len(gs) if args.op.endswith(("hrot", "rsum", "lin")) else 1
    pts = [c.fill_uniform(hb.empty((c.L + c.K, c.n)), seed=10 + i) for i in range(len(gs))] \
        if args.op == "ckks_lin" else []
    fn = {"bfv_mul": lambda: c.mul_relin(a, b, k, out), "ckks_mul": lambda: c.mul_relin(a, b, k, out),
          "ckks_rot": lambda: c.rotate(a, g, k, out), "bfv_rot": lambda: c.rotate(a, g, k, out),
          "ckks_hrot": lambda: c.rotate_hoisted(a, gs, [k] * len(gs), outs),
          "bfv_hrot": lambda: c.rotate_hoisted(a, gs, [k] * len(gs), outs),
          "ckks_rsum": lambda: c.rotate_sum_hoisted(a, gs, [k] * len(gs), out),
          "bfv_rsum": lambda: c.rotate_sum_hoisted(a, gs, [k] * len(gs), out),
          "ckks_lin": lambda: c.linear_hoisted(a, gs, [k] * len(gs), pts, out)}[args.op]
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    print(f"{args.op}: {dt * 1e3:.3f} ms per call of {args.batch} -> {per * args.batch / dt:.1f} ops/s")


if __name__ == "__main__":
    main()
