"""Probe: the two-pass N=2^16 forward NTT over chunks of limbs dealt
round-robin to S streams (one context each), so a chunk's column-pass output
is re-read by its row pass while it is still in the 256 MiB Infinity Cache and
the next chunk's column pass overlaps the previous chunk's row pass.

    python tools/ntt_stream_chunk_probe.py [--limbs 4608]
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
    dev = torch.device("cuda", 0)
    main_s = torch.cuda.current_stream()
    polys = args.limbs // L
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    ctxs = []
    for st in streams:
        c = hb.Context(hb.SCHEME_CKKS, 16, L)
        c.set_stream(st)
        ctxs.append(c)
    x = hb.empty((polys, L, n))
    ctxs[0].fill_uniform(x, seed=1)
    torch.cuda.synchronize()
    for S in (1, 2, 3, 4):
        for chunk_polys in (polys, 64, 32, 16, 8):
            if S > 1 and chunk_polys == polys:
                continue

            def run():
                ev = torch.cuda.Event()
                ev.record(main_s)
                for st in streams[:S]:
                    st.wait_event(ev)
                for i, p0 in enumerate(range(0, polys, chunk_polys)):
                    ctxs[i % S].ntt_fwd(x[p0:p0 + chunk_polys])
                for st in streams[:S]:
                    e = torch.cuda.Event()
                    e.record(st)
                    main_s.wait_event(e)

            for _ in range(2):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            for _ in range(args.reps):
                run()
            e1.record(main_s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            mib = chunk_polys * L * n * 8 / 2**20
            print(f"streams {S} chunk {chunk_polys * L:5d} limbs ({mib:6.0f} MiB): {ms:.3f} ms per {args.limbs} "
                  f"limbs, frac {args.limbs * 2 * n * 8 / (ms * 1e-3) / 8e12:.4f}", flush=True)


if __name__ == "__main__":
    main()
