"""Generate the committed golden vectors from the independent big-int model.

    python tests/golden/make_golden.py

Every fixture is (inputs, expected outputs) computed by
oracle/bigint_model.py with Python integers.  They pin the C oracle
(tests/test_oracle_golden.py) and the HIP backend (tests/test_gpu_parity.py).
No reference code is involved: herdsman has no FHE arithmetic to run
(SURVEY.md §0), so parity vs herdsman/OpenFHE is "unpinned" and these vectors
pin the implementation to the mathematical definitions instead.
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import bigint_model as M  # noqa: E402


def rand_limbs(rng, mods, n):
    return [[rng.randrange(q) for _ in range(n)] for q in mods]


def arr(x):
    return np.array(x, dtype=np.uint64)


def gen_ntt(rng):
    log_n = 10
    n = 1 << log_n
    mods = M.gen_primes(60, log_n, 3)
    p = M.Params(log_n, 3, 0, 1, mods)
    x = rand_limbs(rng, mods, n)
    y = p.ntt(x, range(3))
    # the fast model NTT must agree with the O(N^2) definition
    small = M.Params(6, 1, 0, 1, M.gen_primes(60, 6, 1))
    xs = [rng.randrange(small.moduli[0]) for _ in range(64)]
    assert M.ntt_fwd(xs, small.moduli[0], small.psi[0]) == M.ntt_fwd_direct(xs, small.moduli[0], small.psi[0])
    assert p.intt(y, range(3)) == x
    # negacyclic product theorem
    a, b = x[0], x[1][:]
    q = mods[0]
    lhs = M.ntt_inv([u * v % q for u, v in zip(M.ntt_fwd(a, q, p.psi[0]), M.ntt_fwd(b, q, p.psi[0]))], q, p.psi[0])
    assert lhs == M.negacyclic_mul(a, b, q)
    np.savez(os.path.join(HERE, "ntt_n1024.npz"), log_n=np.uint32(log_n), moduli=arr(mods),
             psi=arr(p.psi), x=arr(x), y=arr(y))


def gen_conv(rng):
    log_n = 10
    n = 1 << log_n
    mods = M.gen_primes(60, log_n, 4) + M.gen_primes(61, log_n, 3)
    src, dst = [0, 1, 2, 3], [4, 5, 6]
    x = rand_limbs(rng, [mods[i] for i in src], n)
    y = M.base_conv(x, [mods[i] for i in src], [mods[i] for i in dst])
    np.savez(os.path.join(HERE, "conv_n1024.npz"), log_n=np.uint32(log_n), moduli=arr(mods),
             src=np.array(src, dtype=np.uint32), dst=np.array(dst, dtype=np.uint32), x=arr(x), y=arr(y))


def gen_ckks(rng):
    log_n, L, K, dnum = 10, 4, 2, 2
    n = 1 << log_n
    Q = M.gen_primes(60, log_n, L)
    P = M.gen_primes(61, log_n, K, exclude=Q)
    p = M.Params(log_n, L, K, dnum, Q + P, "ckks")
    a = [rand_limbs(rng, Q, n) for _ in range(2)]
    b = [rand_limbs(rng, Q, n) for _ in range(2)]
    rlk = [[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(dnum)]
    gk = [[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(dnum)]
    out_mul = M.ckks_mul_relin(p, a, b, rlk)
    g = M.galois_elt(log_n, 3)
    out_rot = M.rotate(p, a, g, gk)
    g_conj = 2 * n - 1
    out_conj = M.rotate(p, b, g_conj, gk)
    np.savez(os.path.join(HERE, "ckks_n1024_l4.npz"), log_n=np.uint32(log_n), L=np.uint32(L), K=np.uint32(K),
             dnum=np.uint32(dnum), moduli=arr(Q + P), a=arr(a), b=arr(b), rlk=arr(rlk), gk=arr(gk),
             out_mul=arr(out_mul), g=np.uint32(g), out_rot=arr(out_rot), g_conj=np.uint32(g_conj),
             out_conj=arr(out_conj))


def gen_bfv(rng):
    log_n, L, K, dnum, t = 10, 4, 2, 2, 65537
    n = 1 << log_n
    Q = M.gen_primes(60, log_n, L)
    P = M.gen_primes(61, log_n, K, exclude=Q)
    Bsk = M.gen_primes(61, log_n, L + 1, exclude=Q + P)
    p = M.Params(log_n, L, K, dnum, Q + P + Bsk, "bfv", t)
    a = [rand_limbs(rng, Q, n) for _ in range(2)]
    b = [rand_limbs(rng, Q, n) for _ in range(2)]
    rlk = [[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(dnum)]
    out_mul = M.bfv_mul_relin(p, a, b, rlk)
    out_add = [[[(x + y) % Q[i] for x, y in zip(a[c][i], b[c][i])] for i in range(L)] for c in range(2)]
    g = M.galois_elt(log_n, 1)
    out_rot = M.rotate(p, a, g, rlk)
    np.savez(os.path.join(HERE, "bfv_n1024_l4.npz"), log_n=np.uint32(log_n), L=np.uint32(L), K=np.uint32(K),
             dnum=np.uint32(dnum), t=np.uint64(t), moduli=arr(Q + P + Bsk), a=arr(a), b=arr(b), rlk=arr(rlk),
             out_mul=arr(out_mul), out_add=arr(out_add), g=np.uint32(g), out_rot=arr(out_rot))


def gen_bfv_hoisted(rng):
    """Hoisted BFV rotations (coefficient form) for steps 1, -3 and the
    conjugation-like element 2N - 1, each with its own key."""
    log_n, L, K, dnum, t = 10, 4, 2, 2, 65537
    n = 1 << log_n
    Q = M.gen_primes(60, log_n, L)
    P = M.gen_primes(61, log_n, K, exclude=Q)
    Bsk = M.gen_primes(61, log_n, L + 1, exclude=Q + P)
    p = M.Params(log_n, L, K, dnum, Q + P + Bsk, "bfv", t)
    ct = [rand_limbs(rng, Q, n) for _ in range(2)]
    gs = [M.galois_elt(log_n, 1), M.galois_elt(log_n, -3), 2 * n - 1]
    gks = [[[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(dnum)] for _ in gs]
    out = M.rotate_hoisted(p, ct, gs, gks)
    np.savez(os.path.join(HERE, "bfv_hoisted_n1024_l4.npz"), log_n=np.uint32(log_n), L=np.uint32(L),
             K=np.uint32(K), dnum=np.uint32(dnum), t=np.uint64(t), moduli=arr(Q + P + Bsk), ct=arr(ct),
             galois=np.array(gs, dtype=np.uint32), gks=arr(gks), out=arr(out))


def gen_rotation_sums(rng):
    """Double-hoisted rotation sums (one ModDown for all the elements): CKKS N=1024
    L=5 and BFV N=1024 L=4, three elements each with their own keys."""
    out = {}
    log_n, n = 10, 1 << 10
    Q = M.gen_primes(60, log_n, 5)
    P = M.gen_primes(61, log_n, 2, exclude=Q)
    p = M.Params(log_n, 5, 2, 2, Q + P)
    ct = [rand_limbs(rng, Q, n) for _ in range(2)]
    gs = [M.galois_elt(log_n, 1), M.galois_elt(log_n, 3), 2 * n - 1]
    gks = [[[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(2)] for _ in gs]
    pts = [rand_limbs(rng, Q + P, n) for _ in gs]
    out["ckks"] = dict(moduli=arr(Q + P), ct=arr(ct), galois=np.array(gs, dtype=np.uint32), gks=arr(gks),
                       out=arr(M.rotate_sum_hoisted(p, ct, gs, gks)), pts=arr(pts),
                       lin=arr(M.linear_hoisted(p, ct, gs, gks, pts)))
    Qb = M.gen_primes(60, log_n, 4)
    Pb = M.gen_primes(61, log_n, 2, exclude=Qb)
    Bsk = M.gen_primes(61, log_n, 5, exclude=Qb + Pb)
    pb = M.Params(log_n, 4, 2, 2, Qb + Pb + Bsk, "bfv", 65537)
    ctb = [rand_limbs(rng, Qb, n) for _ in range(2)]
    gksb = [[[rand_limbs(rng, Qb + Pb, n) for _ in range(2)] for _ in range(2)] for _ in gs]
    out["bfv"] = dict(moduli=arr(Qb + Pb + Bsk), ct=arr(ctb), galois=np.array(gs, dtype=np.uint32), gks=arr(gksb),
                      out=arr(M.rotate_sum_hoisted(pb, ctb, gs, gksb)))
    np.savez(os.path.join(HERE, "rotation_sum_n1024.npz"), log_n=np.uint32(log_n),
             **{f"{s}_{k}": v for s, d in out.items() for k, v in d.items()})


def gen_bfv_hps(rng):
    """BFV mul+relin by HPS (oracle/bigint_model.py bfv_mul_relin_hps, which also
    checks each scaled tensor output against round(t d / Q) on integers)."""
    log_n, L, K, dnum, t = 10, 4, 2, 2, 65537
    n = 1 << log_n
    Q = M.gen_primes(60, log_n, L)
    P = M.gen_primes(61, log_n, K, exclude=Q)
    Bsk = M.gen_primes(61, log_n, L + 1, exclude=Q + P)
    p = M.Params(log_n, L, K, dnum, Q + P + Bsk, "bfv", t)
    a = [rand_limbs(rng, Q, n) for _ in range(2)]
    b = [rand_limbs(rng, Q, n) for _ in range(2)]
    rlk = [[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(dnum)]
    out_mul = M.bfv_mul_relin_hps(p, a, b, rlk)
    np.savez(os.path.join(HERE, "bfv_hps_n1024_l4.npz"), log_n=np.uint32(log_n), L=np.uint32(L), K=np.uint32(K),
             dnum=np.uint32(dnum), t=np.uint64(t), moduli=arr(Q + P + Bsk), a=arr(a), b=arr(b), rlk=arr(rlk),
             out_mul=arr(out_mul))


def gen_ckks_hoisted(rng):
    """Hoisted CKKS rotations (one ModUp of c1, sigma_g on the extensions) for
    steps 1, -3 and conjugation, each with its own key."""
    log_n, L, K, dnum = 10, 5, 2, 2
    n = 1 << log_n
    Q = M.gen_primes(60, log_n, L)
    P = M.gen_primes(61, log_n, K, exclude=Q)
    p = M.Params(log_n, L, K, dnum, Q + P, "ckks")
    ct = [rand_limbs(rng, Q, n) for _ in range(2)]
    gs = [M.galois_elt(log_n, 1), M.galois_elt(log_n, -3), 2 * n - 1]
    gks = [[[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(dnum)] for _ in gs]
    out = M.rotate_hoisted(p, ct, gs, gks)
    np.savez(os.path.join(HERE, "ckks_hoisted_n1024_l5.npz"), log_n=np.uint32(log_n), L=np.uint32(L),
             K=np.uint32(K), dnum=np.uint32(dnum), moduli=arr(Q + P), ct=arr(ct),
             galois=np.array(gs, dtype=np.uint32), gks=arr(gks), out=arr(out))


def gen_ckks_levels(rng):
    """CKKS at reduced levels: L = 5 primes, alpha = 3 (dnum 2), so level 4 has
    a partial second digit, level 3 one full digit and level 2 one partial
    digit; mul+relin / rotate with the full-level key's Q_lvl u P rows, and the
    rescale chain 5 -> 4 -> 3 by its integer definition."""
    log_n, L, K, dnum = 10, 5, 2, 2
    n = 1 << log_n
    Q = M.gen_primes(60, log_n, L)
    P = M.gen_primes(61, log_n, K, exclude=Q)
    p = M.Params(log_n, L, K, dnum, Q + P, "ckks")
    rlk = [[rand_limbs(rng, Q + P, n) for _ in range(2)] for _ in range(dnum)]
    res = {}
    for lvl in (4, 2):
        a = [rand_limbs(rng, Q[:lvl], n) for _ in range(2)]
        b = [rand_limbs(rng, Q[:lvl], n) for _ in range(2)]
        res[f"a{lvl}"], res[f"b{lvl}"] = arr(a), arr(b)
        res[f"mul{lvl}"] = arr(M.ckks_mul_relin_at(p, a, b, rlk, lvl))
    a3 = [rand_limbs(rng, Q[:3], n) for _ in range(2)]
    g = M.galois_elt(log_n, 5)
    c0 = [M.automorph_ntt(x, g) for x in a3[0]]
    c1 = [M.automorph_ntt(x, g) for x in a3[1]]
    ks0, ks1 = M.keyswitch(p, c1, rlk, True, 3)
    res["a3"], res["rot3"] = arr(a3), arr([[[(x + y) % Q[i] for x, y in zip(c0[i], ks0[i])] for i in range(3)], ks1])
    c5 = [rand_limbs(rng, Q, n) for _ in range(2)]
    r4 = M.rescale(p, c5, 5)
    r3 = M.rescale(p, r4, 4)
    res["c5"], res["r4"], res["r3"] = arr(c5), arr(r4), arr(r3)
    np.savez(os.path.join(HERE, "ckks_levels_n1024_l5.npz"), log_n=np.uint32(log_n), L=np.uint32(L),
             K=np.uint32(K), dnum=np.uint32(dnum), moduli=arr(Q + P), rlk=arr(rlk), g=np.uint32(g), **res)


def main():
    rng = random.Random(0x48455244)
    gen_ntt(rng)
    gen_conv(rng)
    gen_ckks(rng)
    gen_bfv(rng)
    gen_ckks_levels(random.Random(0x4C564C53))
    gen_bfv_hps(random.Random(0x485053))
    gen_ckks_hoisted(random.Random(0x484F4953))
    gen_bfv_hoisted(random.Random(0x42484F49))
    gen_rotation_sums(random.Random(0x52534D))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    if sys.argv[1:] == ["levels"]:  # only the level fixture (the others are unchanged)
        gen_ckks_levels(random.Random(0x4C564C53))
    elif sys.argv[1:] == ["hps"]:
        gen_bfv_hps(random.Random(0x485053))
    elif sys.argv[1:] == ["hoisted"]:
        gen_ckks_hoisted(random.Random(0x484F4953))
    elif sys.argv[1:] == ["hoisted_bfv"]:
        gen_bfv_hoisted(random.Random(0x42484F49))
    elif sys.argv[1:] == ["rotation_sums"]:
        gen_rotation_sums(random.Random(0x52534D))
    else:
        main()
