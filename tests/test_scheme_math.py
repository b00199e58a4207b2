"""Scheme-level ground truth for the oracle with REAL keys.

Decrypt(MulRelin(Enc(m1), Enc(m2))) and Decrypt(Rotate(Enc(m))) are checked
with exact CRT reconstruction against the integer negacyclic product /
automorphism.  These identities pin the key-switching
algorithm itself, independently of any golden vector.
"""
import math
import random

import numpy as np
import pytest

from fhe_math import automorph_int, crt_centered, negacyclic_int, to_rns
from oracle_ffi import Oracle, SCHEME_BFV, SCHEME_CKKS


def _keys(o, seed=11):
    s = o.secret(seed)
    s_qp = o.signed_to_rns(s, 0, o.L + o.K, ntt=True)
    return s, s_qp


def _square_ntt(o, s_qp):
    out = np.zeros_like(s_qp)
    for i in range(o.L + o.K):
        q = int(o.moduli[i])
        out[i] = np.array([(int(x) * int(x)) % q for x in s_qp[i]], dtype=np.uint64)
    return out


def test_ckks_mul_relin_decrypts():
    o = Oracle(SCHEME_CKKS, 10, 4, 2, 2)
    Q = [int(q) for q in o.moduli[:o.L]]
    s, s_qp = _keys(o)
    rlk = o.switch_key(_square_ntt(o, s_qp), s_qp, seed=5)
    rng = random.Random(1)
    delta = 1 << 30
    u1 = [rng.randint(-8, 8) for _ in range(o.n)]
    u2 = [rng.randint(-8, 8) for _ in range(o.n)]
    c1 = o.encrypt(to_rns([delta * x for x in u1], Q), s_qp, 101)
    c2 = o.encrypt(to_rns([delta * x for x in u2], Q), s_qp, 202)
    prod = o.mul_relin(c1[None], c2[None], rlk)[0]
    dec = crt_centered(o.decrypt(prod, s_qp), Q)
    want = [delta * delta * v for v in negacyclic_int(u1, u2)]
    err = max(abs(a - b) for a, b in zip(dec, want))
    assert err < 2 ** 56, math.log2(err + 1)


def test_ckks_rotate_decrypts():
    o = Oracle(SCHEME_CKKS, 10, 4, 2, 2)
    Q = [int(q) for q in o.moduli[:o.L]]
    s, s_qp = _keys(o)
    rng = random.Random(2)
    delta = 1 << 40
    u = [rng.randint(-100, 100) for _ in range(o.n)]
    ct = o.encrypt(to_rns([delta * x for x in u], Q), s_qp, 303)
    for steps in (1, 5, -3):
        g = o.galois_elt(steps)
        s_g = o.automorph_ntt(s_qp, g)
        gk = o.switch_key(s_g, s_qp, seed=9 + steps)
        rot = o.rotate(ct[None], g, gk)[0]
        dec = crt_centered(o.decrypt(rot, s_qp), Q)
        want = [delta * v for v in automorph_int(u, g)]
        err = max(abs(a - b) for a, b in zip(dec, want))
        assert err < 2 ** 30, (steps, math.log2(err + 1))


@pytest.mark.parametrize("mult", ["behz", "hps"])
def test_bfv_mul_relin_decrypts_exactly(mult):
    t = 65537
    o = Oracle(SCHEME_BFV, 10, 4, 2, 2, t=t, bfv_mult=mult)
    Q = [int(q) for q in o.moduli[:o.L]]
    Qp = math.prod(Q)
    s, s_qp = _keys(o)
    rlk = o.switch_key(_square_ntt(o, s_qp), s_qp, seed=6)
    rng = random.Random(3)
    delta = Qp // t
    m1 = [rng.randrange(t) for _ in range(o.n)]
    m2 = [rng.randrange(t) for _ in range(o.n)]
    c1 = o.encrypt(to_rns([delta * x for x in m1], Q), s_qp, 404)
    c2 = o.encrypt(to_rns([delta * x for x in m2], Q), s_qp, 505)

    def dec(ct):
        v = crt_centered(o.decrypt(ct, s_qp), Q)
        return [((t * x + Qp // 2) // Qp) % t for x in v]

    assert dec(c1) == m1
    prod = o.mul_relin(c1[None], c2[None], rlk)[0]
    want = [v % t for v in negacyclic_int(m1, m2)]
    assert dec(prod) == want
    add = o.ct_add(c1[None], c2[None])[0]
    assert dec(add) == [(a + b) % t for a, b in zip(m1, m2)]
    g = o.galois_elt(1)
    gk = o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=8)
    rot = o.rotate(c1[None], g, gk)[0]
    assert dec(rot) == [v % t for v in automorph_int(m1, g)]


def test_ckks_hoisted_rotations_decrypt():
    """Hoisted rotations (one ModUp shared) decrypt to the rotated message with
    real Galois keys, like the plain rotation."""
    o = Oracle(SCHEME_CKKS, 10, 4, 2, 2)
    Q = [int(q) for q in o.moduli[:o.L]]
    s, s_qp = _keys(o)
    rng = random.Random(7)
    delta = 1 << 40
    u = [rng.randint(-100, 100) for _ in range(o.n)]
    ct = o.encrypt(to_rns([delta * x for x in u], Q), s_qp, 707)
    steps = (1, 5, -3)
    gs = [o.galois_elt(k) for k in steps]
    gks = np.stack([o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=30 + i) for i, g in enumerate(gs)])
    outs = o.rotate_hoisted(ct[None], gs, gks)
    for r, g in enumerate(gs):
        dec = crt_centered(o.decrypt(outs[r, 0], s_qp), Q)
        want = [delta * v for v in automorph_int(u, g)]
        assert max(abs(a - b) for a, b in zip(dec, want)) < 2 ** 30


def test_ckks_hoisted_rotations_at_level_decrypt():
    """The same at a reduced level (3 of 4 limbs: a partial last digit) with the
    full-level Galois keys."""
    o = Oracle(SCHEME_CKKS, 10, 4, 2, 2)
    lvl = 3
    Q = [int(q) for q in o.moduli[:lvl]]
    s, s_qp = _keys(o)
    rng = random.Random(8)
    delta = 1 << 40
    u = [rng.randint(-100, 100) for _ in range(o.n)]
    ct = o.encrypt(to_rns([delta * x for x in u], [int(q) for q in o.moduli[:o.L]]), s_qp, 808)
    ct = np.ascontiguousarray(ct[:, :lvl])
    gs = [o.galois_elt(k) for k in (2, -1)]
    gks = np.stack([o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=40 + i) for i, g in enumerate(gs)])
    outs = o.rotate_hoisted_at(ct[None], gs, gks, lvl)
    qs = o.moduli[:lvl].astype(object)[:, None]
    for r, g in enumerate(gs):
        c0, c1 = outs[r, 0]
        m = ((c0.astype(object) + c1.astype(object) * s_qp[:lvl].astype(object)) % qs).astype(np.uint64)
        dec = crt_centered(o.ntt_inv(m[None])[0], Q)
        want = [delta * v for v in automorph_int(u, g)]
        assert max(abs(a - b) for a, b in zip(dec, want)) < 2 ** 30


@pytest.mark.parametrize("mult", ["behz", "hps"])
def test_bfv_hoisted_rotations_decrypt_exactly(mult):
    """BFV hoisted rotations (coefficient-form ciphertexts; the extension of c1
    permuted in the NTT domain of the inner product, c0 by the signed
    coefficient map) decrypt exactly to the rotated message, also after a
    product."""
    t = 65537
    o = Oracle(SCHEME_BFV, 10, 4, 2, 2, t=t, bfv_mult=mult)
    Q = [int(q) for q in o.moduli[:o.L]]
    Qp = math.prod(Q)
    s, s_qp = _keys(o)
    rng = random.Random(11)
    delta = Qp // t
    m1 = [rng.randrange(t) for _ in range(o.n)]
    m2 = [rng.randrange(t) for _ in range(o.n)]
    c1 = o.encrypt(to_rns([delta * x for x in m1], Q), s_qp, 606)
    c2 = o.encrypt(to_rns([delta * x for x in m2], Q), s_qp, 707)
    rlk = o.switch_key(_square_ntt(o, s_qp), s_qp, seed=12)
    prod = o.mul_relin(c1[None], c2[None], rlk)[0]
    want_prod = [v % t for v in negacyclic_int(m1, m2)]

    def dec(ct):
        v = crt_centered(o.decrypt(ct, s_qp), Q)
        return [((t * x + Qp // 2) // Qp) % t for x in v]

    gs = [o.galois_elt(k) for k in (1, -2, 5)]
    gks = np.stack([o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=50 + i) for i, g in enumerate(gs)])
    outs = o.rotate_hoisted(np.stack([c1, prod]), gs, gks)
    for r, g in enumerate(gs):
        assert dec(outs[r, 0]) == [v % t for v in automorph_int(m1, g)]
        assert dec(outs[r, 1]) == [v % t for v in automorph_int(want_prod, g)]


def test_rotation_sum_double_hoisted_decrypts():
    """Double-hoisted rotation sum (one ModDown for all the Galois elements):
    BFV decrypts exactly to sum_r rot_r(m) mod t, CKKS within the noise bound,
    at the full level and (CKKS) at a reduced one."""
    t = 65537
    o = Oracle(SCHEME_BFV, 10, 4, 2, 2, t=t)
    Q = [int(q) for q in o.moduli[:o.L]]
    Qp = math.prod(Q)
    s, s_qp = _keys(o)
    rng = random.Random(21)
    m1 = [rng.randrange(t) for _ in range(o.n)]
    c1 = o.encrypt(to_rns([(Qp // t) * x for x in m1], Q), s_qp, 909)
    gs = [o.galois_elt(k) for k in (1, 2, -3)]
    gks = np.stack([o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=60 + i) for i, g in enumerate(gs)])
    out = o.rotate_sum_hoisted(c1[None], gs, gks)[0]
    v = crt_centered(o.decrypt(out, s_qp), Q)
    got = [((t * x + Qp // 2) // Qp) % t for x in v]
    want = [sum(col) % t for col in zip(*[automorph_int(m1, g) for g in gs])]
    assert got == want

    o = Oracle(SCHEME_CKKS, 10, 4, 2, 2)
    s, s_qp = _keys(o)
    delta = 1 << 40
    u = [rng.randint(-100, 100) for _ in range(o.n)]
    for lvl in (4, 3):
        Ql = [int(q) for q in o.moduli[:lvl]]
        ct = o.encrypt(to_rns([delta * x for x in u], [int(q) for q in o.moduli[:o.L]]), s_qp, 919)
        ct = np.ascontiguousarray(ct[:, :lvl])
        gks = np.stack([o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=70 + i) for i, g in enumerate(gs)])
        out = o.rotate_sum_hoisted(ct[None], gs, gks)[0]
        qs = o.moduli[:lvl].astype(object)[:, None]
        m = ((out[0].astype(object) + out[1].astype(object) * s_qp[:lvl].astype(object)) % qs).astype(np.uint64)
        dec = crt_centered(o.ntt_inv(m[None])[0], Ql)
        want = [delta * sum(col) for col in zip(*[automorph_int(u, g) for g in gs])]
        assert max(abs(a - b) for a, b in zip(dec, want)) < 2 ** 30, lvl


def test_linear_transform_hoisted_decrypts():
    """Hoisted linear transform (CKKS): sum_r w_r * rot_r(m) with plaintexts w_r
    (small integer polynomials, NTT form over Q u P), one ModDown for the whole
    sum: decrypts to Delta * sum_r w_r * rot_r(u) within the noise bound."""
    o = Oracle(SCHEME_CKKS, 10, 4, 2, 2)
    Q = [int(q) for q in o.moduli[:o.L]]
    s, s_qp = _keys(o)
    rng = random.Random(31)
    delta = 1 << 40
    u = [rng.randint(-50, 50) for _ in range(o.n)]
    ct = o.encrypt(to_rns([delta * x for x in u], Q), s_qp, 929)
    gs = [o.galois_elt(k) for k in (1, 2, -1)]
    gks = np.stack([o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=80 + i) for i, g in enumerate(gs)])
    ws = []
    for _ in gs:
        w = [0] * o.n
        for _ in range(4):
            w[rng.randrange(o.n)] = rng.randint(-2, 2)
        ws.append(w)
    pts = np.stack([o.signed_to_rns(w, 0, o.L + o.K, ntt=True) for w in ws])
    out = o.linear_hoisted(ct[None], gs, gks, pts)[0]
    dec = crt_centered(o.decrypt(out, s_qp), Q)
    want = [0] * o.n
    for g, w in zip(gs, ws):
        for i, v in enumerate(negacyclic_int(w, automorph_int(u, g))):
            want[i] += delta * v
    assert max(abs(a - b) for a, b in zip(dec, want)) < 2 ** 34
