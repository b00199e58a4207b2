"""Seeded sweep of odd shapes through every ciphertext op, HIP backend vs the
CPU oracle, bit-exact.  The fixed-shape parity tests (test_gpu_parity.py,
test_gpu_levels.py, test_gpu_hoisted.py) pin the BASELINE configs; this
sweep draws (log_n, L, K, dnum, scheme, BFV technique, prime family) from a
fixed seed so that partial last digits, alpha not dividing L, K < alpha,
one-pass and two-pass sizes, both lazy-schedule classes and both BFV
multiplication techniques meet every op: mul+relin, rotate, keyswitch,
hoisted rotations, the double-hoisted rotation sum, and for CKKS rescale, a level-reduced mul+relin and
level-reduced hoisted rotations.
"""
import random

import numpy as np
import pytest

from oracle_ffi import Oracle, SCHEME_BFV, SCHEME_CKKS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hb():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import herdsman_amd.backend as hb

    hb.load_library()
    return hb


def _shapes(seed=0x53574550, count=32):
    rng = random.Random(seed)
    out = []
    for i in range(count):
        scheme = SCHEME_CKKS if i % 3 else SCHEME_BFV
        log_n = rng.choice([12, 13, 14, 15, 15, 16, 17])
        L = rng.randint(2, 4 if log_n == 17 else 9 if log_n >= 15 else 12)
        dnum = rng.randint(1, L)
        K = rng.randint(1, 4)
        generic = rng.random() < 0.3
        mult = rng.choice(["behz", "hps"]) if scheme == SCHEME_BFV else "behz"
        out.append((i, scheme, log_n, L, K, dnum, generic, mult))
    return out


@pytest.mark.parametrize("i,scheme,log_n,L,K,dnum,generic,mult", _shapes())
def test_sweep(hb, i, scheme, log_n, L, K, dnum, generic, mult):
    from herdsman_amd.params import openfhe_style_primes
    mods = openfhe_style_primes([(58, L), (61, K)], log_n) if generic else None
    t = 65537 if scheme == SCHEME_BFV else 0
    if scheme == SCHEME_BFV and generic:
        # BFV needs its Bsk primes too: generic Q, P and Bsk families
        mods = openfhe_style_primes([(58, L), (61, K), (60, L + 1)], log_n)
    o = Oracle(scheme, log_n, L, K, dnum, t=t, moduli=mods, bfv_mult=mult)
    c = hb.Context(scheme, log_n, L, K, dnum, t=t, moduli=o.moduli, bfv_mult=mult)
    assert np.array_equal(c.moduli, o.moduli)
    n, s = o.n, 7000 + 10 * i
    nct = 2
    a = o.uniform((nct, 2, L, n), seed=s)
    b = o.uniform((nct, 2, L, n), seed=s + 1)
    k = o.uniform(o.key_shape(), seed=s + 2)
    da, db, dk = hb.to_device(a), hb.to_device(b), hb.to_device(k)
    out = hb.empty((nct, 2, L, n))
    c.mul_relin(da, db, dk, out)
    assert np.array_equal(hb.to_host(out), o.mul_relin(a, b, k)), "mul_relin"
    steps = (i % 5) - 2 or 3
    g = o.galois_elt(steps)
    c.rotate(da, g, dk, out)
    assert np.array_equal(hb.to_host(out), o.rotate(a, g, k)), ("rotate", steps)
    d = o.uniform((nct, L, n), seed=s + 3)
    c.keyswitch(hb.to_device(d), dk, out)
    assert np.array_equal(hb.to_host(out), o.keyswitch(d, k)), "keyswitch"
    gs = [o.galois_elt(1), o.galois_elt(-3)]
    outs = [hb.empty((nct, 2, L, n)) for _ in gs]
    c.rotate_hoisted(da, gs, [dk, dk], outs)
    want = o.rotate_hoisted(a, gs, np.stack([k, k]))
    for r in range(len(gs)):
        assert np.array_equal(hb.to_host(outs[r]), want[r]), ("hoisted", r)
    c.rotate_sum_hoisted(da, gs, [dk, dk], out)
    assert np.array_equal(hb.to_host(out), o.rotate_sum_hoisted(a, gs, np.stack([k, k]))), "rotation sum"
    if scheme != SCHEME_CKKS:
        return
    if L >= 2:
        r_out = hb.empty((nct, 2, L - 1, n))
        c.rescale(da, r_out, L)
        assert np.array_equal(hb.to_host(r_out), o.rescale(a, L)), "rescale"
        lvl = max(1, L - 1 - (i % 3))
        al = np.ascontiguousarray(a[:, :, :lvl])
        bl = np.ascontiguousarray(b[:, :, :lvl])
        ol = hb.empty((nct, 2, lvl, n))
        c.mul_relin_at(hb.to_device(al), hb.to_device(bl), dk, ol, lvl)
        assert np.array_equal(hb.to_host(ol), o.mul_relin_at(al, bl, k, lvl)), ("mul_relin_at", lvl)
        hl = [hb.empty((nct, 2, lvl, n)) for _ in gs]
        c.rotate_hoisted_at(hb.to_device(al), gs, [dk, dk], hl, lvl)
        want = o.rotate_hoisted_at(al, gs, np.stack([k, k]), lvl)
        for r in range(len(gs)):
            assert np.array_equal(hb.to_host(hl[r]), want[r]), ("hoisted_at", lvl, r)


@pytest.mark.parametrize("log_n,L,K,dnum", [(15, 8, 4, 2), (16, 3, 2, 3)])
def test_bfv_fused_key_switch_paths(hb, log_n, L, K, dnum):
    """BFV at two-pass sizes runs every key switch on the fused passes (ModUp in
    the NTT column pass, the all-limb inner product in INTT(acc)'s first pass,
    one ModDown kernel): keyswitch, rotate apart (c0 read through the
    coefficient map) and in place (sigma(c0) stored first)."""
    o = Oracle(SCHEME_BFV, log_n, L, K, dnum, t=65537)
    c = hb.Context(SCHEME_BFV, log_n, L, K, dnum, t=65537, moduli=o.moduli)
    a = o.uniform((2, 2, L, o.n), seed=9100 + log_n)
    k = o.uniform(o.key_shape(), seed=9101)
    dk = hb.to_device(k)
    g = o.galois_elt(-2)
    want = o.rotate(a, g, k)
    out = hb.empty((2, 2, L, o.n))
    c.rotate(hb.to_device(a), g, dk, out)
    assert np.array_equal(hb.to_host(out), want)
    io = hb.to_device(a)
    c.rotate(io, g, dk, io)
    assert np.array_equal(hb.to_host(io), want)
    d = o.uniform((2, L, o.n), seed=9102)
    c.keyswitch(hb.to_device(d), dk, out)
    assert np.array_equal(hb.to_host(out), o.keyswitch(d, k))
