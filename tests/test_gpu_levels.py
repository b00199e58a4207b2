"""CKKS levels on the HIP backend: ops on level-reduced ciphertexts and rescale
(fhe_*_at, fhe_rescale; SURVEY.md §8(a) a6 "+ optional rescale").

Evidence, as for the full-level ops (tests/test_gpu_parity.py):
  * the big-int golden fixture ckks_levels_n1024_l5.npz (oracle/bigint_model.py:
    keyswitch at a level with a partial last digit, rescale by its integer
    definition round(c / q_last));
  * the CPU oracle (orc_*_at, orc_rescale) on identical seeded inputs at the
    metric parameters N=2^16, L=12, K=4, dnum=3 for levels 12, 8, 5 and 4
    (level 5: one full and one single-limb digit);
  * a depth-3 CKKS product with real keys (mul+relin and rescale at levels 12,
    11 and 10) that decrypts to Delta^4 m1 m2 m3 m4 / (q11 q10 q9) within the
    noise bound.
"""
import os
import random
from fractions import Fraction

import numpy as np
import pytest

from fhe_math import crt_centered, to_rns
from oracle_ffi import Oracle, SCHEME_BFV, SCHEME_CKKS

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def hb():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    import herdsman_amd.backend as hb

    hb.load_library()
    return hb


@pytest.fixture(scope="module")
def metric(hb):
    o = Oracle(SCHEME_CKKS, 16, 12, 4, 3)
    c = hb.Context(SCHEME_CKKS, 16, 12, 4, 3, moduli=o.moduli)
    assert np.array_equal(c.moduli, o.moduli)
    return o, c


def test_levels_golden(hb):
    g = np.load(os.path.join(GOLD, "ckks_levels_n1024_l5.npz"))
    c = hb.Context(SCHEME_CKKS, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), moduli=g["moduli"])
    rlk = hb.to_device(g["rlk"])
    for lvl in (4, 2):
        out = hb.empty((1, 2, lvl, c.n))
        c.mul_relin_at(hb.to_device(g[f"a{lvl}"][None]), hb.to_device(g[f"b{lvl}"][None]), rlk, out, lvl)
        assert np.array_equal(hb.to_host(out)[0], g[f"mul{lvl}"]), lvl
    out = hb.empty((1, 2, 3, c.n))
    c.rotate_at(hb.to_device(g["a3"][None]), int(g["g"]), rlk, out, 3)
    assert np.array_equal(hb.to_host(out)[0], g["rot3"])
    r4 = hb.empty((1, 2, 4, c.n))
    c.rescale(hb.to_device(g["c5"][None]), r4, 5)
    assert np.array_equal(hb.to_host(r4)[0], g["r4"])
    r3 = hb.empty((1, 2, 3, c.n))
    c.rescale(r4, r3, 4)
    assert np.array_equal(hb.to_host(r3)[0], g["r3"])


@pytest.mark.parametrize("lvl", [12, 8, 5, 4])
def test_mul_relin_at_metric_params(hb, metric, lvl):
    o, c = metric
    n = o.n
    a = o.uniform((2, 2, lvl, n), seed=100 + lvl)
    b = o.uniform((2, 2, lvl, n), seed=200 + lvl)
    k = o.uniform(o.key_shape(), seed=300)
    want = o.mul_relin_at(a, b, k, lvl)
    out = hb.empty((2, 2, lvl, n))
    c.mul_relin_at(hb.to_device(a), hb.to_device(b), hb.to_device(k), out, lvl)
    assert np.array_equal(hb.to_host(out), want)
    if lvl == 12:
        assert np.array_equal(want, o.mul_relin(a, b, k))


@pytest.mark.parametrize("lvl,steps", [(7, 1), (4, -3)])
def test_rotate_at_metric_params(hb, metric, lvl, steps):
    o, c = metric
    ct = o.uniform((1, 2, lvl, o.n), seed=400 + lvl)
    gk = o.uniform(o.key_shape(), seed=401)
    g = o.galois_elt(steps)
    want = o.rotate_at(ct, g, gk, lvl)
    out = hb.empty((1, 2, lvl, o.n))
    c.rotate_at(hb.to_device(ct), g, hb.to_device(gk), out, lvl)
    assert np.array_equal(hb.to_host(out), want)


def test_keyswitch_at_metric_params(hb, metric):
    o, c = metric
    lvl = 6
    d = o.uniform((1, lvl, o.n), seed=500)
    k = o.uniform(o.key_shape(), seed=501)
    want = o.keyswitch_at(d, k, lvl)
    out = hb.empty((1, 2, lvl, o.n))
    c.keyswitch_at(hb.to_device(d), hb.to_device(k), out, lvl)
    assert np.array_equal(hb.to_host(out), want)


@pytest.mark.parametrize("lvl", [12, 5, 2])
def test_rescale_metric_params(hb, metric, lvl):
    o, c = metric
    ct = o.uniform((3, 2, lvl, o.n), seed=600 + lvl)
    want = o.rescale(ct, lvl)
    out = hb.empty((3, 2, lvl - 1, o.n))
    c.rescale(hb.to_device(ct), out, lvl)
    assert np.array_equal(hb.to_host(out), want)


def test_add_sub_at(hb, metric):
    o, c = metric
    lvl = 3
    a = o.uniform((2, 2, lvl, o.n), seed=700)
    b = o.uniform((2, 2, lvl, o.n), seed=701)
    qs = o.moduli[:lvl].astype(object)[None, None, :, None]
    out = hb.empty((2, 2, lvl, o.n))
    c.add_at(hb.to_device(a), hb.to_device(b), out, lvl)
    assert np.array_equal(hb.to_host(out), ((a.astype(object) + b) % qs).astype(np.uint64))
    c.sub_at(hb.to_device(a), hb.to_device(b), out, lvl)
    assert np.array_equal(hb.to_host(out), ((a.astype(object) - b) % qs).astype(np.uint64))


def test_level_argument_errors(hb, metric):
    o, c = metric
    n = o.n
    x = hb.empty((1, 2, 3, n))
    k = hb.empty(c.key_shape())
    lib = hb.load_library()
    assert lib.fhe_mul_relin_at(c.h, hb._ptr(x), hb._ptr(x), hb._ptr(k), hb._ptr(x), 1, 0) == hb.FHE_ERR_INVALID
    assert lib.fhe_mul_relin_at(c.h, hb._ptr(x), hb._ptr(x), hb._ptr(k), hb._ptr(x), 1, 13) == hb.FHE_ERR_INVALID
    assert lib.fhe_rescale(c.h, hb._ptr(x), hb._ptr(x), 1, 1) == hb.FHE_ERR_INVALID
    y = hb.empty((1, 2, 3, n))
    # the output of a rescale may not overlap its input
    assert lib.fhe_rescale(c.h, hb._ptr(y), hb._ptr(y), 1, 3) == hb.FHE_ERR_INVALID
    assert b"overlap" in lib.fhe_last_error(c.h)
    bfv = hb.Context(SCHEME_BFV, 12, 3, 1, 1, t=65537)
    z = hb.empty((1, 2, 2, 1 << 12))
    kz = hb.empty(bfv.key_shape())
    rc = lib.fhe_mul_relin_at(bfv.h, hb._ptr(z), hb._ptr(z), hb._ptr(kz), hb._ptr(z), 1, 2)
    assert rc == hb.FHE_ERR_UNSUPPORTED
    assert lib.fhe_rescale(bfv.h, hb._ptr(z), hb._ptr(z), 1, 2) == hb.FHE_ERR_UNSUPPORTED
    # BFV has no reduced levels: the element-wise ops refuse them too
    assert lib.fhe_add_at(bfv.h, hb._ptr(z), hb._ptr(z), hb._ptr(z), 1, 2) == hb.FHE_ERR_UNSUPPORTED
    assert lib.fhe_sub_at(bfv.h, hb._ptr(z), hb._ptr(z), hb._ptr(z), 1, 2) == hb.FHE_ERR_UNSUPPORTED
    w = hb.empty((1, 2, 3, 1 << 12))
    assert lib.fhe_add_at(bfv.h, hb._ptr(w), hb._ptr(w), hb._ptr(w), 1, 3) == hb.FHE_OK


def _decrypt_at(o, ct, s_qp, lvl):
    """c0 + c1 s over Q_lvl, coefficient form, centred CRT."""
    qs = o.moduli[:lvl].astype(object)[:, None]
    m = ((ct[0].astype(object) + ct[1].astype(object) * s_qp[:lvl].astype(object)) % qs).astype(np.uint64)
    m = o.ntt_inv(m[None])[0]
    return crt_centered(m, [int(q) for q in o.moduli[:lvl]])


def test_depth3_real_keys(hb, metric):
    """((m1 m2) m3) m4 with a rescale after each product: levels 12 -> 11 -> 10
    -> 9, one relinearisation key (full level) for every level."""
    o, c = metric
    L, n = o.L, o.n
    Q = [int(q) for q in o.moduli[:L]]
    s = o.secret(21)
    s_qp = o.signed_to_rns(s, 0, L + o.K, ntt=True)
    qs = o.moduli[:L + o.K].astype(object)[:, None]
    sq = ((s_qp.astype(object) * s_qp.astype(object)) % qs).astype(np.uint64)
    rlk = hb.to_device(o.switch_key(sq, s_qp, seed=22))
    delta = 1 << 58
    msgs = [3, -2, 5, 7]
    cts = []
    for i, mv in enumerate(msgs):
        coef = [0] * n
        coef[0] = delta * mv
        cts.append(o.encrypt(to_rns(coef, Q), s_qp, 30 + i))
    cur = hb.to_device(cts[0][None])
    scale = Fraction(delta)
    for step, lvl in enumerate((12, 11, 10)):
        nxt = hb.to_device(np.ascontiguousarray(cts[step + 1][:, :lvl])[None])  # level-dropped fresh ciphertext
        prod = hb.empty((1, 2, lvl, n))
        c.mul_relin_at(cur, nxt, rlk, prod, lvl)
        cur = hb.empty((1, 2, lvl - 1, n))
        c.rescale(prod, cur, lvl)
        scale = scale * delta / Q[lvl - 1]
    dec = _decrypt_at(o, hb.to_host(cur)[0], s_qp, 9)
    want = scale * (3 * -2 * 5 * 7)
    assert abs(dec[0] - want) < 2 ** 32, (dec[0], float(want))
    assert max(abs(v) for v in dec[1:]) < 2 ** 32
    assert abs(want) > 2 ** 56  # the message is far above the noise (2^32)


def test_level_reduce_and_reduce_at(hb, metric):
    """fhe_level_reduce keeps the first limbs of every poly; fhe_reduce_at runs
    the balanced tree on a level view (add and mul+relin)."""
    o, c = metric
    ct = o.uniform((3, 2, 9, o.n), seed=800)
    out = hb.empty((3, 2, 5, o.n))
    c.level_reduce(hb.to_device(ct), out, 9, 5)
    assert np.array_equal(hb.to_host(out), ct[:, :, :5])
    lvl = 6
    cts = o.uniform((5, 2, lvl, o.n), seed=801)
    k = o.uniform(o.key_shape(), seed=802)
    lib = hb.load_library()
    d = hb.to_device(cts)
    res = hb.empty((1, 2, lvl, o.n))
    assert lib.fhe_reduce_at(c.h, hb._ptr(d), 5, hb.REDUCE_MUL_RELIN, hb._ptr(hb.to_device(k)), hb._ptr(res),
                             lvl) == 0
    live = list(cts)
    while len(live) > 1:
        half = len(live) // 2
        comb = o.mul_relin_at(np.stack(live[:half]), np.stack(live[len(live) - half:]), k, lvl)
        live = list(comb) + live[half:len(live) - half]
    assert np.array_equal(hb.to_host(res)[0], live[0])


@pytest.mark.parametrize("log_n", [15, 14])
def test_rescale_generic_primes(hb, log_n):
    """OpenFHE-style primes (q = 1 mod 2N, generic Montgomery; 55- and 61-bit so
    the fused lift meets both lazy schedules) at a two-pass size (the lift in the
    column pass prologue) and a one-pass size (the lift kernel)."""
    from herdsman_amd.params import openfhe_style_primes
    mods = openfhe_style_primes([(55, 3), (61, 3), (61, 2)], log_n)
    o = Oracle(SCHEME_CKKS, log_n, 6, 2, 3, moduli=mods)
    c = hb.Context(SCHEME_CKKS, log_n, 6, 2, 3, moduli=o.moduli)
    for lvl in (6, 4):
        ct = o.uniform((2, 2, lvl, o.n), seed=900 + lvl)
        out = hb.empty((2, 2, lvl - 1, o.n))
        c.rescale(hb.to_device(ct), out, lvl)
        assert np.array_equal(hb.to_host(out), o.rescale(ct, lvl)), lvl
