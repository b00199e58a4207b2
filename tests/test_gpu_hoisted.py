"""Hoisted CKKS rotations on the HIP backend (fhe_rotate_hoisted[_at]): one
ModUp of c1 shared by every Galois element, sigma_g applied to the extension
(OpenFHE EvalFastRotationPrecompute / EvalFastRotation; oracle
orc_rotate_hoisted, oracle/bigint_model.py rotate_hoisted).

Evidence:
  * the big-int golden fixture ckks_hoisted_n1024_l5.npz (one-pass size: the
    generic path that materialises sigma_g(ext) and sigma_g(c0));
  * the CPU oracle on identical seeded inputs at the metric parameters
    N=2^16, L=12, K=4, dnum=3 (the fused path: sigma_g is a gather inside the
    inner-product passes) at levels 12, 7 (partial last digit) and 5;
  * N=2^15 with dnum=5 (more digits than the fused inner product takes: the
    generic path at a two-pass size) and OpenFHE-style generic primes.
"""
import os

import numpy as np
import pytest

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
    return o, c


def _run(hb, c, ct, gs, gks, lvl=None):
    n = ct.shape[0]
    shape = (n, 2, ct.shape[2], c.n)
    outs = [hb.empty(shape) for _ in gs]
    d_ct = hb.to_device(ct)
    d_gk = [hb.to_device(k) for k in gks]
    if lvl is None:
        c.rotate_hoisted(d_ct, gs, d_gk, outs)
    else:
        c.rotate_hoisted_at(d_ct, gs, d_gk, outs, lvl)
    return np.stack([hb.to_host(o) for o in outs])


def test_hoisted_golden(hb):
    g = np.load(os.path.join(GOLD, "ckks_hoisted_n1024_l5.npz"))
    c = hb.Context(SCHEME_CKKS, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), moduli=g["moduli"])
    got = _run(hb, c, g["ct"][None], [int(x) for x in g["galois"]], list(g["gks"]))
    assert np.array_equal(got[:, 0], g["out"])


def test_bfv_hoisted_golden(hb):
    g = np.load(os.path.join(GOLD, "bfv_hoisted_n1024_l4.npz"))
    c = hb.Context(SCHEME_BFV, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), t=int(g["t"]),
                   moduli=g["moduli"])
    got = _run(hb, c, g["ct"][None], [int(x) for x in g["galois"]], list(g["gks"]))
    assert np.array_equal(got[:, 0], g["out"])


def test_hoisted_metric_params(hb, metric):
    o, c = metric
    ct = o.uniform((2, 2, o.L, o.n), seed=1100)
    gs = [o.galois_elt(1), o.galois_elt(-7), 2 * o.n - 1]
    gks = [o.uniform(o.key_shape(), seed=1101 + i) for i in range(len(gs))]
    want = o.rotate_hoisted(ct, gs, np.stack(gks))
    got = _run(hb, c, ct, gs, gks)
    assert np.array_equal(got, want)
    # one Galois element: the hoisted result differs from the plain rotation
    # only by the ModUp error term, so it is a distinct (but valid) ciphertext
    plain = o.rotate(ct[:1], gs[0], gks[0])
    assert not np.array_equal(plain, want[0, :1])


@pytest.mark.parametrize("n_ct,steps", [(1, (1, 2, 3, 4, 5, 6, 7, -1, -2, -3)), (16, (1, -1, 3))])
def test_hoisted_rotation_batches(hb, metric, n_ct, steps):
    """Few ciphertexts: several Galois elements per launch of the gather passes
    (FHE_ROT_BATCH = 8 per launch while n_ct * batch <= 32): 10 elements on one
    ciphertext run as 8 + 2, 3 elements on 16 ciphertexts as 2 + 1."""
    o, c = metric
    ct = o.uniform((n_ct, 2, o.L, o.n), seed=1600 + n_ct)
    gs = [o.galois_elt(k) for k in steps]
    gks = [o.uniform(o.key_shape(), seed=1610 + i) for i in range(len(gs))]
    want = o.rotate_hoisted(ct, gs, np.stack(gks))
    assert np.array_equal(_run(hb, c, ct, gs, gks), want)


@pytest.mark.parametrize("lvl", [7, 5])
def test_hoisted_at_levels(hb, metric, lvl):
    o, c = metric
    ct = o.uniform((1, 2, lvl, o.n), seed=1200 + lvl)
    gs = [o.galois_elt(3), o.galois_elt(-1)]
    gks = [o.uniform(o.key_shape(), seed=1210 + i) for i in range(len(gs))]
    want = o.rotate_hoisted_at(ct, gs, np.stack(gks), lvl)
    assert np.array_equal(_run(hb, c, ct, gs, gks, lvl), want)


def test_hoisted_many_digits_generic_primes(hb):
    """dnum = 5 > 4 digits at N = 2^15: sigma_g(ext) is materialised; generic
    (OpenFHE-style) primes take the generic Montgomery path."""
    from herdsman_amd.params import openfhe_style_primes
    mods = openfhe_style_primes([(55, 5), (61, 5), (61, 2)], 15)
    o = Oracle(SCHEME_CKKS, 15, 10, 2, 5, moduli=mods)
    c = hb.Context(SCHEME_CKKS, 15, 10, 2, 5, moduli=o.moduli)
    ct = o.uniform((1, 2, o.L, o.n), seed=1300)
    gs = [o.galois_elt(2), o.galois_elt(-5)]
    gks = [o.uniform(o.key_shape(), seed=1301 + i) for i in range(len(gs))]
    assert np.array_equal(_run(hb, c, ct, gs, gks), o.rotate_hoisted(ct, gs, np.stack(gks)))


def test_hoisted_errors(hb, metric):
    o, c = metric
    lib = hb.load_library()
    import ctypes as C
    ct = hb.empty((1, 2, o.L, o.n))
    k = hb.empty(o.key_shape())
    ga = (C.c_uint32 * 1)(o.galois_elt(1))
    ka = (C.c_uint64 * 1)(hb._ptr(k))
    oa = (C.c_uint64 * 1)(hb._ptr(ct))  # output == input
    assert lib.fhe_rotate_hoisted(c.h, hb._ptr(ct), 1, C.addressof(ga), C.addressof(ka), C.addressof(oa), 1) \
        == hb.FHE_ERR_INVALID
    out = hb.empty((1, 2, o.L, o.n))
    oa[0] = hb._ptr(out)
    ga[0] = 4  # even
    assert lib.fhe_rotate_hoisted(c.h, hb._ptr(ct), 1, C.addressof(ga), C.addressof(ka), C.addressof(oa), 1) \
        == hb.FHE_ERR_INVALID
    assert lib.fhe_rotate_hoisted(c.h, hb._ptr(ct), 0, None, None, None, 1) == hb.FHE_OK
    ga2 = (C.c_uint32 * 2)(o.galois_elt(1), o.galois_elt(2))
    ka2 = (C.c_uint64 * 2)(hb._ptr(k), hb._ptr(k))
    oa2 = (C.c_uint64 * 2)(hb._ptr(out), hb._ptr(out))  # two outputs on one buffer
    assert lib.fhe_rotate_hoisted(c.h, hb._ptr(ct), 2, C.addressof(ga2), C.addressof(ka2), C.addressof(oa2), 1) \
        == hb.FHE_ERR_INVALID
    bfv = hb.Context(SCHEME_BFV, 12, 3, 1, 1, t=65537)
    z = hb.empty((1, 2, 3, bfv.n))
    kz = hb.empty(bfv.key_shape())
    ka[0] = hb._ptr(kz)
    oa[0] = hb._ptr(hb.empty((1, 2, 3, bfv.n)))
    ga[0] = 5
    # BFV has no reduced levels
    assert lib.fhe_rotate_hoisted_at(bfv.h, hb._ptr(z), 1, C.addressof(ga), C.addressof(ka), C.addressof(oa), 1,
                                     2) == hb.FHE_ERR_UNSUPPORTED


@pytest.mark.parametrize("log_n,L,K,dnum", [(15, 8, 4, 2), (12, 5, 2, 3)])
def test_bfv_hoisted(hb, log_n, L, K, dnum):
    """BFV (coefficient form): ext permuted in the NTT domain, c0 by the signed
    coefficient map, the coefficient-domain ModDown; C3 parameters and a
    one-pass size with a partial digit."""
    o = Oracle(SCHEME_BFV, log_n, L, K, dnum, t=65537)
    c = hb.Context(SCHEME_BFV, log_n, L, K, dnum, t=65537, moduli=o.moduli)
    ct = o.uniform((2, 2, L, o.n), seed=1500 + log_n)
    gs = [o.galois_elt(1), o.galois_elt(-4), 2 * o.n - 1]
    gks = [o.uniform(o.key_shape(), seed=1510 + i) for i in range(len(gs))]
    assert np.array_equal(_run(hb, c, ct, gs, gks), o.rotate_hoisted(ct, gs, np.stack(gks)))


def test_bfv_hoisted_rotation_batches(hb):
    """BFV at C3 parameters, one ciphertext, 10 Galois elements: 8 + 2 per launch."""
    o = Oracle(SCHEME_BFV, 15, 8, 4, 2, t=65537)
    c = hb.Context(SCHEME_BFV, 15, 8, 4, 2, t=65537, moduli=o.moduli)
    ct = o.uniform((1, 2, o.L, o.n), seed=1700)
    gs = [o.galois_elt(k) for k in (1, 2, 3, 4, 5, -1, -2, -3, -4, -5)]
    gks = [o.uniform(o.key_shape(), seed=1710 + i) for i in range(len(gs))]
    assert np.array_equal(_run(hb, c, ct, gs, gks), o.rotate_hoisted(ct, gs, np.stack(gks)))


def test_hoisted_chunked_batch(hb):
    """More ciphertexts than one internal pass (kCtChunk = 512): the outputs of
    every chunk land at their own offsets."""
    o = Oracle(SCHEME_CKKS, 12, 3, 2, 3)
    c = hb.Context(SCHEME_CKKS, 12, 3, 2, 3, moduli=o.moduli)
    ct = o.uniform((520, 2, o.L, o.n), seed=1400)
    gs = [o.galois_elt(1), o.galois_elt(-2)]
    gks = [o.uniform(o.key_shape(), seed=1401 + i) for i in range(len(gs))]
    c.reserve(520)
    assert np.array_equal(_run(hb, c, ct, gs, gks), o.rotate_hoisted(ct, gs, np.stack(gks)))


# ---- double-hoisted rotation sum (fhe_rotate_sum_hoisted[_at]): one ModDown
@pytest.mark.parametrize("scheme,log_n,L,K,dnum,n_ct,steps", [
    (SCHEME_CKKS, 16, 12, 4, 3, 2, (1, 2, -1, 5, -7)),
    (SCHEME_CKKS, 12, 5, 2, 3, 3, (1, 2, 3)),
    (SCHEME_CKKS, 12, 4, 2, 2, 1, tuple(range(1, 19))),  # two chunks of the 16-element kernel
    (SCHEME_BFV, 15, 8, 4, 2, 2, (1, -2, 3)),
    (SCHEME_BFV, 12, 5, 2, 3, 1, (2, 4)),
])
def test_rotation_sum_double_hoisted(hb, scheme, log_n, L, K, dnum, n_ct, steps):
    t = 65537 if scheme == SCHEME_BFV else 0
    o = Oracle(scheme, log_n, L, K, dnum, t=t)
    c = hb.Context(scheme, log_n, L, K, dnum, t=t, moduli=o.moduli)
    ct = o.uniform((n_ct, 2, L, o.n), seed=1800 + log_n + len(steps))
    gs = [o.galois_elt(k) for k in steps]
    gks = [o.uniform(o.key_shape(), seed=1820 + i) for i in range(len(gs))]
    want = o.rotate_sum_hoisted(ct, gs, np.stack(gks))
    d_gk = [hb.to_device(k) for k in gks]
    out = hb.empty(ct.shape)
    c.rotate_sum_hoisted(hb.to_device(ct), gs, d_gk, out)
    assert np.array_equal(hb.to_host(out), want)
    io = hb.to_device(ct)  # in place
    c.rotate_sum_hoisted(io, gs, d_gk, io)
    assert np.array_equal(hb.to_host(io), want)


def test_rotation_sum_partial_overlap_is_refused(hb):
    """out == ct (in place) or apart; a partial overlap is FHE_ERR_INVALID (the
    work runs in chunks, and a shifted out would overwrite rows a later chunk reads)."""
    o = Oracle(SCHEME_CKKS, 12, 4, 2, 2)
    c = hb.Context(SCHEME_CKKS, 12, 4, 2, 2, moduli=o.moduli)
    buf = hb.empty((3, 2, 4, o.n))
    gs = [o.galois_elt(1)]
    d_gk = [hb.to_device(o.uniform(o.key_shape(), seed=1830))]
    with pytest.raises(hb.FheBackendError, match="overlap"):
        c.rotate_sum_hoisted(buf[:2], gs, d_gk, buf[1:])


def test_rotation_sum_double_hoisted_at_level(hb, metric):
    o, c = metric
    lvl = 7
    ct = o.uniform((1, 2, lvl, o.n), seed=1900)
    gs = [o.galois_elt(k) for k in (1, 3, -2)]
    gks = [o.uniform(o.key_shape(), seed=1910 + i) for i in range(len(gs))]
    out = hb.empty(ct.shape)
    c.rotate_sum_hoisted_at(hb.to_device(ct), gs, [hb.to_device(k) for k in gks], out, lvl)
    assert np.array_equal(hb.to_host(out), o.rotate_sum_hoisted(ct, gs, np.stack(gks), lvl))


@pytest.mark.parametrize("scheme", ["ckks", "bfv"])
def test_rotation_sum_golden(hb, scheme):
    g = np.load(os.path.join(GOLD, "rotation_sum_n1024.npz"))
    if scheme == "ckks":
        c = hb.Context(SCHEME_CKKS, int(g["log_n"]), 5, 2, 2, moduli=g["ckks_moduli"])
    else:
        c = hb.Context(SCHEME_BFV, int(g["log_n"]), 4, 2, 2, t=65537, moduli=g["bfv_moduli"])
    out = hb.empty((1,) + g[f"{scheme}_ct"].shape)
    c.rotate_sum_hoisted(hb.to_device(g[f"{scheme}_ct"][None]), [int(x) for x in g[f"{scheme}_galois"]],
                         [hb.to_device(k) for k in g[f"{scheme}_gks"]], out)
    assert np.array_equal(hb.to_host(out)[0], g[f"{scheme}_out"])
    if scheme == "ckks":
        c.linear_hoisted(hb.to_device(g["ckks_ct"][None]), [int(x) for x in g["ckks_galois"]],
                         [hb.to_device(k) for k in g["ckks_gks"]], [hb.to_device(p) for p in g["ckks_pts"]], out)
        assert np.array_equal(hb.to_host(out)[0], g["ckks_lin"])


# ---- hoisted linear transform (fhe_linear_hoisted[_at], CKKS): sum_r pt_r (.) rot_r(ct)
@pytest.mark.parametrize("log_n,L,K,dnum,n_ct,steps,lvl", [
    (16, 12, 4, 3, 2, (1, 2, -1, 5), None),
    (16, 12, 4, 3, 1, (1, 3, -2), 7),
    (12, 5, 2, 3, 3, tuple(range(1, 19)), None),  # two chunks of the 16-element kernel, one-pass ModDown
])
def test_linear_transform_hoisted(hb, log_n, L, K, dnum, n_ct, steps, lvl):
    o = Oracle(SCHEME_CKKS, log_n, L, K, dnum)
    c = hb.Context(SCHEME_CKKS, log_n, L, K, dnum, moduli=o.moduli)
    m = L if lvl is None else lvl
    ct = o.uniform((n_ct, 2, m, o.n), seed=2000 + log_n + m)
    gs = [o.galois_elt(k) for k in steps]
    gks = [o.uniform(o.key_shape(), seed=2010 + i) for i in range(len(gs))]
    pts = [o.uniform((L + K, o.n), seed=2100 + i) for i in range(len(gs))]
    want = o.linear_hoisted(ct, gs, np.stack(gks), np.stack(pts), m)
    d_gk = [hb.to_device(k) for k in gks]
    d_pt = [hb.to_device(p) for p in pts]
    out = hb.empty(ct.shape)
    if lvl is None:
        c.linear_hoisted(hb.to_device(ct), gs, d_gk, d_pt, out)
        io = hb.to_device(ct)
        c.linear_hoisted(io, gs, d_gk, d_pt, io)  # in place
        assert np.array_equal(hb.to_host(io), want)
    else:
        c.linear_hoisted_at(hb.to_device(ct), gs, d_gk, d_pt, out, lvl)
    assert np.array_equal(hb.to_host(out), want)


def test_linear_transform_hoisted_bfv_unsupported(hb):
    import ctypes as C
    lib = hb.load_library()
    bfv = hb.Context(SCHEME_BFV, 12, 3, 1, 1, t=65537)
    z = hb.empty((1, 2, 3, bfv.n))
    k = hb.empty(bfv.key_shape())
    p = hb.empty((4, bfv.n))
    ga = (C.c_uint32 * 1)(5)
    ka = (C.c_uint64 * 1)(hb._ptr(k))
    pa = (C.c_uint64 * 1)(hb._ptr(p))
    assert lib.fhe_linear_hoisted(bfv.h, hb._ptr(z), 1, C.addressof(ga), C.addressof(ka), C.addressof(pa),
                                  hb._ptr(hb.empty((1, 2, 3, bfv.n))), 1) == hb.FHE_ERR_UNSUPPORTED
