"""HIP backend (libherdsman_fhe.so, through the C ABI) vs the CPU oracle.

Bit-exact for every op (all arithmetic is integer mod q).  Three kinds of
evidence:
  * golden fixtures (tests/golden/, big-int model) at N = 1024;
  * the oracle on identical seeded inputs at the BASELINE.json configs
    C2 (NTT, N=2^14 L=4), C3 (BFV mul+relin, N=2^15 L=8), C4 (CKKS rotate,
    N=2^16 L=12 dnum=3) and the metric config (CKKS mul+relin N=2^16 L=12);
  * scheme-level decryption identities with real keys.
"""
import math
import os
import random

import numpy as np
import pytest

from fhe_math import automorph_int, crt_centered, negacyclic_int, to_rns
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


def pair(hb, scheme, log_n, L, K=0, dnum=1, t=0, moduli=None):
    o = Oracle(scheme, log_n, L, K, dnum, t=t, moduli=moduli)
    g = hb.Context(scheme, log_n, L, K, dnum, t=t, moduli=o.moduli)
    assert np.array_equal(g.moduli, o.moduli)
    return o, g


def load(name):
    return np.load(os.path.join(GOLD, name))


# --------------------------------------------------------------------- NTT
def test_ntt_golden(hb):
    g = load("ntt_n1024.npz")
    o, c = pair(hb, SCHEME_CKKS, 10, 3, moduli=g["moduli"])
    x = hb.to_device(g["x"])
    c.ntt_fwd(x)
    assert np.array_equal(hb.to_host(x), g["y"])
    c.ntt_inv(x)
    assert np.array_equal(hb.to_host(x), g["x"])


@pytest.mark.parametrize("log_n,L,polys", [(10, 2, 3), (11, 2, 1), (12, 3, 2), (13, 2, 1), (14, 4, 2),
                                            (15, 3, 1), (16, 4, 2), (17, 2, 1)])
def test_ntt_vs_oracle(hb, log_n, L, polys):
    o, c = pair(hb, SCHEME_CKKS, log_n, L)
    x = o.uniform((polys, L, 1 << log_n), seed=log_n * 131 + L)
    want = o.ntt_fwd(x)
    d = hb.to_device(x)
    c.ntt_fwd(d)
    assert np.array_equal(hb.to_host(d), want)
    c.ntt_inv(d)
    assert np.array_equal(hb.to_host(d), x)
    # inverse from an arbitrary (non-NTT-image) canonical input too
    d = hb.to_device(x)
    c.ntt_inv(d)
    assert np.array_equal(hb.to_host(d), o.ntt_inv(x))


@pytest.mark.parametrize("log_n,L,K", [(12, 2, 1), (15, 2, 1), (16, 3, 2)])
def test_ntt_fwd_lazy_inputs(hb, log_n, L, K):
    """The forward NTT accepts lazy inputs in [0, 4q) (the oracle's Harvey bound)
    on both lazy schedules: the wide one (60-bit Q primes, reductions skipped
    down to 7 of 16 stages) and the narrow one (61-bit P primes)."""
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K=K, dnum=1)
    n, nm = 1 << log_n, L + K
    x = o.uniform((2, nm, n), seed=log_n * 7 + nm)
    q = np.asarray(o.moduli[:nm], dtype=np.uint64)[None, :, None]
    lazy = x + (np.arange(2 * nm * n, dtype=np.uint64).reshape(2, nm, n) % np.uint64(4)) * q
    lazy[0, :, :8] = 4 * q[0] - np.uint64(1)  # the top of the range
    assert int(lazy.max()) < 4 * int(max(o.moduli[:nm]))
    want = o.ntt_fwd(x)
    d = hb.to_device(lazy)
    c.ntt_fwd(d)
    want_top = o.ntt_fwd(np.where(np.arange(n)[None, None, :] < 8, (4 * q - np.uint64(1)) % q, x)[:1])
    got = hb.to_host(d)
    assert np.array_equal(got[1:], want[1:])
    assert np.array_equal(got[:1], want_top)


def test_ntt_c2_config(hb):
    """BASELINE.json configs[1]: forward+inverse NTT, N=2^14, 4 limbs, bit-exact vs CPU."""
    o, c = pair(hb, SCHEME_CKKS, 14, 4)
    x = o.uniform((8, 4, 1 << 14), seed=2)
    d = hb.to_device(x)
    c.ntt_fwd(d)
    assert np.array_equal(hb.to_host(d), o.ntt_fwd(x))
    c.ntt_inv(d)
    assert np.array_equal(hb.to_host(d), x)


def test_ntt_p_part_mod_offset(hb):
    o, c = pair(hb, SCHEME_CKKS, 12, 3, K=2, dnum=3)
    x = o.uniform((2, 2, 1 << 12), seed=9, mod_begin=3)
    d = hb.to_device(x)
    c.ntt_fwd(d, mod_begin=3)
    assert np.array_equal(hb.to_host(d), o.ntt_fwd(x, mod_begin=3))


def test_fill_uniform_matches_oracle(hb):
    o, c = pair(hb, SCHEME_CKKS, 12, 3)
    d = hb.empty((2, 3, 1 << 12))
    c.fill_uniform(d, seed=77)
    assert np.array_equal(hb.to_host(d), o.uniform((2, 3, 1 << 12), seed=77))


def test_poly_ops(hb):
    o, c = pair(hb, SCHEME_CKKS, 11, 3)
    a = o.uniform((2, 3, 1 << 11), seed=1)
    b = o.uniform((2, 3, 1 << 11), seed=2)
    da, db, dout = hb.to_device(a), hb.to_device(b), hb.empty(a.shape)
    for op in ("add", "sub", "mul"):
        c.poly_op(op, da, db, dout)
        want = np.zeros_like(a)
        getattr(o.lib, f"orc_{op}")(o.h, a, b, want, 2, 0, 3)
        assert np.array_equal(hb.to_host(dout), want), op


def test_base_conv_golden(hb):
    g = load("conv_n1024.npz")
    c = hb.Context(SCHEME_CKKS, int(g["log_n"]), len(g["moduli"]), moduli=g["moduli"])
    x = hb.to_device(g["x"][None])
    y = hb.empty((1, len(g["dst"]), 1 << int(g["log_n"])))
    c.base_conv(x, g["src"], y, g["dst"])
    assert np.array_equal(hb.to_host(y)[0], g["y"])


# -------------------------------------------------------------------- CKKS
def test_ckks_golden(hb):
    g = load("ckks_n1024_l4.npz")
    o, c = pair(hb, SCHEME_CKKS, 10, 4, 2, 2, moduli=g["moduli"])
    a, b = hb.to_device(g["a"][None]), hb.to_device(g["b"][None])
    rlk, gk = hb.to_device(g["rlk"]), hb.to_device(g["gk"])
    out = hb.empty(a.shape)
    c.mul_relin(a, b, rlk, out)
    assert np.array_equal(hb.to_host(out)[0], g["out_mul"])
    c.rotate(a, int(g["g"]), gk, out)
    assert np.array_equal(hb.to_host(out)[0], g["out_rot"])
    c.rotate(b, int(g["g_conj"]), gk, out)
    assert np.array_equal(hb.to_host(out)[0], g["out_conj"])


@pytest.mark.parametrize("log_n,L,K,dnum,n_ct", [(12, 5, 2, 3, 3), (16, 12, 4, 3, 2), (15, 5, 2, 2, 3),
                                                (17, 3, 2, 3, 1)])
def test_ckks_mul_relin_vs_oracle(hb, log_n, L, K, dnum, n_ct):
    """(16, 12, 4, 3) is the BASELINE metric config (ct-mult+relin, N=2^16, L=12).
    log_n 15..17 run the two-pass NTT whose last pass carries the fused ModDown finish
    (ragged digits at 15).  There the call with a separate output splits the tensor
    product (d2 in INTT(d2)'s first pass, d0 / d1 in the ModDown finish: PRO_TENSOR2 +
    EPI_KSQT); the in-place call takes the unsplit path (ckks_mul_relin_impl)."""
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K, dnum)
    a = o.uniform((n_ct, 2, L, 1 << log_n), seed=10)
    b = o.uniform((n_ct, 2, L, 1 << log_n), seed=11)
    rlk = o.uniform(o.key_shape(), seed=12)
    want = o.mul_relin(a, b, rlk)
    da, db, dk, dout = hb.to_device(a), hb.to_device(b), hb.to_device(rlk), hb.empty(a.shape)
    c.mul_relin(da, db, dk, dout)
    assert np.array_equal(hb.to_host(dout), want)
    # in-place output aliasing the first operand
    c.mul_relin(da, db, dk, da)
    assert np.array_equal(hb.to_host(da), want)


def test_ckks_rotate_c4(hb):
    """BASELINE.json configs[3]: CKKS rotate + hybrid KS (dnum=3), N=2^16, L=12."""
    o, c = pair(hb, SCHEME_CKKS, 16, 12, 4, 3)
    ct = o.uniform((2, 2, 12, 1 << 16), seed=20)
    gk = o.uniform(o.key_shape(), seed=21)
    for steps in (1, -7):
        g = o.galois_elt(steps)
        want = o.rotate(ct, g, gk)
        dct, dgk, dout = hb.to_device(ct), hb.to_device(gk), hb.empty(ct.shape)
        c.rotate(dct, g, dgk, dout)
        assert np.array_equal(hb.to_host(dout), want), steps


@pytest.mark.parametrize("log_n,L,K,dnum", [(13, 7, 3, 3), (15, 8, 2, 4), (15, 5, 1, 5), (12, 12, 2, 12),
                                            (12, 18, 2, 18), (15, 10, 4, 2), (15, 4, 2, 1)])
def test_keyswitch_vs_oracle(hb, log_n, L, K, dnum):
    """(13,7,3,3): ragged digits (alpha=3, last digit 1 limb); (15,8,2,4): 4 digits;
    (15,5,1,5): 5 single-limb digits; 12 and 18 digits: the register-cached (<= 16) and
    streamed (> 16) key paths of the inner product; (15,10,4,2): alpha 5, so the fused
    ModDown (and its fused Q-limb inner product) runs after the separate ModUp kernel;
    (15,4,2,1): one digit (the inner product fused into the finish with one term)."""
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K, dnum)
    d = o.uniform((2, L, 1 << log_n), seed=30)
    k = o.uniform(o.key_shape(), seed=31)
    want = o.keyswitch(d, k)
    dout = hb.empty(want.shape)
    c.keyswitch(hb.to_device(d), hb.to_device(k), dout)
    assert np.array_equal(hb.to_host(dout), want)


@pytest.mark.parametrize("log_n,sparse", [(12, False), (16, True)])
def test_ckks_real_keys_decrypt(hb, log_n, sparse):
    """Real keys, decrypt, CRT: the product's error stays far below Delta^2.  At
    N = 2^16 the whole fused pipeline runs (tensor in INTT(d2), ModUp and ModDown
    inside the NTT column passes, the combine epilogue); the first message is
    sparse there so the exact negacyclic reference stays cheap."""
    o, c = pair(hb, SCHEME_CKKS, log_n, 4, 2, 2)
    Q = [int(q) for q in o.moduli[:o.L]]
    s = o.secret(3)
    s_qp = o.signed_to_rns(s, 0, o.L + o.K, ntt=True)
    qs = np.asarray(o.moduli[:o.L + o.K], dtype=object)[:, None]
    sq = ((s_qp.astype(object) * s_qp.astype(object)) % qs).astype(np.uint64)
    rlk = o.switch_key(sq, s_qp, seed=4)
    rng = random.Random(5)
    delta = 1 << 30
    if sparse:
        u1 = [0] * o.n
        for k in rng.sample(range(o.n), 48):
            u1[k] = rng.choice([-4, -3, -2, -1, 1, 2, 3, 4])
    else:
        u1 = [rng.randint(-4, 4) for _ in range(o.n)]
    u2 = [rng.randint(-4, 4) for _ in range(o.n)]
    c1 = o.encrypt(to_rns([delta * x for x in u1], Q), s_qp, 1)
    c2 = o.encrypt(to_rns([delta * x for x in u2], Q), s_qp, 2)
    dout = hb.empty((1, 2, o.L, o.n))
    c.mul_relin(hb.to_device(c1[None]), hb.to_device(c2[None]), hb.to_device(rlk), dout)
    dec = crt_centered(o.decrypt(hb.to_host(dout)[0], s_qp), Q)
    want = [delta * delta * v for v in negacyclic_int(u1, u2)]
    assert max(abs(x - y) for x, y in zip(dec, want)) < 2 ** 56


def _tree_expected(o, cts, combine):
    """fhe_reduce's pairing: item i < live/2 absorbs item i + live - live/2."""
    cts = cts.copy()
    live = cts.shape[0]
    while live > 1:
        half = live // 2
        cts[:half] = combine(cts[:half], cts[live - half:live])
        live -= half
    return cts[:1]


def test_reduce_tree_ckks(hb):
    """fhe_reduce (ReduceTask evaluation): add and mul+relin trees
    over an odd count, bit-exact against the oracle's ops in the same pairing."""
    o, c = pair(hb, SCHEME_CKKS, 12, 3, 2, 2)
    cts = o.uniform((5, 2, 3, 1 << 12), seed=80)
    rlk = o.uniform(o.key_shape(), seed=81)
    want_add = _tree_expected(o, cts, o.ct_add)
    want_mul = _tree_expected(o, cts, lambda a, b: o.mul_relin(a, b, rlk))
    d = hb.to_device(cts)
    out = hb.empty((1, 2, 3, 1 << 12))
    c.reduce(d, hb.REDUCE_ADD, out=out)
    assert np.array_equal(hb.to_host(out), want_add)
    d = hb.to_device(cts)
    c.reduce(d, hb.REDUCE_MUL_RELIN, hb.to_device(rlk), out=out)
    assert np.array_equal(hb.to_host(out), want_mul)
    one = hb.to_device(cts[:1])
    c.reduce(one, hb.REDUCE_ADD, out=out)
    assert np.array_equal(hb.to_host(out), cts[:1])


# --------------------------------------------------------------------- BFV
def test_bfv_golden(hb):
    g = load("bfv_n1024_l4.npz")
    o, c = pair(hb, SCHEME_BFV, 10, 4, 2, 2, t=int(g["t"]), moduli=g["moduli"])
    a, b = hb.to_device(g["a"][None]), hb.to_device(g["b"][None])
    rlk = hb.to_device(g["rlk"])
    out = hb.empty(a.shape)
    c.add(a, b, out)
    assert np.array_equal(hb.to_host(out)[0], g["out_add"])
    c.mul_relin(a, b, rlk, out)
    assert np.array_equal(hb.to_host(out)[0], g["out_mul"])
    c.rotate(a, int(g["g"]), rlk, out)
    assert np.array_equal(hb.to_host(out)[0], g["out_rot"])


def test_bfv_c1_add(hb):
    """BASELINE.json configs[0]: BFV add, N=4096, one 60-bit prime."""
    o, c = pair(hb, SCHEME_BFV, 12, 1, 1, 1, t=65537)
    a = o.uniform((4, 2, 1, 4096), seed=40)
    b = o.uniform((4, 2, 1, 4096), seed=41)
    out = hb.empty(a.shape)
    c.add(hb.to_device(a), hb.to_device(b), out)
    assert np.array_equal(hb.to_host(out), o.ct_add(a, b))


def test_bfv_mul_relin_c3(hb):
    """BASELINE.json configs[2]: BFV ct x ct multiply + relinearize, N=2^15, L=8."""
    o, c = pair(hb, SCHEME_BFV, 15, 8, 4, 2, t=65537)
    a = o.uniform((2, 2, 8, 1 << 15), seed=50)
    b = o.uniform((2, 2, 8, 1 << 15), seed=51)
    rlk = o.uniform(o.key_shape(), seed=52)
    want = o.mul_relin(a, b, rlk)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), want)


def test_bfv_real_keys_exact(hb):
    t = 65537
    o, c = pair(hb, SCHEME_BFV, 12, 3, 3, 1, t=t)
    Q = [int(q) for q in o.moduli[:o.L]]
    Qp = math.prod(Q)
    s = o.secret(8)
    s_qp = o.signed_to_rns(s, 0, o.L + o.K, ntt=True)
    sq = np.array([[(int(x) * int(x)) % int(o.moduli[i]) for x in s_qp[i]] for i in range(o.L + o.K)],
                  dtype=np.uint64)
    rlk = o.switch_key(sq, s_qp, seed=9)
    rng = random.Random(10)
    m1 = [rng.randrange(t) for _ in range(o.n)]
    m2 = [rng.randrange(t) for _ in range(o.n)]
    delta = Qp // t
    c1 = o.encrypt(to_rns([delta * x for x in m1], Q), s_qp, 11)
    c2 = o.encrypt(to_rns([delta * x for x in m2], Q), s_qp, 12)
    dout = hb.empty((1, 2, o.L, o.n))
    c.mul_relin(hb.to_device(c1[None]), hb.to_device(c2[None]), hb.to_device(rlk), dout)
    v = crt_centered(o.decrypt(hb.to_host(dout)[0], s_qp), Q)
    dec = [((t * x + Qp // 2) // Qp) % t for x in v]
    assert dec == [x % t for x in negacyclic_int(m1, m2)]
    g = o.galois_elt(3)
    gk = o.switch_key(o.automorph_ntt(s_qp, g), s_qp, seed=13)
    c.rotate(hb.to_device(c1[None]), g, hb.to_device(gk), dout)
    v = crt_centered(o.decrypt(hb.to_host(dout)[0], s_qp), Q)
    assert [((t * x + Qp // 2) // Qp) % t for x in v] == [x % t for x in automorph_int(m1, g)]


# ------------------------------------------------- generic (non 2^32) moduli
def _generic_primes(bits, log_n, count):
    """q = 1 mod 2N but q != 1 mod 2^32: exercises the generic Montgomery path."""
    import bigint_model as M
    two_n = 2 << log_n
    out, k = [], ((1 << bits) - 2) // two_n
    while len(out) < count:
        q = k * two_n + 1
        if q % (1 << 32) != 1 and M.is_prime(q):
            out.append(q)
        k -= 1
    return out


def test_generic_moduli_ckks(hb):
    log_n, L, K, dnum = 13, 4, 2, 2
    mods = np.array(_generic_primes(60, log_n, L + K), dtype=np.uint64)
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K, dnum, moduli=mods)
    a = o.uniform((2, 2, L, 1 << log_n), seed=60)
    b = o.uniform((2, 2, L, 1 << log_n), seed=61)
    k = o.uniform(o.key_shape(), seed=62)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(k), dout)
    assert np.array_equal(hb.to_host(dout), o.mul_relin(a, b, k))
    g = o.galois_elt(2)
    c.rotate(hb.to_device(a), g, hb.to_device(k), dout)
    assert np.array_equal(hb.to_host(dout), o.rotate(a, g, k))


@pytest.mark.parametrize("bits", [[60] * 4, [61] * 4, [60, 61, 60, 61]])
def test_generic_moduli_c2_persistent(hb, bits):
    """C2's shape (N=2^14, 4 limbs) on OpenFHE-style primes: the persistent
    one-pass kernel on the generic Montgomery path (round 6) for each lazy-
    schedule class (60-bit: wide, 61-bit: narrow), and a launch mixing both
    (two passes), forward and inverse, against the oracle, from lazy inputs too."""
    log_n = 14
    mods = []
    for b in bits:
        mods.append(next(q for q in _generic_primes(b, log_n, len(mods) + 1) if q not in mods))
    mods = np.array(mods, dtype=np.uint64)
    o, c = pair(hb, SCHEME_CKKS, log_n, 4, moduli=mods)
    x = o.uniform((9, 4, 1 << log_n), seed=sum(bits))
    d = hb.to_device(x)
    c.ntt_fwd(d)
    assert np.array_equal(hb.to_host(d), o.ntt_fwd(x))
    c.ntt_inv(d)
    assert np.array_equal(hb.to_host(d), x)
    d = hb.to_device(x)
    c.ntt_inv(d)
    assert np.array_equal(hb.to_host(d), o.ntt_inv(x))
    q = np.asarray(o.moduli[:4], dtype=np.uint64)[None, :, None]
    lazy = x + (np.arange(x.size, dtype=np.uint64).reshape(x.shape) % np.uint64(4)) * q  # [0, 4q)
    d = hb.to_device(lazy)
    c.ntt_fwd(d)
    assert np.array_equal(hb.to_host(d), o.ntt_fwd(x))


def test_generic_moduli_ntt_and_bfv(hb):
    log_n, L, K, dnum = 15, 3, 2, 2
    mods = np.array(_generic_primes(60, log_n, 2 * L + K + 1), dtype=np.uint64)
    o, c = pair(hb, SCHEME_BFV, log_n, L, K, dnum, t=65537, moduli=mods)
    x = o.uniform((3, L, 1 << log_n), seed=70)
    d = hb.to_device(x)
    c.ntt_fwd(d)
    assert np.array_equal(hb.to_host(d), o.ntt_fwd(x))
    a = o.uniform((1, 2, L, 1 << log_n), seed=71)
    b = o.uniform((1, 2, L, 1 << log_n), seed=72)
    k = o.uniform(o.key_shape(), seed=73)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(k), dout)
    assert np.array_equal(hb.to_host(dout), o.mul_relin(a, b, k))


# ---------------------------------------------------------------- errors
def test_errors_are_loud(hb):
    c = hb.Context(SCHEME_CKKS, 12, 2)
    x = hb.empty((1, 2, 1 << 12))
    with pytest.raises(hb.FheBackendError):
        c.ntt_fwd(x, mod_begin=5)  # out of modulus range
    with pytest.raises(hb.FheBackendError):
        c.mul_relin(hb.empty((1, 2, 2, 1 << 12)), hb.empty((1, 2, 2, 1 << 12)), x, hb.empty((1, 2, 2, 1 << 12)))
    with pytest.raises(hb.FheBackendError):
        hb.Context(SCHEME_CKKS, 9, 2)  # N below the supported range
    with pytest.raises(hb.FheBackendError, match="CKKS context"):
        hb.Context(SCHEME_CKKS, 12, 2, 1, 1, bfv_mult="hps")  # HPS is a BFV technique
    with pytest.raises(hb.FheBackendError, match="unknown BFV"):
        hb.Context(SCHEME_BFV, 12, 2, 1, 1, t=65537, bfv_mult="behz+")


# ------------------------------------------------------------ edge values
def _edge_inputs(o, shape, seed):
    """Residues at the boundaries of the Montgomery / lazy-reduction ranges:
    0 (every partial product word zero: the folded carries must vanish), 1,
    q-1, q-2 and 2^32-multiples (zero low words), mixed with uniform words."""
    x = o.uniform(shape, seed=seed)
    nl = shape[-2]
    flat = x.reshape(-1, nl, shape[-1])
    for li in range(nl):
        q = int(o.moduli[li])
        specials = np.array([0, 1, q - 1, q - 2, 1 << 32, (q - 1) & ~0xFFFFFFFF, q >> 1], dtype=np.uint64)
        flat[:, li, : specials.size] = specials
        flat[:, li, specials.size: 2 * specials.size] = specials[::-1]
    flat[0, :, :] = 0  # one all-zero polynomial
    return x


@pytest.mark.parametrize("log_n,L", [(12, 3), (16, 4)])
def test_ntt_edge_values(hb, log_n, L):
    o, c = pair(hb, SCHEME_CKKS, log_n, L)
    x = _edge_inputs(o, (3, L, 1 << log_n), seed=90)
    d = hb.to_device(x)
    c.ntt_fwd(d)
    y = o.ntt_fwd(x.copy())
    assert np.array_equal(hb.to_host(d), y)
    c.ntt_inv(d)
    assert np.array_equal(hb.to_host(d), x)


@pytest.mark.parametrize("log_n", [12, 16])
def test_ckks_mul_relin_edge_values(hb, log_n):
    L, K, dnum = (5, 2, 3) if log_n == 12 else (12, 4, 3)
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K, dnum)
    a = _edge_inputs(o, (2, 2, L, 1 << log_n), seed=91)
    b = _edge_inputs(o, (2, 2, L, 1 << log_n), seed=92)
    b[1] = 0  # ct x zero ciphertext
    rlk = o.uniform(o.key_shape(), seed=93)
    want = o.mul_relin(a, b, rlk)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), want)


def test_bfv_mul_relin_edge_values(hb):
    o, c = pair(hb, SCHEME_BFV, 13, 3, 2, 2, t=65537)
    a = _edge_inputs(o, (2, 2, 3, 1 << 13), seed=94)
    b = _edge_inputs(o, (2, 2, 3, 1 << 13), seed=95)
    rlk = o.uniform(o.key_shape(), seed=96)
    want = o.mul_relin(a, b, rlk)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), want)


def test_empty_batches_are_no_ops(hb):
    o, c = pair(hb, SCHEME_CKKS, 12, 3, 2, 2)
    z = hb.empty((0, 2, 3, 1 << 12))
    k = hb.to_device(o.uniform(o.key_shape(), seed=97))
    c.mul_relin(z, z, k, z)
    c.rotate(z, c.galois_elt(1), k, z)
    c.add(z, z, z)
    c.keyswitch(hb.empty((0, 3, 1 << 12)), k, z)
    c.ntt_fwd(hb.empty((0, 3, 1 << 12)))


def test_graph_capture_replay(hb):
    """With the scratch pre-sized (fhe_reserve), a mul+relin step captures into a
    HIP graph (torch.cuda.CUDAGraph) and its replays are bit-exact."""
    import torch
    o, c = pair(hb, SCHEME_CKKS, 13, 4, 2, 2)
    a = o.uniform((3, 2, 4, 1 << 13), seed=100)
    b = o.uniform((3, 2, 4, 1 << 13), seed=101)
    rlk = o.uniform(o.key_shape(), seed=102)
    want = o.mul_relin(a, b, rlk)
    da, db, dk, dout = hb.to_device(a), hb.to_device(b), hb.to_device(rlk), hb.empty(a.shape)
    c.reserve(3)
    main = torch.cuda.current_stream()
    c.set_stream(main)
    c.mul_relin(da, db, dk, dout)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        c.set_stream(torch.cuda.current_stream())
        c.mul_relin(da, db, dk, dout)
    c.set_stream(main)
    dout.zero_()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(hb.to_host(dout), want)


@pytest.mark.parametrize("scheme,log_n,L,K,dnum", [(SCHEME_CKKS, 12, 32, 16, 2), (SCHEME_CKKS, 15, 20, 8, 5),
                                                   (SCHEME_BFV, 12, 15, 4, 3)])
def test_large_modulus_counts(hb, scheme, log_n, L, K, dnum):
    """The widest shapes the context accepts: 48 moduli with 16-limb digits (ModUp/ModDown
    NS=16 paths), 5 digits at a two-pass size, and BFV with a 16-modulus BEHZ base."""
    t = 65537 if scheme == SCHEME_BFV else 0
    o, c = pair(hb, scheme, log_n, L, K, dnum, t=t)
    a = o.uniform((2, 2, L, 1 << log_n), seed=110)
    b = o.uniform((2, 2, L, 1 << log_n), seed=111)
    rlk = o.uniform(o.key_shape(), seed=112)
    want = o.mul_relin(a, b, rlk)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), want)
    g = o.galois_elt(3)
    want_r = o.rotate(a, g, rlk)
    c.rotate(hb.to_device(a), g, hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), want_r)


def test_large_batches_are_chunked(hb):
    """Batches beyond one launch's grid (2^16 (item, limb) rows) and beyond one
    internal ciphertext pass (kCtChunk = 512) give the same bits as the oracle."""
    o, c = pair(hb, SCHEME_CKKS, 10, 2, 1, 1)
    n_big = 20000  # 2 * 20000 * 2 = 80000 (item, limb) rows
    a = o.uniform((n_big, 2, 2, 1 << 10), seed=120)
    b = o.uniform((n_big, 2, 2, 1 << 10), seed=121)
    da = c.fill_uniform(hb.empty(a.shape), seed=120)
    assert np.array_equal(hb.to_host(da), a)
    dout = hb.empty(a.shape)
    c.add(da, hb.to_device(b), dout)
    assert np.array_equal(hb.to_host(dout), o.ct_add(a, b))
    n = 600
    rlk = o.uniform(o.key_shape(), seed=122)
    want = o.mul_relin(a[:n], b[:n], rlk)
    dout = hb.empty((n, 2, 2, 1 << 10))
    c.mul_relin(hb.to_device(a[:n]), hb.to_device(b[:n]), hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), want)
    g = o.galois_elt(5)
    c.rotate(hb.to_device(a[:n]), g, hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), o.rotate(a[:n], g, rlk))


def test_rccl_entry_points_single_rank(hb):
    """fhe_bcast_key and fhe_reduce_ranks on a real one-rank RCCL communicator (the
    box has one GPU): the calls go through RCCL and leave the data as it is."""
    import ctypes as C
    import torch
    # the communicator must come from the RCCL instance libherdsman_fhe.so bound to:
    # in a process that imported torch that is torch's bundled librccl.so.1, which a
    # soname lookup returns (a second copy would see a "corrupted comm object")
    hb.load_library()
    rccl = C.CDLL("librccl.so.1")
    comm = C.c_void_p()
    dev = (C.c_int * 1)(0)
    assert rccl.ncclCommInitAll(C.byref(comm), 1, dev) == 0
    try:
        o, c = pair(hb, SCHEME_CKKS, 12, 3, 2, 2)
        key = o.uniform(o.key_shape(), seed=130)
        dk = hb.to_device(key)
        lib = hb.load_library()
        rc = lib.fhe_bcast_key(c.h, dk.data_ptr(), key.size, comm, 0)
        assert rc == 0, lib.fhe_last_error(c.h)
        ct = o.uniform((1, 2, 3, 1 << 12), seed=131)
        dct, tmp = hb.to_device(ct), hb.empty(ct.shape)
        assert lib.fhe_reduce_ranks(c.h, dct.data_ptr(), hb.REDUCE_ADD, None, comm, 0, tmp.data_ptr()) == 0
        torch.cuda.synchronize()
        assert np.array_equal(hb.to_host(dk), key)
        assert np.array_equal(hb.to_host(dct), ct)
        assert lib.fhe_reduce_ranks(c.h, dct.data_ptr(), 7, None, comm, 0, tmp.data_ptr()) == hb.FHE_ERR_INVALID
        # the same join on a level-2 ciphertext (a level view of the context)
        ct2 = np.ascontiguousarray(ct[:, :, :2])
        d2, t2 = hb.to_device(ct2), hb.empty(ct2.shape)
        rc = lib.fhe_reduce_ranks_at(c.h, d2.data_ptr(), hb.REDUCE_ADD, None, comm, 0, t2.data_ptr(), 2)
        assert rc == 0, lib.fhe_last_error(c.h)
        torch.cuda.synchronize()
        assert np.array_equal(hb.to_host(d2), ct2)
    finally:
        rccl.ncclCommDestroy(comm)


@pytest.mark.parametrize("scheme", [SCHEME_CKKS, SCHEME_BFV])
def test_conjugation_and_identity_galois(hb, scheme):
    """Galois elements 2N-1 (conjugation) and 1 (identity automorphism + key switch)."""
    t = 65537 if scheme == SCHEME_BFV else 0
    o, c = pair(hb, scheme, 12, 4, 2, 2, t=t)
    ct = o.uniform((2, 2, 4, 1 << 12), seed=140)
    gk = o.uniform(o.key_shape(), seed=141)
    dout = hb.empty(ct.shape)
    for g in (2 * o.n - 1, 1):
        c.rotate(hb.to_device(ct), g, hb.to_device(gk), dout)
        assert np.array_equal(hb.to_host(dout), o.rotate(ct, g, gk)), g


@pytest.mark.parametrize("log_n,L,K,dnum", [(15, 5, 2, 2), (17, 3, 1, 3)])
def test_ckks_rotate_fused_automorphism(hb, log_n, L, K, dnum):
    """Two-pass sizes run the automorphism inside the first INTT pass (PRO_AUTOMORPH):
    generic rotations, conjugation (2N-1), identity (1), and an in-place call."""
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K, dnum)
    ct = o.uniform((2, 2, L, 1 << log_n), seed=150 + log_n)
    gk = o.uniform(o.key_shape(), seed=151 + log_n)
    dgk = hb.to_device(gk)
    dout = hb.empty(ct.shape)
    for g in (o.galois_elt(1), o.galois_elt(-5), 2 * o.n - 1, 1):
        c.rotate(hb.to_device(ct), g, dgk, dout)
        assert np.array_equal(hb.to_host(dout), o.rotate(ct, g, gk)), g
    g = o.galois_elt(7)
    dct = hb.to_device(ct)
    c.rotate(dct, g, dgk, dct)
    assert np.array_equal(hb.to_host(dct), o.rotate(ct, g, gk))


@pytest.mark.parametrize("log_n,L,K,dnum", [(16, 3, 2, 3), (17, 2, 1, 2)])
def test_bfv_mul_relin_fused_tensor_sizes(hb, log_n, L, K, dnum):
    """The BFV tensor product runs inside the first pass of INTT(eq)/INTT(eb)
    (PRO_BFVT) at every two-pass ring size; 3 products so every (ct, e) poly
    index is hit, plus an in-place call (out aliases a)."""
    o, c = pair(hb, SCHEME_BFV, log_n, L, K, dnum, t=65537)
    a = o.uniform((3, 2, L, 1 << log_n), seed=160 + log_n)
    b = o.uniform((3, 2, L, 1 << log_n), seed=161 + log_n)
    rlk = o.uniform(o.key_shape(), seed=162 + log_n)
    want = o.mul_relin(a, b, rlk)
    da = hb.to_device(a)
    c.mul_relin(da, hb.to_device(b), hb.to_device(rlk), da)
    assert np.array_equal(hb.to_host(da), want)


@pytest.mark.parametrize("bits", [0, 60, 61])
def test_bfv_fused_tensor_row_passes_edge_values(hb, bits):
    """BFV mul+relin at N=2^15 runs the forward row passes, the tensor product
    and the inverse row passes in one kernel per base (bfvt_fused_pass,
    ntt_bfvt.hip): edge residues (0, 1, q-1, 2^32 multiples, a zero ciphertext)
    on the default special primes (bits 0) and on generic primes of both
    lazy-schedule classes (60: wide, 61: narrow), plus an in-place call."""
    log_n, L, K, dnum = 15, 3, 2, 2
    mods = np.array(_generic_primes(bits, log_n, 2 * L + K + 1), dtype=np.uint64) if bits else None
    o, c = pair(hb, SCHEME_BFV, log_n, L, K, dnum, t=65537, moduli=mods)
    a = _edge_inputs(o, (2, 2, L, 1 << log_n), seed=170 + bits)
    b = _edge_inputs(o, (2, 2, L, 1 << log_n), seed=171 + bits)
    b[1] = 0
    rlk = o.uniform(o.key_shape(), seed=172 + bits)
    want = o.mul_relin(a, b, rlk)
    da = hb.to_device(a)
    c.mul_relin(da, hb.to_device(b), hb.to_device(rlk), da)
    assert np.array_equal(hb.to_host(da), want)


def test_generic_moduli_metric_size(hb):
    """OpenFHE-style primes at the metric parameters (N=2^16, L=12, K=4, dnum=3;
    60-bit Q on the wide lazy schedule, 61-bit P on the narrow one): the fused
    mul+relin pipeline on the generic 32-bit CIOS Montgomery product, edge
    values (0, 1, q-1) included, and an NTT round trip of edge values."""
    log_n, L, K, dnum = 16, 12, 4, 3
    mods = np.array(_generic_primes(60, log_n, L) + _generic_primes(61, log_n, K), dtype=np.uint64)
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K, dnum, moduli=mods)
    a = _edge_inputs(o, (1, 2, L, 1 << log_n), seed=180)
    b = _edge_inputs(o, (1, 2, L, 1 << log_n), seed=181)
    k = o.uniform(o.key_shape(), seed=182)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(k), dout)
    assert np.array_equal(hb.to_host(dout), o.mul_relin(a, b, k))
    x = _edge_inputs(o, (2, L + K, 1 << log_n), seed=183)
    d = hb.to_device(x)
    c.ntt_fwd(d)
    assert np.array_equal(hb.to_host(d), o.ntt_fwd(x.copy()))
    c.ntt_inv(d)
    assert np.array_equal(hb.to_host(d), x)


def test_generic_moduli_two_pass_fused_paths(hb):
    """Generic (non 2^32) moduli at a two-pass size: the CKKS tensor and
    automorphism prologues and the unscaled inverse NTTs on the generic
    Montgomery path (BFV's tensor prologue: test_generic_moduli_ntt_and_bfv)."""
    log_n, L, K, dnum = 15, 3, 2, 2
    mods = np.array(_generic_primes(60, log_n, L + K), dtype=np.uint64)
    o, c = pair(hb, SCHEME_CKKS, log_n, L, K, dnum, moduli=mods)
    a = o.uniform((2, 2, L, 1 << log_n), seed=170)
    b = o.uniform((2, 2, L, 1 << log_n), seed=171)
    k = o.uniform(o.key_shape(), seed=172)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(k), dout)
    assert np.array_equal(hb.to_host(dout), o.mul_relin(a, b, k))
    g = o.galois_elt(3)
    c.rotate(hb.to_device(a), g, hb.to_device(k), dout)
    assert np.array_equal(hb.to_host(dout), o.rotate(a, g, k))


def test_concurrent_contexts_on_streams(hb):
    """bench.py's configuration: several contexts, one HIP stream each, run
    ct-mult+relin on slices of one batch concurrently with a shared key; every
    slice must match the oracle (per-context workspaces, no cross-talk)."""
    import torch

    log_n, L, K, dnum, S, per = 15, 4, 2, 2, 4, 2
    o, c0 = pair(hb, SCHEME_CKKS, log_n, L, K, dnum)
    ctxs = [c0] + [hb.Context(SCHEME_CKKS, log_n, L, K, dnum, moduli=o.moduli) for _ in range(S - 1)]
    streams = [torch.cuda.Stream() for _ in range(S)]
    for c, s in zip(ctxs, streams):
        c.set_stream(s)
    a = o.uniform((S * per, 2, L, 1 << log_n), seed=180)
    b = o.uniform((S * per, 2, L, 1 << log_n), seed=181)
    k = o.uniform(o.key_shape(), seed=182)
    da, db, dk = hb.to_device(a), hb.to_device(b), hb.to_device(k)
    dout = hb.empty(a.shape)
    torch.cuda.synchronize()
    for rep in range(2):
        for i, c in enumerate(ctxs):
            sl = slice(i * per, (i + 1) * per)
            c.mul_relin(da[sl], db[sl], dk, dout[sl])
    torch.cuda.synchronize()
    assert np.array_equal(hb.to_host(dout), o.mul_relin(a, b, k))


def test_base_conv_contexts_recreated(hb):
    """fhe_base_conv's tables belong to the context.  Contexts with
    different moduli / ring sizes are created, used and destroyed in sequence
    (a freed context's address is typically handed to the next one) with the
    same index lists; every conversion must match the oracle of ITS context."""
    import torch

    src, dst = [0, 1, 2], [3, 4, 5, 6]
    for rep, (log_n, bits) in enumerate([(12, 60), (12, 55), (13, 60), (12, 50)]):
        mods = np.array(_generic_primes(bits, log_n, 7), dtype=np.uint64) if bits != 60 else None
        o = Oracle(SCHEME_CKKS, log_n, 7, moduli=mods)
        c = hb.Context(SCHEME_CKKS, log_n, 7, moduli=o.moduli)
        x = o.uniform((2, 3, 1 << log_n), seed=190 + rep)
        y = hb.empty((2, len(dst), 1 << log_n))
        c.base_conv(hb.to_device(x), src, y, dst)
        c.base_conv(hb.to_device(x), src, y, dst)  # cached table
        torch.cuda.synchronize()
        assert np.array_equal(hb.to_host(y), o.base_conv(x, src, dst)), (log_n, bits)
        c.close()


# ------------------------------------------------------------------ BFV HPS
def hps_pair(hb, log_n, L, K, dnum, t=65537, moduli=None):
    o = Oracle(SCHEME_BFV, log_n, L, K, dnum, t=t, moduli=moduli, bfv_mult="hps")
    g = hb.Context(SCHEME_BFV, log_n, L, K, dnum, t=t, moduli=o.moduli, bfv_mult="hps")
    assert np.array_equal(g.moduli, o.moduli)
    return o, g


def test_bfv_hps_golden(hb):
    """HPS multiplication against the big-int model's restatement (its float
    parts included; the model checks round(t d / Q) on integers)."""
    g = load("bfv_hps_n1024_l4.npz")
    o, c = hps_pair(hb, 10, 4, 2, 2, t=int(g["t"]), moduli=g["moduli"])
    out = hb.empty((1, 2, 4, 1 << 10))
    c.mul_relin(hb.to_device(g["a"][None]), hb.to_device(g["b"][None]), hb.to_device(g["rlk"]), out)
    assert np.array_equal(hb.to_host(out)[0], g["out_mul"])


@pytest.mark.parametrize("log_n,L,K,dnum,n_ct", [(15, 8, 4, 2, 2), (13, 5, 2, 3, 3), (12, 11, 3, 4, 1)])
def test_bfv_hps_mul_relin_vs_oracle(hb, log_n, L, K, dnum, n_ct):
    """(15, 8, 4, 2) is BASELINE C3; L = 5 and 11 take the non-exact-L kernels."""
    o, c = hps_pair(hb, log_n, L, K, dnum)
    a = o.uniform((n_ct, 2, L, 1 << log_n), seed=61)
    b = o.uniform((n_ct, 2, L, 1 << log_n), seed=62)
    rlk = o.uniform(o.key_shape(), seed=63)
    want = o.mul_relin(a, b, rlk)
    dout = hb.empty(a.shape)
    c.mul_relin(hb.to_device(a), hb.to_device(b), hb.to_device(rlk), dout)
    assert np.array_equal(hb.to_host(dout), want)


def test_bfv_hps_edge_values(hb):
    """All-zero, all q-1 and mixed extreme residues (the float sums at their ends)."""
    o, c = hps_pair(hb, 13, 3, 2, 2)
    n = o.n
    qs = o.moduli[:3][None, None, :, None]
    a = np.broadcast_to(qs - 1, (1, 2, 3, n)).astype(np.uint64).copy()
    b = np.zeros((1, 2, 3, n), dtype=np.uint64)
    b[..., ::2] = 1
    b[..., 1::3] = (qs - 1).reshape(1, 1, 3, 1)
    rlk = o.uniform(o.key_shape(), seed=64)
    for x, y in ((a, a), (a, b), (b, b), (np.zeros_like(a), a)):
        want = o.mul_relin(x, y, rlk)
        dout = hb.empty(x.shape)
        c.mul_relin(hb.to_device(x), hb.to_device(y), hb.to_device(rlk), dout)
        assert np.array_equal(hb.to_host(dout), want)


def test_bfv_hps_real_keys_exact(hb):
    """Dec(Mul+Relin(Enc m1, Enc m2)) = m1 m2 mod t with HPS at C3's ring size."""
    t = 65537
    o, c = hps_pair(hb, 15, 8, 4, 2, t=t)
    Q = [int(q) for q in o.moduli[:o.L]]
    Qp = math.prod(Q)
    s = o.secret(18)
    s_qp = o.signed_to_rns(s, 0, o.L + o.K, ntt=True)
    qs = o.moduli[:o.L + o.K].astype(object)[:, None]
    sq = ((s_qp.astype(object) * s_qp.astype(object)) % qs).astype(np.uint64)
    rlk = o.switch_key(sq, s_qp, seed=19)
    rng = random.Random(20)
    m1 = [0] * o.n
    for k in rng.sample(range(o.n), 40):
        m1[k] = rng.randrange(t)
    m2 = [rng.randrange(t) for _ in range(o.n)]
    delta = Qp // t
    c1 = o.encrypt(to_rns([delta * x for x in m1], Q), s_qp, 21)
    c2 = o.encrypt(to_rns([delta * x for x in m2], Q), s_qp, 22)
    dout = hb.empty((1, 2, o.L, o.n))
    c.mul_relin(hb.to_device(c1[None]), hb.to_device(c2[None]), hb.to_device(rlk), dout)
    v = crt_centered(o.decrypt(hb.to_host(dout)[0], s_qp), Q)
    dec = [((t * x + Qp // 2) // Qp) % t for x in v]
    assert dec == [x % t for x in negacyclic_int(m1, m2)]
