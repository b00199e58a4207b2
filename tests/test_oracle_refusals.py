"""The oracle is the checker: it must refuse what it does not implement, as the
GPU ABI does (fhe_backend.cpp ctx_level / ew_level_ok), instead of silently
computing another scheme's result (a BFV
expectation once came from the CKKS-only level product)."""
import numpy as np
import pytest

from oracle_ffi import SCHEME_BFV, SCHEME_CKKS, Oracle, OracleUnsupported

LOG_N, L, K, DNUM, T = 10, 3, 1, 3, 65537


@pytest.fixture(scope="module")
def bfv():
    return Oracle(SCHEME_BFV, LOG_N, L, K, DNUM, t=T)


def _ct(o, lvl, seed):
    return o.uniform((1, 2, lvl, o.n), seed=seed)


@pytest.mark.parametrize("lvl", [1, L - 1])
def test_bfv_reduced_levels_refused(bfv, lvl):
    a, b = _ct(bfv, lvl, 1), _ct(bfv, lvl, 2)
    k = bfv.uniform(bfv.key_shape(), seed=3)
    g = bfv.lib.orc_galois_elt(bfv.h, 1)
    with pytest.raises(OracleUnsupported):
        bfv.mul_relin_at(a, b, k, lvl)
    with pytest.raises(OracleUnsupported):
        bfv.rotate_at(a, g, k, lvl)
    with pytest.raises(OracleUnsupported):
        bfv.keyswitch_at(a[:, 1], k, lvl)
    with pytest.raises(OracleUnsupported):
        bfv.rotate_hoisted_at(a, [g], k[None], lvl)
    with pytest.raises(OracleUnsupported):
        bfv.rotate_sum_hoisted(a, [g], k[None], lvl)


def test_bfv_ckks_only_entries_refused(bfv):
    a = _ct(bfv, L, 4)
    k = bfv.uniform(bfv.key_shape(), seed=5)
    g = bfv.lib.orc_galois_elt(bfv.h, 1)
    pts = bfv.uniform((1, L + K, bfv.n), seed=6)
    with pytest.raises(OracleUnsupported):
        bfv.rescale(a, L)
    with pytest.raises(OracleUnsupported):
        bfv.linear_hoisted(a, [g], k[None], pts)


def test_bfv_full_level_runs_the_bfv_op(bfv):
    """At level L the BFV context's level entry is the BFV product (the GPU's
    fhe_mul_relin_at routes level L to the full context), not the CKKS one."""
    a, b = _ct(bfv, L, 7), _ct(bfv, L, 8)
    k = bfv.uniform(bfv.key_shape(), seed=9)
    assert np.array_equal(bfv.mul_relin_at(a, b, k, L), bfv.mul_relin(a, b, k))
    g = bfv.lib.orc_galois_elt(bfv.h, 1)
    assert np.array_equal(bfv.rotate_at(a, g, k, L), bfv.rotate(a, g, k))


def test_levels_outside_range_refused():
    o = Oracle(SCHEME_CKKS, LOG_N, L, K, DNUM)
    a = _ct(o, L, 10)
    k = o.uniform(o.key_shape(), seed=11)
    with pytest.raises(OracleUnsupported):
        o.mul_relin_at(a, a, k, L + 1)
    with pytest.raises(OracleUnsupported):
        o.rescale(_ct(o, 1, 12), 1)
    # a valid CKKS level still computes
    out = o.mul_relin_at(_ct(o, 2, 13), _ct(o, 2, 14), k, 2)
    assert out.shape == (1, 2, 2, o.n) and out.any()
