"""The C oracle (oracle/fhe_oracle.c) against the big-int golden vectors.

This is what pins the oracle before it is trusted as the checker for the HIP
backend (tests/test_gpu_parity.py).  Fixtures: tests/golden/*.npz, produced by
tests/golden/make_golden.py from oracle/bigint_model.py.
"""
import os

import numpy as np
import pytest

from oracle_ffi import Oracle, SCHEME_BFV, SCHEME_CKKS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name))


def test_prime_generation_matches_model():
    g = load("ckks_n1024_l4.npz")
    o = Oracle(SCHEME_CKKS, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]))
    assert np.array_equal(o.moduli, g["moduli"])


def test_ntt_golden():
    g = load("ntt_n1024.npz")
    o = Oracle(SCHEME_CKKS, int(g["log_n"]), 3, moduli=g["moduli"])
    for i in range(3):
        assert o.lib.orc_psi(o.h, i) == int(g["psi"][i])
    y = o.ntt_fwd(g["x"])
    assert np.array_equal(y, g["y"])
    assert np.array_equal(o.ntt_inv(y), g["x"])


def test_base_conv_golden():
    g = load("conv_n1024.npz")
    o = Oracle(SCHEME_CKKS, int(g["log_n"]), len(g["moduli"]), moduli=g["moduli"])
    y = o.base_conv(g["x"], g["src"], g["dst"])
    assert np.array_equal(y[0], g["y"])


def _ckks():
    g = load("ckks_n1024_l4.npz")
    o = Oracle(SCHEME_CKKS, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), moduli=g["moduli"])
    return g, o


def test_ckks_mul_relin_golden():
    g, o = _ckks()
    out = o.mul_relin(g["a"][None], g["b"][None], g["rlk"])
    assert np.array_equal(out[0], g["out_mul"])


def test_ckks_rotate_golden():
    g, o = _ckks()
    out = o.rotate(g["a"][None], int(g["g"]), g["gk"])
    assert np.array_equal(out[0], g["out_rot"])
    out = o.rotate(g["b"][None], int(g["g_conj"]), g["gk"])
    assert np.array_equal(out[0], g["out_conj"])


def _bfv():
    g = load("bfv_n1024_l4.npz")
    o = Oracle(SCHEME_BFV, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), t=int(g["t"]),
               moduli=g["moduli"])
    return g, o


def test_bfv_add_golden():
    g, o = _bfv()
    assert np.array_equal(o.ct_add(g["a"][None], g["b"][None])[0], g["out_add"])


def test_bfv_mul_relin_golden():
    g, o = _bfv()
    out = o.mul_relin(g["a"][None], g["b"][None], g["rlk"])
    assert np.array_equal(out[0], g["out_mul"])


def test_bfv_rotate_golden():
    g, o = _bfv()
    out = o.rotate(g["a"][None], int(g["g"]), g["rlk"])
    assert np.array_equal(out[0], g["out_rot"])


def _levels():
    g = load("ckks_levels_n1024_l5.npz")
    o = Oracle(SCHEME_CKKS, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), moduli=g["moduli"])
    return g, o


def test_ckks_level_mul_relin_golden():
    """mul+relin at levels 4 (partial second digit) and 2 (one partial digit)
    with the full-level key's Q_lvl u P rows (oracle/bigint_model.py keyswitch(lvl))."""
    g, o = _levels()
    for lvl in (4, 2):
        out = o.mul_relin_at(g[f"a{lvl}"][None], g[f"b{lvl}"][None], g["rlk"], lvl)
        assert np.array_equal(out[0], g[f"mul{lvl}"]), lvl


def test_ckks_level_rotate_golden():
    g, o = _levels()
    out = o.rotate_at(g["a3"][None], int(g["g"]), g["rlk"], 3)
    assert np.array_equal(out[0], g["rot3"])


def test_ckks_rescale_golden():
    """The RNS rescale equals round(c / q_last) on CRT-reconstructed integers."""
    g, o = _levels()
    r4 = o.rescale(g["c5"][None], 5)
    assert np.array_equal(r4[0], g["r4"])
    assert np.array_equal(o.rescale(r4, 4)[0], g["r3"])


def test_full_level_calls_match_level_calls():
    g, o = _ckks()
    L = int(g["L"])
    assert np.array_equal(o.mul_relin_at(g["a"][None], g["b"][None], g["rlk"], L),
                          o.mul_relin(g["a"][None], g["b"][None], g["rlk"]))


def test_bfv_hps_mul_relin_golden():
    """HPS multiplication (float parts bit-identical to the big-int model's
    restatement, which checks round(t d / Q) on integers)."""
    g = load("bfv_hps_n1024_l4.npz")
    o = Oracle(SCHEME_BFV, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), t=int(g["t"]),
               moduli=g["moduli"], bfv_mult="hps")
    out = o.mul_relin(g["a"][None], g["b"][None], g["rlk"])
    assert np.array_equal(out[0], g["out_mul"])


def test_ckks_hoisted_rotations_golden():
    g = load("ckks_hoisted_n1024_l5.npz")
    o = Oracle(SCHEME_CKKS, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), moduli=g["moduli"])
    out = o.rotate_hoisted(g["ct"][None], g["galois"], g["gks"])
    assert np.array_equal(out[:, 0], g["out"])
    assert np.array_equal(o.rotate_hoisted_at(g["ct"][None], g["galois"], g["gks"], o.L)[:, 0], g["out"])


def test_bfv_hoisted_rotations_golden():
    g = load("bfv_hoisted_n1024_l4.npz")
    o = Oracle(SCHEME_BFV, int(g["log_n"]), int(g["L"]), int(g["K"]), int(g["dnum"]), t=int(g["t"]),
               moduli=g["moduli"])
    out = o.rotate_hoisted(g["ct"][None], g["galois"], g["gks"])
    assert np.array_equal(out[:, 0], g["out"])


@pytest.mark.parametrize("scheme", ["ckks", "bfv"])
def test_rotation_sum_golden(scheme):
    g = load("rotation_sum_n1024.npz")
    mods = g[f"{scheme}_moduli"]
    if scheme == "ckks":
        o = Oracle(SCHEME_CKKS, int(g["log_n"]), 5, 2, 2, moduli=mods)
    else:
        o = Oracle(SCHEME_BFV, int(g["log_n"]), 4, 2, 2, t=65537, moduli=mods)
    out = o.rotate_sum_hoisted(g[f"{scheme}_ct"][None], g[f"{scheme}_galois"], g[f"{scheme}_gks"])
    assert np.array_equal(out[0], g[f"{scheme}_out"])
    if scheme == "ckks":  # the hoisted linear transform on the same inputs, plaintext-weighted
        lin = o.linear_hoisted(g["ckks_ct"][None], g["ckks_galois"], g["ckks_gks"], g["ckks_pts"])
        assert np.array_equal(lin[0], g["ckks_lin"])
