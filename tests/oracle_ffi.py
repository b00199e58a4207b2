"""ctypes binding of the CPU oracle (oracle/build/libfhe_oracle.so).

Test infrastructure: the oracle is the CHECKER, never the product.  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "libfhe_oracle.so")

SCHEME_CKKS = 0
SCHEME_BFV = 1
BFV_MULT = {"behz": 0, "hps": 1}

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_lib = None


class OracleUnsupported(ValueError):
    """The oracle refused an op it does not implement (ORC_ERR_*), as the GPU ABI does."""


def _ck(rc: int) -> None:
    if rc != 0:
        raise OracleUnsupported(f"oracle refused the call: {'ORC_ERR_UNSUPPORTED' if rc == -4 else 'ORC_ERR_INVALID' if rc == -1 else rc}")


def build_oracle() -> str:
    src = os.path.join(ORACLE_DIR, "fhe_oracle.c")
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    L = C.CDLL(build_oracle())
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "orc_ctx_create": (vp, [u32, u32, u32, u32, u32, u32, u32, u64, C.c_void_p]),
        "orc_ctx_destroy": (None, [vp]),
        "orc_num_moduli": (u32, [vp]),
        "orc_moduli": (None, [vp, _u64p]),
        "orc_psi": (u64, [vp, u32]),
        "orc_gen_primes": (u32, [u32, u32, u32, C.c_void_p, u32, _u64p]),
        "orc_set_threads": (None, [C.c_int]),
        "orc_set_bfv_mult": (C.c_int, [vp, u32]),
        "orc_ntt_fwd": (None, [vp, _u64p, u32, u32, u32]),
        "orc_ntt_inv": (None, [vp, _u64p, u32, u32, u32]),
        "orc_add": (None, [vp, _u64p, _u64p, _u64p, u32, u32, u32]),
        "orc_sub": (None, [vp, _u64p, _u64p, _u64p, u32, u32, u32]),
        "orc_mul": (None, [vp, _u64p, _u64p, _u64p, u32, u32, u32]),
        "orc_automorph_ntt": (None, [vp, _u64p, _u64p, u32, u32, u32]),
        "orc_automorph_coef": (None, [vp, _u64p, _u64p, u32, u32, u32, u32]),
        "orc_base_conv": (None, [vp, _u64p, _u32p, u32, _u64p, _u32p, u32, u32]),
        "orc_ct_add": (None, [vp, _u64p, _u64p, _u64p, u32]),
        "orc_keyswitch": (None, [vp, _u64p, _u64p, _u64p, u32]),
        "orc_mul_relin": (None, [vp, _u64p, _u64p, _u64p, _u64p, u32]),
        "orc_rotate": (None, [vp, _u64p, u32, _u64p, _u64p, u32]),
        "orc_galois_elt": (u32, [vp, i32]),
        "orc_keyswitch_at": (C.c_int, [vp, _u64p, _u64p, _u64p, u32, u32]),
        "orc_mul_relin_at": (C.c_int, [vp, _u64p, _u64p, _u64p, _u64p, u32, u32]),
        "orc_rotate_at": (C.c_int, [vp, _u64p, u32, _u64p, _u64p, u32, u32]),
        "orc_rescale": (C.c_int, [vp, _u64p, _u64p, u32, u32]),
        "orc_rotate_hoisted": (None, [vp, _u64p, u32, _u32p, _u64p, _u64p, u32]),
        "orc_rotate_hoisted_at": (C.c_int, [vp, _u64p, u32, _u32p, _u64p, _u64p, u32, u32]),
        "orc_rotate_sum_hoisted_at": (C.c_int, [vp, _u64p, u32, _u32p, _u64p, _u64p, u32, u32]),
        "orc_linear_hoisted_at": (C.c_int, [vp, _u64p, u32, _u32p, _u64p, _u64p, _u64p, u32, u32]),
        "orc_fill_uniform": (None, [vp, _u64p, u32, u32, u32, u64]),
        "orc_sample_ternary": (None, [vp, u64, _i64p]),
        "orc_sample_cbd": (None, [vp, u64, _i64p]),
        "orc_signed_to_rns": (None, [vp, _i64p, _u64p, u32, u32, C.c_int]),
        "orc_gen_switch_key": (None, [vp, _u64p, _u64p, u64, _u64p]),
        "orc_encrypt": (None, [vp, _u64p, _u64p, u64, _u64p]),
        "orc_decrypt": (None, [vp, _u64p, _u64p, _u64p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    _lib = L
    return L


class Oracle:
    """Thin object wrapper mirroring the backend's context."""

    def __init__(self, scheme: int, log_n: int, L: int, K: int = 0, dnum: int = 1,
                 q_bits: int = 60, p_bits: int = 61, t: int = 0, moduli=None, bfv_mult: str = "behz"):
        self.lib = lib()
        self.scheme, self.log_n, self.n = scheme, log_n, 1 << log_n
        self.L, self.K, self.dnum, self.t = L, K, dnum, t
        self.alpha = -(-L // dnum)
        mp = None
        if moduli is not None:
            self._mod_keep = np.ascontiguousarray(moduli, dtype=np.uint64)
            mp = self._mod_keep.ctypes.data
        self.h = self.lib.orc_ctx_create(scheme, log_n, L, K, dnum, q_bits, p_bits, t, mp)
        if not self.h:
            raise ValueError("orc_ctx_create failed")
        if bfv_mult not in ("behz", "hps") or self.lib.orc_set_bfv_mult(self.h, BFV_MULT[bfv_mult]) != 0:
            raise ValueError(f"unknown BFV multiplication technique {bfv_mult!r}")
        nm = self.lib.orc_num_moduli(self.h)
        self.moduli = np.zeros(nm, dtype=np.uint64)
        self.lib.orc_moduli(self.h, self.moduli)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_ctx_destroy(self.h)
            self.h = None

    # shapes
    def ct_shape(self, n_ct=1):
        return (n_ct, 2, self.L, self.n)

    def key_shape(self):
        return (self.dnum, 2, self.L + self.K, self.n)

    def ntt_fwd(self, x, mod_begin=0):
        x = np.ascontiguousarray(x, dtype=np.uint64).copy()
        nl = x.shape[-2]
        self.lib.orc_ntt_fwd(self.h, x, x.size // (nl * self.n), mod_begin, nl)
        return x

    def ntt_inv(self, x, mod_begin=0):
        x = np.ascontiguousarray(x, dtype=np.uint64).copy()
        nl = x.shape[-2]
        self.lib.orc_ntt_inv(self.h, x, x.size // (nl * self.n), mod_begin, nl)
        return x

    def uniform(self, shape, seed, mod_begin=0):
        x = np.zeros(shape, dtype=np.uint64)
        nl = shape[-2]
        self.lib.orc_fill_uniform(self.h, x, x.size // (nl * self.n), mod_begin, nl, seed)
        return x

    def mul_relin(self, a, b, rlk):
        out = np.zeros_like(a)
        self.lib.orc_mul_relin(self.h, np.ascontiguousarray(a), np.ascontiguousarray(b),
                               np.ascontiguousarray(rlk), out, a.shape[0])
        return out

    def rotate(self, ct, g, gk):
        out = np.zeros_like(ct)
        self.lib.orc_rotate(self.h, np.ascontiguousarray(ct), g, np.ascontiguousarray(gk), out, ct.shape[0])
        return out

    def keyswitch(self, d, ksk):
        out = np.zeros((d.shape[0], 2, self.L, self.n), dtype=np.uint64)
        self.lib.orc_keyswitch(self.h, np.ascontiguousarray(d), np.ascontiguousarray(ksk), out, d.shape[0])
        return out

    # ---- CKKS levels: ciphertexts [n][2][lvl][N] over the first lvl Q primes
    def mul_relin_at(self, a, b, rlk, lvl):
        out = np.zeros_like(a)
        _ck(self.lib.orc_mul_relin_at(self.h, np.ascontiguousarray(a), np.ascontiguousarray(b),
                                  np.ascontiguousarray(rlk), out, a.shape[0], lvl))
        return out

    def rotate_at(self, ct, g, gk, lvl):
        out = np.zeros_like(ct)
        _ck(self.lib.orc_rotate_at(self.h, np.ascontiguousarray(ct), g, np.ascontiguousarray(gk), out, ct.shape[0], lvl))
        return out

    def keyswitch_at(self, d, ksk, lvl):
        out = np.zeros((d.shape[0], 2, lvl, self.n), dtype=np.uint64)
        _ck(self.lib.orc_keyswitch_at(self.h, np.ascontiguousarray(d), np.ascontiguousarray(ksk), out, d.shape[0], lvl))
        return out

    def rotate_hoisted(self, ct, galois, gks):
        """ct [n][2][L][N], galois [r], gks [r][key] -> [r][n][2][L][N]"""
        ct = np.ascontiguousarray(ct)
        gs = np.ascontiguousarray(galois, dtype=np.uint32)
        out = np.zeros((len(gs),) + ct.shape, dtype=np.uint64)
        self.lib.orc_rotate_hoisted(self.h, ct, len(gs), gs, np.ascontiguousarray(gks), out, ct.shape[0])
        return out

    def rotate_sum_hoisted(self, ct, galois, gks, lvl=None):
        """double-hoisted sum of rotations: ct [n][2][lvl][N] -> [n][2][lvl][N]"""
        ct = np.ascontiguousarray(ct)
        gs = np.ascontiguousarray(galois, dtype=np.uint32)
        out = np.zeros(ct.shape, dtype=np.uint64)
        _ck(self.lib.orc_rotate_sum_hoisted_at(self.h, ct, len(gs), gs, np.ascontiguousarray(gks), out, ct.shape[0],
                                           ct.shape[2] if lvl is None else lvl))
        return out

    def linear_hoisted(self, ct, galois, gks, pts, lvl=None):
        """hoisted linear transform: sum_r pts[r] (.) rot_r(ct); pts [r][L+K][N] NTT form"""
        ct = np.ascontiguousarray(ct)
        gs = np.ascontiguousarray(galois, dtype=np.uint32)
        out = np.zeros(ct.shape, dtype=np.uint64)
        _ck(self.lib.orc_linear_hoisted_at(self.h, ct, len(gs), gs, np.ascontiguousarray(gks), np.ascontiguousarray(pts),
                                       out, ct.shape[0], ct.shape[2] if lvl is None else lvl))
        return out

    def rotate_hoisted_at(self, ct, galois, gks, lvl):
        """ct [n][2][lvl][N] at level lvl, full-level keys -> [r][n][2][lvl][N]"""
        ct = np.ascontiguousarray(ct)
        gs = np.ascontiguousarray(galois, dtype=np.uint32)
        out = np.zeros((len(gs),) + ct.shape, dtype=np.uint64)
        _ck(self.lib.orc_rotate_hoisted_at(self.h, ct, len(gs), gs, np.ascontiguousarray(gks), out, ct.shape[0], lvl))
        return out

    def rescale(self, ct, lvl):
        out = np.zeros((ct.shape[0], 2, lvl - 1, self.n), dtype=np.uint64)
        _ck(self.lib.orc_rescale(self.h, np.ascontiguousarray(ct), out, ct.shape[0], lvl))
        return out

    def ct_add(self, a, b):
        out = np.zeros_like(a)
        self.lib.orc_ct_add(self.h, np.ascontiguousarray(a), np.ascontiguousarray(b), out, a.shape[0])
        return out

    def galois_elt(self, steps):
        return self.lib.orc_galois_elt(self.h, steps)

    def automorph_ntt(self, x, g):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        out = np.zeros_like(x)
        nl = x.shape[-2]
        self.lib.orc_automorph_ntt(self.h, x, out, g, x.size // (nl * self.n), nl)
        return out

    def base_conv(self, x, src_mods, dst_mods):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        s = np.ascontiguousarray(src_mods, dtype=np.uint32)
        d = np.ascontiguousarray(dst_mods, dtype=np.uint32)
        n = x.size // (len(s) * self.n)
        out = np.zeros((n, len(d), self.n), dtype=np.uint64)
        self.lib.orc_base_conv(self.h, x, s, len(s), out, d, len(d), n)
        return out

    # ---- keys / encryption (tests)
    def secret(self, seed):
        s = np.zeros(self.n, dtype=np.int64)
        self.lib.orc_sample_ternary(self.h, seed, s)
        return s

    def signed_to_rns(self, coef, mod_begin, n_limbs, ntt=True):
        out = np.zeros((n_limbs, self.n), dtype=np.uint64)
        self.lib.orc_signed_to_rns(self.h, np.ascontiguousarray(coef, dtype=np.int64), out,
                                   mod_begin, n_limbs, 1 if ntt else 0)
        return out

    def switch_key(self, s_from_ntt, s_to_ntt, seed):
        k = np.zeros(self.key_shape(), dtype=np.uint64)
        self.lib.orc_gen_switch_key(self.h, np.ascontiguousarray(s_from_ntt), np.ascontiguousarray(s_to_ntt),
                                    seed, k)
        return k

    def encrypt(self, m_coef, s_ntt, seed):
        ct = np.zeros((2, self.L, self.n), dtype=np.uint64)
        self.lib.orc_encrypt(self.h, np.ascontiguousarray(m_coef, dtype=np.uint64),
                             np.ascontiguousarray(s_ntt), seed, ct)
        return ct

    def decrypt(self, ct, s_ntt):
        m = np.zeros((self.L, self.n), dtype=np.uint64)
        self.lib.orc_decrypt(self.h, np.ascontiguousarray(ct), np.ascontiguousarray(s_ntt), m)
        return m
