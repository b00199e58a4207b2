"""ctypes binding of libherdsman_fhe.so (include/plugins/fhe_backend.h).

Device buffers are torch tensors on a HIP device (PyTorch is only the
allocator/stream provider here); their data pointers go straight to the C ABI.
There is NO CPU fallback: if the library is missing or no GPU is present every
call raises FheBackendError.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SCHEME_CKKS = 0
SCHEME_BFV = 1

FHE_OK = 0
FHE_ERR_INVALID, FHE_ERR_DEVICE, FHE_ERR_OOM, FHE_ERR_UNSUPPORTED = -1, -2, -3, -4
FHE_FLAG_BFV_HPS = 1
_ERRORS = {FHE_ERR_INVALID: "FHE_ERR_INVALID", FHE_ERR_DEVICE: "FHE_ERR_DEVICE", FHE_ERR_OOM: "FHE_ERR_OOM",
           FHE_ERR_UNSUPPORTED: "FHE_ERR_UNSUPPORTED"}


class FheBackendError(RuntimeError):
    pass


class _Params(C.Structure):
    _fields_ = [
        ("scheme", C.c_uint32),
        ("log_n", C.c_uint32),
        ("num_q", C.c_uint32),
        ("num_p", C.c_uint32),
        ("dnum", C.c_uint32),
        ("q_bits", C.c_uint32),
        ("p_bits", C.c_uint32),
        ("flags", C.c_uint32),
        ("plain_modulus", C.c_uint64),
        ("moduli", C.c_void_p),
    ]


# name -> (restype, argtypes); also the list of exported symbols the CPU
# tests check against include/plugins/fhe_backend.h
_vp, _u32, _u64, _i32, _sz = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32, C.c_size_t
SIGNATURES = {
    "fhe_ctx_create": (C.c_int, [C.POINTER(_Params), C.c_int, C.POINTER(_vp)]),
    "fhe_ctx_destroy": (None, [_vp]),
    "fhe_last_error": (C.c_char_p, [_vp]),
    "fhe_build_id": (C.c_char_p, []),
    "fhe_ctx_moduli": (C.c_int, [_vp, _vp, _u32, C.POINTER(_u32)]),
    "fhe_set_stream": (C.c_int, [_vp, _vp]),
    "fhe_synchronize": (C.c_int, [_vp]),
    "fhe_reserve": (C.c_int, [_vp, _u32]),
    "fhe_dev_alloc": (C.c_int, [_vp, _sz, C.POINTER(_vp)]),
    "fhe_dev_free": (C.c_int, [_vp, _vp]),
    "fhe_memcpy_h2d": (C.c_int, [_vp, _vp, _vp, _sz]),
    "fhe_memcpy_d2h": (C.c_int, [_vp, _vp, _vp, _sz]),
    "fhe_host_alloc": (C.c_int, [_vp, _sz, C.POINTER(_vp)]),
    "fhe_host_free": (C.c_int, [_vp, _vp]),
    "fhe_memcpy_h2d_async": (C.c_int, [_vp, _vp, _vp, _sz]),
    "fhe_memcpy_d2h_async": (C.c_int, [_vp, _vp, _vp, _sz]),
    "fhe_memcpy_d2d_async": (C.c_int, [_vp, _vp, _vp, _sz]),
    "fhe_use_own_stream": (C.c_int, [_vp]),
    "fhe_mark": (C.c_int, [_vp, C.c_uint32]),
    "fhe_wait_mark": (C.c_int, [_vp, C.c_uint32]),
    "fhe_ntt_fwd": (C.c_int, [_vp, _vp, _u32, _u32, _u32]),
    "fhe_ntt_inv": (C.c_int, [_vp, _vp, _u32, _u32, _u32]),
    "fhe_poly_add": (C.c_int, [_vp, _vp, _vp, _vp, _u32, _u32, _u32]),
    "fhe_poly_sub": (C.c_int, [_vp, _vp, _vp, _vp, _u32, _u32, _u32]),
    "fhe_poly_mul": (C.c_int, [_vp, _vp, _vp, _vp, _u32, _u32, _u32]),
    "fhe_base_conv": (C.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _u32, _u32]),
    "fhe_fill_uniform": (C.c_int, [_vp, _vp, _u32, _u32, _u32, _u64]),
    "fhe_add": (C.c_int, [_vp, _vp, _vp, _vp, _u32]),
    "fhe_sub": (C.c_int, [_vp, _vp, _vp, _vp, _u32]),
    "fhe_mul_relin": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _u32]),
    "fhe_keyswitch": (C.c_int, [_vp, _vp, _vp, _vp, _u32]),
    "fhe_rotate": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _u32]),
    "fhe_galois_elt": (C.c_int, [_vp, _i32, C.POINTER(_u32)]),
    "fhe_rotate_hoisted": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _u32]),
    "fhe_rotate_hoisted_at": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _u32, _u32]),
    "fhe_rotate_sum_hoisted": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _u32]),
    "fhe_rotate_sum_hoisted_at": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _u32, _u32]),
    "fhe_linear_hoisted": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32]),
    "fhe_linear_hoisted_at": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32, _u32]),
    "fhe_add_at": (C.c_int, [_vp, _vp, _vp, _vp, _u32, _u32]),
    "fhe_sub_at": (C.c_int, [_vp, _vp, _vp, _vp, _u32, _u32]),
    "fhe_mul_relin_at": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _u32, _u32]),
    "fhe_rotate_at": (C.c_int, [_vp, _vp, _u32, _vp, _vp, _u32, _u32]),
    "fhe_keyswitch_at": (C.c_int, [_vp, _vp, _vp, _vp, _u32, _u32]),
    "fhe_rescale": (C.c_int, [_vp, _vp, _vp, _u32, _u32]),
    "fhe_level_reduce": (C.c_int, [_vp, _vp, _vp, _u32, _u32, _u32]),
    "fhe_reduce_at": (C.c_int, [_vp, _vp, _u32, C.c_int, _vp, _vp, _u32]),
    "fhe_reduce": (C.c_int, [_vp, _vp, _u32, C.c_int, _vp, _vp]),
    "fhe_bcast_key": (C.c_int, [_vp, _vp, _sz, _vp, C.c_int]),
    "fhe_reduce_ranks": (C.c_int, [_vp, _vp, C.c_int, _vp, _vp, C.c_int, _vp]),
    "fhe_reduce_ranks_at": (C.c_int, [_vp, _vp, C.c_int, _vp, _vp, C.c_int, _vp, _u32]),
    "fhe_reduce_schedule": (C.c_int, [C.c_int, C.c_int, C.c_int, _vp, C.c_int]),
}

REDUCE_ADD = 0
REDUCE_MUL_RELIN = 1

_lib = None


def library_path() -> str:
    # HERD_FHE_LIB selects another in-tree build of the same library (A/B
    # experiments on the GPU box); it is still the HIP backend, never a fallback
    return os.environ.get("HERD_FHE_LIB") or os.path.join(HERE, "lib", "libherdsman_fhe.so")


def source_build_id(root: str = HERE) -> Optional[str]:
    """SHA-256 of the library's sources as the Makefile bakes it into
    fhe_build_id(): every file of csrc/ and include/plugins/fhe_backend.h, in
    sorted relative-path order, contents concatenated.  None if the sources are
    not there (an installed copy without them)."""
    csrc = os.path.join(root, "csrc")
    hdr = os.path.join(root, "..", "include", "plugins", "fhe_backend.h")
    if not os.path.isdir(csrc) or not os.path.exists(hdr):
        return None
    rel = ["csrc/" + f for f in os.listdir(csrc) if os.path.isfile(os.path.join(csrc, f))]
    rel.append("../include/plugins/fhe_backend.h")
    h = hashlib.sha256()
    for r in sorted(rel):
        with open(os.path.join(root, r), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def check_build_id(lib, root: str = HERE) -> str:
    """Refuse a library whose baked-in build id does not match the sources
    under `root` (a stale .so next to newer sources).  Returns the id."""
    if not hasattr(lib, "fhe_build_id"):
        raise FheBackendError("library exports no fhe_build_id(): rebuild it (make -C herdsman_amd)")
    lib.fhe_build_id.restype, lib.fhe_build_id.argtypes = C.c_char_p, []
    built = lib.fhe_build_id().decode()
    want = source_build_id(root)
    if want is not None and built != want:
        raise FheBackendError(f"libherdsman_fhe.so was built from other sources (build id {built[:16]}, "
                              f"sources {want[:16]}): rebuild it (make -C herdsman_amd)")
    return built


def load_library():
    """Load the HIP backend; raises (never falls back) when it is missing or
    was built from sources other than the ones checked out."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise FheBackendError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    variant = bool(os.environ.get("HERD_FHE_LIB"))
    if not variant:  # an A/B variant is built from modified sources on purpose
        check_build_id(lib)
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue  # an older build under A/B may predate an entry point it is not asked for
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    _lib = lib
    return lib


def _ptr(t) -> int:
    """Device pointer of a torch tensor (must be contiguous, on a HIP device)."""
    if not t.is_cuda:
        raise FheBackendError("buffer must live on the GPU (torch tensor on a HIP device)")
    if not t.is_contiguous():
        raise FheBackendError("buffer must be contiguous")
    if t.element_size() != 8:
        raise FheBackendError("buffer must hold 64-bit words")
    return t.data_ptr()


class Context:
    """One device context (params + twiddle/CRT tables + workspace)."""

    def __init__(self, scheme: int, log_n: int, L: int, K: int = 0, dnum: int = 1, q_bits: int = 60,
                 p_bits: int = 61, t: int = 0, moduli: Optional[Sequence[int]] = None, device: int = 0,
                 bfv_mult: str = "behz"):
        self.lib = load_library()
        self.scheme, self.log_n, self.n = scheme, log_n, 1 << log_n
        self.L, self.K, self.dnum, self.t = L, K, dnum, t
        self.alpha = -(-L // dnum)
        self._mods_keep = None
        mp = None
        if moduli is not None:
            self._mods_keep = np.ascontiguousarray(np.asarray(moduli, dtype=np.uint64))
            mp = self._mods_keep.ctypes.data
        if bfv_mult not in ("behz", "hps"):
            raise FheBackendError(f"unknown BFV multiplication technique {bfv_mult!r} (behz or hps)")
        self.bfv_mult = bfv_mult
        flags = FHE_FLAG_BFV_HPS if bfv_mult == "hps" else 0
        p = _Params(scheme, log_n, L, K, dnum, q_bits, p_bits, flags, t, mp)
        h = C.c_void_p()
        rc = self.lib.fhe_ctx_create(C.byref(p), device, C.byref(h))
        if rc != FHE_OK:
            msg = self.lib.fhe_last_error(None)
            raise FheBackendError(f"fhe_ctx_create: {_ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")
        self.h = h
        cnt = _u32()
        self.lib.fhe_ctx_moduli(self.h, None, 0, C.byref(cnt))
        self.moduli = np.zeros(cnt.value, dtype=np.uint64)
        self.lib.fhe_ctx_moduli(self.h, self.moduli.ctypes.data, cnt.value, None)
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self.lib.fhe_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc, what):
        if rc != FHE_OK:
            msg = self.lib.fhe_last_error(self.h)
            raise FheBackendError(f"{what}: {_ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")

    # ---- streams
    def set_stream(self, stream):
        """Enqueue on a torch.cuda.Stream (or raw hipStream_t int)."""
        raw = stream if isinstance(stream, int) else stream.cuda_stream
        self._ck(self.lib.fhe_set_stream(self.h, raw), "fhe_set_stream")

    def synchronize(self):
        self._ck(self.lib.fhe_synchronize(self.h), "fhe_synchronize")

    def reserve(self, max_batch: int):
        self._ck(self.lib.fhe_reserve(self.h, max_batch), "fhe_reserve")

    # ---- shapes
    def ct_shape(self, n_ct: int = 1):
        return (n_ct, 2, self.L, self.n)

    def key_shape(self):
        return (self.dnum, 2, self.L + self.K, self.n)

    # ---- argument checks (the C ABI trusts its sizes: a short buffer would be
    # read or written out of bounds on the GPU, so shapes and devices are
    # checked here, before any pointer crosses the ABI)
    def _on_device(self, *ts):
        for t in ts:
            if t.device.type != "cuda" or t.device.index != self.device:
                raise FheBackendError(f"buffer on {t.device}, context on cuda:{self.device}")

    def _ct_batch(self, *cts):
        n = cts[0].shape[0] if cts[0].dim() == 4 else -1
        for t in cts:
            if tuple(t.shape) != self.ct_shape(n):
                raise FheBackendError(f"ciphertext batch shape {tuple(t.shape)}, expected {self.ct_shape(max(n, 0))}")
        self._on_device(*cts)
        return n

    def _key(self, k):
        if tuple(k.shape) != self.key_shape():
            raise FheBackendError(f"key shape {tuple(k.shape)}, expected {self.key_shape()}")
        self._on_device(k)

    # ---- primitives
    def _limbs(self, x, mod_begin: int = 0):
        if x.dim() < 2 or x.shape[-1] != self.n:
            raise FheBackendError(f"last dim must be N={self.n}")
        nl = x.shape[-2]
        if mod_begin < 0 or nl < 1 or mod_begin + nl > len(self.moduli):
            raise FheBackendError(f"limbs [{mod_begin}, {mod_begin + nl}) outside the {len(self.moduli)} moduli")
        self._on_device(x)
        return x.numel() // (nl * self.n), nl

    def ntt_fwd(self, x, mod_begin: int = 0):
        n, nl = self._limbs(x, mod_begin)
        self._ck(self.lib.fhe_ntt_fwd(self.h, _ptr(x), n, mod_begin, nl), "fhe_ntt_fwd")
        return x

    def ntt_inv(self, x, mod_begin: int = 0):
        n, nl = self._limbs(x, mod_begin)
        self._ck(self.lib.fhe_ntt_inv(self.h, _ptr(x), n, mod_begin, nl), "fhe_ntt_inv")
        return x

    def poly_op(self, op: str, a, b, out, mod_begin: int = 0):
        n, nl = self._limbs(a, mod_begin)
        if b.shape != a.shape or out.shape != a.shape:
            raise FheBackendError("poly_op operands must have one shape")
        self._on_device(b, out)
        fn = {"add": self.lib.fhe_poly_add, "sub": self.lib.fhe_poly_sub, "mul": self.lib.fhe_poly_mul}[op]
        self._ck(fn(self.h, _ptr(a), _ptr(b), _ptr(out), n, mod_begin, nl), f"fhe_poly_{op}")
        return out

    def base_conv(self, src, src_mods, dst, dst_mods):
        s = np.ascontiguousarray(src_mods, dtype=np.uint32)
        d = np.ascontiguousarray(dst_mods, dtype=np.uint32)
        n = src.numel() // (len(s) * self.n)
        if src.numel() != n * len(s) * self.n or dst.numel() != n * len(d) * self.n:
            raise FheBackendError("base_conv: src / dst sizes do not match the modulus lists")
        self._on_device(src, dst)
        self._ck(self.lib.fhe_base_conv(self.h, _ptr(src), s.ctypes.data, len(s), _ptr(dst), d.ctypes.data,
                                        len(d), n), "fhe_base_conv")
        return dst

    def fill_uniform(self, x, seed: int, mod_begin: int = 0):
        n, nl = self._limbs(x, mod_begin)
        self._ck(self.lib.fhe_fill_uniform(self.h, _ptr(x), n, mod_begin, nl, seed & (2**64 - 1)),
                 "fhe_fill_uniform")
        return x

    # ---- ciphertext ops
    def add(self, a, b, out):
        n = self._ct_batch(a, b, out)
        self._ck(self.lib.fhe_add(self.h, _ptr(a), _ptr(b), _ptr(out), n), "fhe_add")
        return out

    def sub(self, a, b, out):
        n = self._ct_batch(a, b, out)
        self._ck(self.lib.fhe_sub(self.h, _ptr(a), _ptr(b), _ptr(out), n), "fhe_sub")
        return out

    def mul_relin(self, a, b, rlk, out):
        n = self._ct_batch(a, b, out)
        self._key(rlk)
        self._ck(self.lib.fhe_mul_relin(self.h, _ptr(a), _ptr(b), _ptr(rlk), _ptr(out), n), "fhe_mul_relin")
        return out

    def keyswitch(self, d, ksk, out):
        n = self._ct_batch(out)
        if tuple(d.shape) != (n, self.L, self.n):
            raise FheBackendError(f"keyswitch input shape {tuple(d.shape)}, expected {(n, self.L, self.n)}")
        self._on_device(d)
        self._key(ksk)
        self._ck(self.lib.fhe_keyswitch(self.h, _ptr(d), _ptr(ksk), _ptr(out), n), "fhe_keyswitch")
        return out

    def rotate(self, ct, galois: int, gk, out):
        n = self._ct_batch(ct, out)
        self._key(gk)
        self._ck(self.lib.fhe_rotate(self.h, _ptr(ct), galois, _ptr(gk), _ptr(out), n), "fhe_rotate")
        return out

    def _hoisted(self, fn, ct, galois, gks, outs, n, *extra):
        if not (len(galois) == len(gks) == len(outs)):
            raise FheBackendError("hoisted rotations: galois, gks and outs must have one length")
        for k in gks:
            self._key(k)
        nr = len(galois)
        ga = np.ascontiguousarray(galois, dtype=np.uint32)
        ka = (C.c_uint64 * max(nr, 1))(*[_ptr(k) for k in gks])
        oa = (C.c_uint64 * max(nr, 1))(*[_ptr(o) for o in outs])
        self._ck(fn(self.h, _ptr(ct), nr, ga.ctypes.data, C.addressof(ka), C.addressof(oa), n, *extra),
                 fn.__name__)
        return outs

    def rotate_hoisted(self, ct, galois, gks, outs):
        """CKKS: outs[r] = rotation of ct by galois[r] with key gks[r], one ModUp of c1 for all."""
        n = self._ct_batch(ct, *outs)
        return self._hoisted(self.lib.fhe_rotate_hoisted, ct, galois, gks, outs, n)

    def _rot_sum(self, fn, ct, galois, gks, out, n, *extra):
        if len(galois) != len(gks) or not galois:
            raise FheBackendError("rotation sum: galois and gks must have one (non-zero) length")
        for k in gks:
            self._key(k)
        ga = np.ascontiguousarray(galois, dtype=np.uint32)
        ka = (C.c_uint64 * len(gks))(*[_ptr(k) for k in gks])
        self._ck(fn(self.h, _ptr(ct), len(ga), ga.ctypes.data, C.addressof(ka), _ptr(out), n, *extra), fn.__name__)
        return out

    def _linear(self, fn, ct, galois, gks, pts, out, n, *extra):
        if not (len(galois) == len(gks) == len(pts)) or not galois:
            raise FheBackendError("linear transform: galois, gks and pts must have one (non-zero) length")
        for k in gks:
            self._key(k)
        for p in pts:
            if tuple(p.shape) != (self.L + self.K, self.n):
                raise FheBackendError(f"plaintext shape {tuple(p.shape)}, expected {(self.L + self.K, self.n)}")
            self._on_device(p)
        ga = np.ascontiguousarray(galois, dtype=np.uint32)
        ka = (C.c_uint64 * len(gks))(*[_ptr(k) for k in gks])
        pa = (C.c_uint64 * len(pts))(*[_ptr(p) for p in pts])
        self._ck(fn(self.h, _ptr(ct), len(ga), ga.ctypes.data, C.addressof(ka), C.addressof(pa), _ptr(out), n,
                    *extra), fn.__name__)
        return out

    def linear_hoisted(self, ct, galois, gks, pts, out):
        """CKKS: out = sum_r pts[r] (.) rot_{galois[r]}(ct), one ModDown (pts [L+K][N] NTT form)."""
        n = self._ct_batch(ct, out)
        return self._linear(self.lib.fhe_linear_hoisted, ct, galois, gks, pts, out, n)

    def linear_hoisted_at(self, ct, galois, gks, pts, out, level: int):
        n = self._ct_level(level, ct, out)
        return self._linear(self.lib.fhe_linear_hoisted_at, ct, galois, gks, pts, out, n, level)

    def rotate_sum_hoisted(self, ct, galois, gks, out):
        """out = sum_r rot_{galois[r]}(ct), one ModDown for all the elements (double hoisting)."""
        n = self._ct_batch(ct, out)
        return self._rot_sum(self.lib.fhe_rotate_sum_hoisted, ct, galois, gks, out, n)

    def rotate_sum_hoisted_at(self, ct, galois, gks, out, level: int):
        n = self._ct_level(level, ct, out)
        return self._rot_sum(self.lib.fhe_rotate_sum_hoisted_at, ct, galois, gks, out, n, level)

    # ---- CKKS levels: ciphertexts [n][2][level][N] over the first `level` Q primes
    def _ct_level(self, level: int, *cts):
        if not 1 <= level <= self.L:
            raise FheBackendError(f"level {level} outside [1, {self.L}]")
        n = cts[0].shape[0] if cts[0].dim() == 4 else -1
        want = (n, 2, level, self.n)
        for t in cts:
            if tuple(t.shape) != want:
                raise FheBackendError(f"level-{level} ciphertext batch shape {tuple(t.shape)}, expected {want}")
        self._on_device(*cts)
        return n

    def add_at(self, a, b, out, level: int):
        n = self._ct_level(level, a, b, out)
        self._ck(self.lib.fhe_add_at(self.h, _ptr(a), _ptr(b), _ptr(out), n, level), "fhe_add_at")
        return out

    def sub_at(self, a, b, out, level: int):
        n = self._ct_level(level, a, b, out)
        self._ck(self.lib.fhe_sub_at(self.h, _ptr(a), _ptr(b), _ptr(out), n, level), "fhe_sub_at")
        return out

    def mul_relin_at(self, a, b, rlk, out, level: int):
        n = self._ct_level(level, a, b, out)
        self._key(rlk)
        self._ck(self.lib.fhe_mul_relin_at(self.h, _ptr(a), _ptr(b), _ptr(rlk), _ptr(out), n, level),
                 "fhe_mul_relin_at")
        return out

    def rotate_at(self, ct, galois: int, gk, out, level: int):
        n = self._ct_level(level, ct, out)
        self._key(gk)
        self._ck(self.lib.fhe_rotate_at(self.h, _ptr(ct), galois, _ptr(gk), _ptr(out), n, level), "fhe_rotate_at")
        return out

    def rotate_hoisted_at(self, ct, galois, gks, outs, level: int):
        n = self._ct_level(level, ct, *outs)
        return self._hoisted(self.lib.fhe_rotate_hoisted_at, ct, galois, gks, outs, n, level)

    def keyswitch_at(self, d, ksk, out, level: int):
        n = self._ct_level(level, out)
        if tuple(d.shape) != (n, level, self.n):
            raise FheBackendError(f"keyswitch input shape {tuple(d.shape)}, expected {(n, level, self.n)}")
        self._on_device(d)
        self._key(ksk)
        self._ck(self.lib.fhe_keyswitch_at(self.h, _ptr(d), _ptr(ksk), _ptr(out), n, level), "fhe_keyswitch_at")
        return out

    def rescale(self, ct, out, level: int):
        """level -> level - 1: out [n][2][level-1][N] = round(ct / q_{level-1})."""
        n = self._ct_level(level, ct)
        if level < 2:
            raise FheBackendError("rescale needs level >= 2")
        self._ct_level(level - 1, out)
        if out.shape[0] != ct.shape[0]:
            raise FheBackendError("rescale: input and output batch sizes differ")
        self._ck(self.lib.fhe_rescale(self.h, _ptr(ct), _ptr(out), n, level), "fhe_rescale")
        return out

    def level_reduce(self, ct, out, level_in: int, level_out: int):
        """Drop the Q limbs past level_out (no scaling)."""
        n = self._ct_level(level_in, ct)
        self._ct_level(level_out, out)
        self._ck(self.lib.fhe_level_reduce(self.h, _ptr(ct), _ptr(out), n, level_in, level_out), "fhe_level_reduce")
        return out

    def reduce(self, cts, op: int, rlk=None, out=None):
        """Balanced-tree reduction of cts [n][2][L][N] to out [1][2][L][N] (cts is scratch)."""
        out = cts[:1] if out is None else out
        self._ct_batch(cts)
        if out.dim() != 4 or out.shape[0] < 1:
            raise FheBackendError("reduce output must hold one ciphertext")
        self._ct_batch(out)
        if rlk is not None:
            self._key(rlk)
        self._ck(self.lib.fhe_reduce(self.h, _ptr(cts), cts.shape[0], op, _ptr(rlk) if rlk is not None else None,
                                     _ptr(out)), "fhe_reduce")
        return out

    def galois_elt(self, steps: int) -> int:
        g = _u32()
        self._ck(self.lib.fhe_galois_elt(self.h, steps, C.byref(g)), "fhe_galois_elt")
        return g.value

    def bcast_key(self, key, nccl_comm: int, root: int = 0):
        self._on_device(key)
        self._ck(self.lib.fhe_bcast_key(self.h, _ptr(key), key.numel(), nccl_comm, root), "fhe_bcast_key")


# ---- torch <-> numpy helpers (u64 payload in int64 tensors)
def to_device(arr: np.ndarray, device="cuda"):
    import torch

    a = np.ascontiguousarray(arr, dtype=np.uint64)
    return torch.from_numpy(a.view(np.int64)).to(device)


def to_host(t) -> np.ndarray:
    return t.detach().cpu().numpy().view(np.uint64)


def empty(shape, device="cuda"):
    import torch

    return torch.empty(shape, dtype=torch.int64, device=device)


def reduce_schedule(rank: int, world: int, root: int = 0):
    """fhe_reduce_schedule: this rank's steps of the cross-rank tree, as
    ("recv", peer) / ("send", peer) pairs (host only, no device needed)."""
    lib = load_library()
    buf = (C.c_int32 * 32)()
    n = lib.fhe_reduce_schedule(rank, world, root, C.cast(buf, _vp), 32)
    if n < 0:
        raise FheBackendError(f"fhe_reduce_schedule({rank}, {world}, {root}) = {n}")
    return [("recv", v - 1) if v > 0 else ("send", -v - 1) for v in buf[:n]]
