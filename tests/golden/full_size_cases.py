"""Full-size parity cases pinned by SHA-256 digests.

Every case draws its inputs and keys from the SplitMix64 uniform stream
(oracle orc_fill_uniform == backend fhe_fill_uniform) with fixed seeds, so a
case is fully described by (params, seeds) and its expected output by one
digest.  make_digests.py computes the digests with the CPU oracle and writes
digests.json; test_digests.py re-derives them on the CPU (oracle pinned) and
on the GPU (HIP path, inputs generated on the device).
"""
from __future__ import annotations

import hashlib

import numpy as np

CKKS, BFV = 0, 1

# name -> (scheme, log_n, L, K, dnum, t, op, n_ct, extra)
# extra: the rotation steps (rotate), or "hps" for BFV mul_relin by HPS (else BEHZ)
CASES = {
    "C1_bfv_add_n4096_l1": (BFV, 12, 1, 1, 1, 65537, "add", 4, None),
    "C2_ntt_fwd_n16384_l4": (CKKS, 14, 4, 0, 1, 0, "ntt_fwd", 2, None),
    "C2_ntt_inv_n16384_l4": (CKKS, 14, 4, 0, 1, 0, "ntt_inv", 2, None),
    "C3_bfv_mul_relin_n32768_l8": (BFV, 15, 8, 4, 2, 65537, "mul_relin", 1, None),
    "C3_bfv_hps_mul_relin_n32768_l8": (BFV, 15, 8, 4, 2, 65537, "mul_relin", 1, "hps"),
    "C4_ckks_rotate_n65536_l12": (CKKS, 16, 12, 4, 3, 0, "rotate", 1, 1),
    "metric_ckks_mul_relin_n65536_l12": (CKKS, 16, 12, 4, 3, 0, "mul_relin", 1, None),
    "ckks_keyswitch_n65536_l12": (CKKS, 16, 12, 4, 3, 0, "keyswitch", 1, None),
}
SEED_A, SEED_B, SEED_KEY = 0x48455244, 0x48455245, 0x4B4559


def digest(arr: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(arr, dtype=np.uint64).tobytes()).hexdigest()


def shapes(case):
    scheme, log_n, L, K, dnum, t, op, n_ct, extra = case
    n = 1 << log_n
    if op in ("ntt_fwd", "ntt_inv"):
        return {"a": (n_ct, L, n)}
    if op == "keyswitch":
        return {"a": (n_ct, L, n)}
    return {"a": (n_ct, 2, L, n), "b": (n_ct, 2, L, n)}
