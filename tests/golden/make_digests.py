"""Compute tests/golden/digests.json with the CPU oracle.

    python tests/golden/make_digests.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from full_size_cases import CASES, SEED_A, SEED_B, SEED_KEY, digest, shapes  # noqa: E402
from oracle_ffi import Oracle  # noqa: E402


def oracle_output(name):
    scheme, log_n, L, K, dnum, t, op, n_ct, extra = CASES[name]
    o = Oracle(scheme, log_n, L, K, dnum, t=t, bfv_mult="hps" if extra == "hps" else "behz")
    sh = shapes(CASES[name])
    a = o.uniform(sh["a"], seed=SEED_A)
    if op == "ntt_fwd":
        return o, o.ntt_fwd(a)
    if op == "ntt_inv":
        return o, o.ntt_inv(a)
    b = o.uniform(sh["b"], seed=SEED_B) if "b" in sh else None
    if op == "add":
        return o, o.ct_add(a, b)
    key = o.uniform(o.key_shape(), seed=SEED_KEY)
    if op == "mul_relin":
        return o, o.mul_relin(a, b, key)
    if op == "rotate":
        return o, o.rotate(a, o.galois_elt(extra), key)
    if op == "keyswitch":
        return o, o.keyswitch(a, key)
    raise ValueError(op)


def main(only=None):
    path = os.path.join(HERE, "digests.json")
    out = json.load(open(path)) if only else {}
    for name in CASES:
        if only and name not in only:
            continue
        o, y = oracle_output(name)
        out[name] = {"sha256": digest(y), "moduli": [int(q) for q in o.moduli], "shape": list(y.shape)}
        print(name, out[name]["sha256"], flush=True)
    with open(path, "w") as f:
        json.dump({k: out[k] for k in CASES}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or None)  # names: recompute only those cases
