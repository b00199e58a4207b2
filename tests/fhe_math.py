"""Exact-integer helpers for scheme-level checks (decrypt -> CRT -> compare)."""
from __future__ import annotations

import math

import numpy as np


def crt_centered(m_rns, mods):
    """[L][N] residues -> list of centered Python ints in (-Q/2, Q/2]."""
    mods = [int(q) for q in mods]
    Q = math.prod(mods)
    hats = [Q // q for q in mods]
    coef = [h * pow(h % q, -1, q) for h, q in zip(hats, mods)]
    out = []
    L, n = m_rns.shape
    cols = [[int(v) for v in m_rns[i]] for i in range(L)]
    for k in range(n):
        x = sum(cols[i][k] * coef[i] for i in range(L)) % Q
        out.append(x - Q if x > Q // 2 else x)
    return out


def negacyclic_int(a, b):
    n = len(a)
    out = [0] * n
    for i, ai in enumerate(a):
        if ai == 0:
            continue
        for j, bj in enumerate(b):
            k = i + j
            if k < n:
                out[k] += ai * bj
            else:
                out[k - n] -= ai * bj
    return out


def automorph_int(a, g):
    n = len(a)
    out = [0] * n
    for j, v in enumerate(a):
        d = j * g % (2 * n)
        if d >= n:
            out[d - n] = -v
        else:
            out[d] = v
    return out


def to_rns(coef, mods):
    return np.array([[int(c) % int(q) for c in coef] for q in mods], dtype=np.uint64)
