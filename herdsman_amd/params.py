"""Host-side parameter helpers (no device work).

openfhe_style_primes: NTT-friendly primes q = 1 (mod 2N) as OpenFHE generates
them (descending from 2^bits, step 2N), excluding the backend's default family
q = 1 (mod 2^32): a context built on these runs the generic 7-multiply
Montgomery path (csrc/modarith.hpp) instead of the 2-multiply special one.
Used by bench.py's generic-moduli measurement and by the tests.
"""
from __future__ import annotations

from typing import List, Sequence

_MR_BASES = (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)  # deterministic below 3.3e24


def is_prime(n: int) -> bool:
    if n < 2:
        return False
    for p in _MR_BASES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in _MR_BASES:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def openfhe_style_primes(bits_counts: Sequence[tuple], log_n: int) -> List[int]:
    """[(bits, count), ...] -> distinct primes q < 2^bits, q = 1 mod 2N, q != 1 mod 2^32,
    largest first within each group (groups in the order given)."""
    two_n = 2 << log_n
    out: List[int] = []
    for bits, count in bits_counts:
        k = ((1 << bits) - 2) // two_n
        got = 0
        while got < count:
            q = k * two_n + 1
            k -= 1
            if q % (1 << 32) == 1 or q in out or not is_prime(q):
                continue
            out.append(q)
            got += 1
    return out
