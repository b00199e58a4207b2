"""Independent Python big-integer model of the RNS-FHE hot path.

TEST INFRASTRUCTURE ONLY (see oracle/fhe_oracle.h).  Used by
tests/golden/make_golden.py to generate the committed golden vectors that pin
the C oracle (oracle/fhe_oracle.c) and, transitively, the HIP backend.

Parity status: "parity unpinned" against herdsman -- /root/reference contains
no FHE arithmetic (OpenFHE linked at CMakeLists.txt:73,
210-211 but never called).  This model is pinned to mathematical ground truth
instead: every transform here is written from its defining formula with
Python integers, using algorithms deliberately different from the C oracle
(e.g. the NTT is a twist + recursive cyclic FFT checked against the O(N^2)
evaluation definition, not Harvey's in-place butterflies), and the scheme
level checks (decryption of products / rotations) are done with exact CRT
reconstruction in tests/.

Conventions are those of include/plugins/fhe_backend.h.
"""
from __future__ import annotations

import math
from typing import List, Sequence

MASK64 = (1 << 64) - 1


# ----------------------------------------------------------------- primes
def is_prime(n: int) -> bool:
    if n < 2:
        return False
    small = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37]
    for p in small:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in small:
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


def gen_primes(bits: int, log_n: int, count: int, exclude: Sequence[int] = ()) -> List[int]:
    """The backend's prime family: largest primes q < 2^bits with q = 1 mod 2^32
    (which implies q = 1 mod 2N for N <= 2^31), descending."""
    assert 2 << log_n <= 1 << 32
    step = 1 << 32
    k = ((1 << bits) - 2) // step
    out: List[int] = []
    while k > 0 and len(out) < count:
        q = k * step + 1
        if q not in exclude and is_prime(q):
            out.append(q)
        k -= 1
    return out


def min_psi(q: int, log_n: int) -> int:
    """Smallest primitive 2N-th root of unity mod q."""
    n = 1 << log_n
    x = 2
    while True:
        g = pow(x, (q - 1) // (2 * n), q)
        if pow(g, n, q) == q - 1:
            break
        x += 1
    return min(pow(g, 2 * k + 1, q) for k in range(n))


def brv(x: int, bits: int) -> int:
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


# -------------------------------------------------------------------- NTT
def _fft_cyclic(a: List[int], w: int, q: int) -> List[int]:
    n = len(a)
    if n == 1:
        return list(a)
    ev = _fft_cyclic(a[0::2], w * w % q, q)
    od = _fft_cyclic(a[1::2], w * w % q, q)
    out = [0] * n
    t = 1
    for k in range(n // 2):
        x = od[k] * t % q
        out[k] = (ev[k] + x) % q
        out[k + n // 2] = (ev[k] - x) % q
        t = t * w % q
    return out


def ntt_fwd(a: Sequence[int], q: int, psi: int) -> List[int]:
    """out[k] = a(psi^(2 brv(k) + 1)) mod q  (twist + cyclic FFT)."""
    n = len(a)
    lg = n.bit_length() - 1
    b = [a[j] * pow(psi, j, q) % q for j in range(n)]
    B = _fft_cyclic(b, psi * psi % q, q)
    return [B[brv(k, lg)] for k in range(n)]


def ntt_fwd_direct(a: Sequence[int], q: int, psi: int) -> List[int]:
    """O(N^2) defining formula (used only to validate ntt_fwd)."""
    n = len(a)
    lg = n.bit_length() - 1
    out = []
    for k in range(n):
        x = pow(psi, 2 * brv(k, lg) + 1, q)
        acc = 0
        for c in reversed(a):
            acc = (acc * x + c) % q
        out.append(acc)
    return out


def ntt_inv(A: Sequence[int], q: int, psi: int) -> List[int]:
    n = len(A)
    lg = n.bit_length() - 1
    B = [0] * n
    for k in range(n):
        B[brv(k, lg)] = A[k]
    winv = pow(psi * psi % q, q - 2, q)
    b = _fft_cyclic(B, winv, q)
    ninv = pow(n, q - 2, q)
    ipsi = pow(psi, q - 2, q)
    return [b[j] * ninv % q * pow(ipsi, j, q) % q for j in range(n)]


def negacyclic_mul(a: Sequence[int], b: Sequence[int], q: int) -> List[int]:
    n = len(a)
    out = [0] * n
    for i in range(n):
        if a[i] == 0:
            continue
        for j in range(n):
            k = i + j
            if k < n:
                out[k] += a[i] * b[j]
            else:
                out[k - n] -= a[i] * b[j]
    return [x % q for x in out]


# ----------------------------------------------------------- automorphism
def automorph_ntt(A: Sequence[int], g: int) -> List[int]:
    n = len(A)
    lg = n.bit_length() - 1
    out = [0] * n
    for k in range(n):
        e = 2 * brv(k, lg) + 1
        e2 = e * g % (2 * n)
        out[k] = A[brv((e2 - 1) // 2, lg)]
    return out


def automorph_coef(a: Sequence[int], g: int, q: int) -> List[int]:
    n = len(a)
    out = [0] * n
    for j in range(n):
        d = j * g % (2 * n)
        if d >= n:
            out[d - n] = (-a[j]) % q
        else:
            out[d] = a[j] % q
    return out


def galois_elt(log_n: int, steps: int) -> int:
    n = 1 << log_n
    return pow(5, steps % (n // 2), 2 * n)


# -------------------------------------------------------- base conversion
def base_conv(xs: Sequence[Sequence[int]], src: Sequence[int], dst: Sequence[int]) -> List[List[int]]:
    """Fast (approximate) base conversion, defined per coefficient:
    y_m = sum_i [x_i (S/s_i)^-1]_{s_i} * (S/s_i)  mod m."""
    S = math.prod(src)
    n = len(xs[0])
    hats = [S // s for s in src]
    hinv = [pow(h % s, -1, s) for h, s in zip(hats, src)]
    out = [[0] * n for _ in dst]
    for k in range(n):
        v = [xs[i][k] * hinv[i] % src[i] for i in range(len(src))]
        total = sum(vi * h for vi, h in zip(v, hats))  # exact integer = x + u*S
        for m, dm in enumerate(dst):
            out[m][k] = total % dm
    return out


# ----------------------------------------------------------------- params
class Params:
    def __init__(self, log_n: int, L: int, K: int, dnum: int, moduli: Sequence[int],
                 scheme: str = "ckks", t: int = 0):
        self.log_n, self.n, self.L, self.K, self.dnum = log_n, 1 << log_n, L, K, dnum
        self.alpha = -(-L // dnum)
        self.moduli = list(moduli)
        self.scheme, self.t = scheme, t
        self.psi = [min_psi(q, log_n) for q in self.moduli]
        self.Q = self.moduli[:L]
        self.P = self.moduli[L:L + K]
        self.Bsk = self.moduli[L + K:]

    def ntt(self, limbs, mods):
        return [ntt_fwd(x, self.moduli[m], self.psi[m]) for x, m in zip(limbs, mods)]

    def intt(self, limbs, mods):
        return [ntt_inv(x, self.moduli[m], self.psi[m]) for x, m in zip(limbs, mods)]


# ------------------------------------------------------- hybrid keyswitch
def keyswitch(p: Params, d: List[List[int]], ksk, ntt_form: bool, lvl: int = None, ext_g: int = 0, multi=None):
    """Hybrid key switching at level lvl (default L).  d: lvl limbs (NTT form if
    ntt_form).  ksk[j][b][i] limb i of Q u P of the FULL-level key (NTT form);
    at a reduced level the digits partition the lvl active limbs by alpha and
    only the key rows of Q_lvl u P are used.  Returns (ks0, ks1), each lvl limbs.
    multi = [(ksk_r, g_r), ...] (double-hoisted rotation sum): the inner products
    of every key with sigma_{g_r}(ext) are summed before the one ModDown."""
    keys = [(kk[0], kk[1], kk[2] if len(kk) > 2 else None) for kk in multi] if multi is not None \
        else [(ksk, ext_g, None)]
    L, K = (p.L if lvl is None else lvl), p.K
    mi = list(range(L)) + [p.L + k for k in range(K)]  # level space -> modulus / key row
    QP = list(range(L + K))
    if ntt_form:
        dn, dc = d, p.intt(d, range(L))
    else:
        dc, dn = d, p.ntt(d, range(L))
    acc = [[[0] * p.n for _ in QP] for _ in range(2)]
    for j in range(p.dnum):
        lo, hi = j * p.alpha, min((j + 1) * p.alpha, L)
        if lo >= L:
            break
        others = [i for i in QP if not (lo <= i < hi)]
        conv = base_conv(dc[lo:hi], p.moduli[lo:hi], [p.moduli[mi[i]] for i in others])
        conv_n = p.ntt(conv, [mi[i] for i in others])
        ext = {}
        for i in range(lo, hi):
            ext[i] = dn[i]
        for i, c in zip(others, conv_n):
            ext[i] = c
        for kr, g, pt in keys:
            # hoisted rotation: sigma_g applied to the digit's extension; pt: a
            # plaintext weight (hoisted linear transform), rows like the key's
            ex = {i: automorph_ntt(e, g) for i, e in ext.items()} if g else ext
            for b in range(2):
                for i in QP:
                    q = p.moduli[mi[i]]
                    kb = kr[j][b][mi[i]]
                    e = ex[i]
                    row = acc[b][i]
                    w = pt[mi[i]] if pt is not None else None
                    for k in range(p.n):
                        v = e[k] * kb[k]
                        if w is not None:
                            v = v % q * w[k]
                        row[k] = (row[k] + v) % q
    Pprod = math.prod(p.P)
    Qs = p.moduli[:L]
    out = []
    for b in range(2):
        if ntt_form:
            accP = p.intt(acc[b][L:], range(p.L, p.L + K))
            accQ = acc[b][:L]
        else:
            accQ = p.intt(acc[b][:L], range(L))
            accP = p.intt(acc[b][L:], range(p.L, p.L + K))
        conv = base_conv(accP, p.P, Qs)
        if ntt_form:
            conv = p.ntt(conv, range(L))
        res = []
        for i in range(L):
            q = p.moduli[i]
            pinv = pow(Pprod % q, -1, q)
            res.append([(accQ[i][k] - conv[i][k]) * pinv % q for k in range(p.n)])
        out.append(res)
    return out


def rotate_sum_hoisted(p: Params, ct, gs, gks):
    """Double-hoisted rotation sum: sum_r rot_{g_r}(ct) with the inner products of
    every key summed before ONE ModDown, plus sum_r sigma_{g_r}(c0)."""
    ckks = p.scheme == "ckks"
    ks0, ks1 = keyswitch(p, ct[1], None, ckks, None, 0, list(zip(gks, gs)))
    c0 = ks0
    for g in gs:
        if ckks:
            r0 = [automorph_ntt(x, g) for x in ct[0]]
        else:
            r0 = [automorph_coef(x, g, p.moduli[i]) for i, x in enumerate(ct[0])]
        c0 = [[(x + y) % p.moduli[i] for x, y in zip(c0[i], r0[i])] for i in range(p.L)]
    return [c0, ks1]


def linear_hoisted(p: Params, ct, gs, gks, pts):
    """Hoisted linear transform (CKKS): sum_r pts[r] (.) rot_{g_r}(ct) with the
    plaintext-weighted inner products summed before ONE ModDown.  pts[r]: L+K
    limbs in the NTT domain."""
    ks0, ks1 = keyswitch(p, ct[1], None, True, None, 0, list(zip(gks, gs, pts)))
    c0 = ks0
    for g, pt in zip(gs, pts):
        r0 = [automorph_ntt(x, g) for x in ct[0]]
        c0 = [[(x + y * w) % p.moduli[i] for x, y, w in zip(c0[i], r0[i], pt[i])] for i in range(p.L)]
    return [c0, ks1]


def ckks_mul_relin_at(p: Params, a, b, rlk, lvl: int):
    """ckks_mul_relin on ciphertexts of lvl limbs (the first lvl Q primes)."""
    n = p.n
    d0, d1, d2 = [], [], []
    for i in range(lvl):
        q = p.moduli[i]
        d0.append([a[0][i][k] * b[0][i][k] % q for k in range(n)])
        d1.append([(a[0][i][k] * b[1][i][k] + a[1][i][k] * b[0][i][k]) % q for k in range(n)])
        d2.append([a[1][i][k] * b[1][i][k] % q for k in range(n)])
    ks0, ks1 = keyswitch(p, d2, rlk, True, lvl)
    return [[[(x + y) % p.moduli[i] for x, y in zip(d0[i], ks0[i])] for i in range(lvl)],
            [[(x + y) % p.moduli[i] for x, y in zip(d1[i], ks1[i])] for i in range(lvl)]]


def rescale(p: Params, ct, lvl: int):
    """CKKS rescale of an NTT-form ciphertext of lvl limbs, by its definition on
    integers: each coefficient c in [0, Q_lvl) (CRT) becomes round(c / q_{lvl-1})
    = (c - r) / q_{lvl-1} with r the centred residue of c mod q_{lvl-1} (ties,
    r = (q-1)/2, round down as in OpenFHE / SEAL), reduced mod the remaining
    lvl - 1 primes and transformed back."""
    Qs, ql = p.moduli[:lvl], p.moduli[lvl - 1]
    out = []
    for poly in ct:
        coef = p.intt(poly, range(lvl))
        res = [[0] * p.n for _ in range(lvl - 1)]
        for k in range(p.n):
            c = crt([coef[i][k] for i in range(lvl)], Qs)
            r = c % ql
            if r > ql // 2:
                r -= ql
            v = (c - r) // ql
            for i in range(lvl - 1):
                res[i][k] = v % Qs[i]
        out.append(p.ntt(res, range(lvl - 1)))
    return out


def ckks_mul_relin(p: Params, a, b, rlk):
    """a, b: ciphertexts [2][L][N] in NTT form."""
    L, n = p.L, p.n
    d0, d1, d2 = [], [], []
    for i in range(L):
        q = p.moduli[i]
        d0.append([a[0][i][k] * b[0][i][k] % q for k in range(n)])
        d1.append([(a[0][i][k] * b[1][i][k] + a[1][i][k] * b[0][i][k]) % q for k in range(n)])
        d2.append([a[1][i][k] * b[1][i][k] % q for k in range(n)])
    ks0, ks1 = keyswitch(p, d2, rlk, True)
    return [[[(x + y) % p.moduli[i] for x, y in zip(d0[i], ks0[i])] for i in range(L)],
            [[(x + y) % p.moduli[i] for x, y in zip(d1[i], ks1[i])] for i in range(L)]]


def rotate(p: Params, ct, g: int, gk):
    L = p.L
    if p.scheme == "ckks":
        c0 = [automorph_ntt(x, g) for x in ct[0]]
        c1 = [automorph_ntt(x, g) for x in ct[1]]
    else:
        c0 = [automorph_coef(x, g, p.moduli[i]) for i, x in enumerate(ct[0])]
        c1 = [automorph_coef(x, g, p.moduli[i]) for i, x in enumerate(ct[1])]
    ks0, ks1 = keyswitch(p, c1, gk, p.scheme == "ckks")
    return [[[(x + y) % p.moduli[i] for x, y in zip(c0[i], ks0[i])] for i in range(L)], ks1]


def rotate_hoisted(p: Params, ct, gs, gks):
    """Rotations of one ciphertext by every g in gs sharing one ModUp of c1: KS
    over sigma_g(ModUp(c1)) with key gks[r] (OpenFHE EvalFastRotation).  CKKS in
    the NTT domain; BFV in the coefficient domain (c0 by the signed coefficient
    map, the extension permuted in the NTT domain of the inner product)."""
    ckks = p.scheme == "ckks"
    out = []
    for g, gk in zip(gs, gks):
        if ckks:
            c0 = [automorph_ntt(x, g) for x in ct[0]]
        else:
            c0 = [automorph_coef(x, g, p.moduli[i]) for i, x in enumerate(ct[0])]
        ks0, ks1 = keyswitch(p, ct[1], gk, ckks, None, g)
        out.append([[[(x + y) % p.moduli[i] for x, y in zip(c0[i], ks0[i])] for i in range(p.L)], ks1])
    return out


# -------------------------------------------------------------- BFV BEHZ
def _centered(x: int, m: int) -> int:
    return x - m if x >= (m + 1) // 2 else x


def bfv_mul_relin(p: Params, a, b, rlk):
    """BEHZ multiplication (SEAL RNSTool form) + hybrid relinearization.
    a, b: [2][L][N] coefficient form."""
    L, n, t = p.L, p.n, p.t
    Q, Bsk = p.Q, p.Bsk
    B, msk = Bsk[:-1], Bsk[-1]
    mt = 1 << 32
    Qp, Bp = math.prod(Q), math.prod(B)
    qhat = [Qp // q for q in Q]
    qhinv = [pow(h % q, -1, q) for h, q in zip(qhat, Q)]
    bsk_mods = list(range(L + p.K, L + p.K + len(Bsk)))

    def extend(x):  # fastbconv_m_tilde + sm_mrq, per coefficient
        out = [[0] * n for _ in Bsk]
        for k in range(n):
            v = [x[i][k] * mt * qhinv[i] % Q[i] for i in range(L)]
            total = sum(vi * h for vi, h in zip(v, qhat))
            xmt = total % mt
            r = (-xmt * pow(Qp, -1, mt)) % mt
            r = r - mt if r >= mt // 2 else r
            for j, bj in enumerate(Bsk):
                out[j][k] = (total + Qp * r) * pow(mt, -1, bj) % bj
        return out

    polys = [a[0], a[1], b[0], b[1]]
    xq = [p.ntt(x, range(L)) for x in polys]
    xb = [p.ntt(extend(x), bsk_mods) for x in polys]

    def tensor(x, mods):
        e0, e1, e2 = [], [], []
        for i, m in enumerate(mods):
            q = p.moduli[m]
            a0, a1, b0, b1 = x[0][i], x[1][i], x[2][i], x[3][i]
            e0.append([u * v % q for u, v in zip(a0, b0)])
            e1.append([(u * v + w * z) % q for u, v, w, z in zip(a0, b1, a1, b0)])
            e2.append([u * v % q for u, v in zip(a1, b1)])
        return [e0, e1, e2]

    eq = [p.intt(e, range(L)) for e in tensor(xq, range(L))]
    eb = [p.intt(e, bsk_mods) for e in tensor(xb, bsk_mods)]
    res = []
    bhat = [Bp // bb for bb in B]
    bhinv = [pow(h % bb, -1, bb) for h, bb in zip(bhat, B)]
    for e_q, e_b in zip(eq, eb):
        out = [[0] * n for _ in Q]
        for k in range(n):
            # fast_floor: ((t x)_b - conv_Q->b((t x)_Q)) * Q^-1 mod b
            v = [e_q[i][k] * t % Q[i] * qhinv[i] % Q[i] for i in range(L)]
            total = sum(vi * h for vi, h in zip(v, qhat))
            fl = [((e_b[j][k] * t - total) * pow(Qp, -1, bj)) % bj for j, bj in enumerate(Bsk)]
            # fastbconv_sk
            w = [fl[j] * bhinv[j] % B[j] for j in range(len(B))]
            tot_b = sum(wj * h for wj, h in zip(w, bhat))
            alpha = ((tot_b - fl[-1]) * pow(Bp, -1, msk)) % msk
            alpha = alpha - msk if alpha > msk // 2 else alpha
            for i, q in enumerate(Q):
                out[i][k] = (tot_b - alpha * Bp) % q
        res.append(out)
    ks0, ks1 = keyswitch(p, res[2], rlk, False)
    return [[[(x + y) % Q[i] for x, y in zip(res[0][i], ks0[i])] for i in range(L)],
            [[(x + y) % Q[i] for x, y in zip(res[1][i], ks1[i])] for i in range(L)]]


# ------------------------------------------------------------- BFV HPS
def hps_tables(p: Params):
    """Constants of the HPS multiplication (Halevi-Polyakov-Shoup 2018; OpenFHE
    BFVrns multiplication technique HPS) with P = the Bsk primes.  The doubles
    are formed exactly as the C oracle and the backend form them:
    (double)num / (double)q and 1.0 / (double)q, each a correctly rounded
    IEEE-754 operation."""
    Q, P, t = p.Q, p.Bsk, p.t
    Qp, Pp = math.prod(Q), math.prod(P)
    T = {"Q": Q, "P": P, "Qp": Qp, "Pp": Pp}
    T["qt"] = [pow((Qp // q) % q, -1, q) for q in Q]                      # (Q/q_i)^-1 mod q_i
    T["invq"] = [1.0 / float(q) for q in Q]
    T["qstar_p"] = [[(Qp // q) % pj for pj in P] for q in Q]              # Q/q_i mod p_j
    T["Q_p"] = [Qp % pj for pj in P]
    num = [t * qt % q for qt, q in zip(T["qt"], Q)]                        # t (Q/q_i)^-1 mod q_i
    T["frac"] = [float(nm) / float(q) for nm, q in zip(num, Q)]           # frac(t P c_i / q_i)
    T["I"] = [[(-nm * pow(q, -1, pj)) % pj for pj in P] for nm, q in zip(num, Q)]
    T["lam"] = [t * pow(Qp % pj, -1, pj) % pj for pj in P]                # t Q^-1 mod p_j
    T["pt"] = [pow((Pp // pj) % pj, -1, pj) for pj in P]
    T["invp"] = [1.0 / float(pj) for pj in P]
    T["pstar_q"] = [[(Pp // pj) % q for q in Q] for pj in P]
    T["P_q"] = [Pp % q for q in Q]
    return T


def hps_extend(T, xq):
    """Q -> P exact base extension of the centred lift (HPS section 2.4): y_i =
    [x_i (Q/q_i)^-1]_{q_i}, v = floor(0.5 + sum_i y_i / q_i) in doubles, and
    x mod p_j = sum_i y_i [Q/q_i]_{p_j} - v [Q]_{p_j}."""
    Q, P = T["Q"], T["P"]
    n = len(xq[0])
    out = [[0] * n for _ in P]
    for k in range(n):
        y = [xq[i][k] * T["qt"][i] % q for i, q in enumerate(Q)]
        sm = 0.0
        for i in range(len(Q)):
            sm = sm + float(y[i]) * T["invq"][i]
        v = int(sm + 0.5)
        for j, pj in enumerate(P):
            out[j][k] = (sum(y[i] * T["qstar_p"][i][j] for i in range(len(Q))) - v * T["Q_p"][j]) % pj
    return out


def hps_scale(T, eq, ep):
    """round(t d / Q) for d given in Q u P (coefficient form, canonical), in P
    (HPS simple scaling: integer parts I_ij, fractional parts in doubles), then
    P -> Q by the exact extension of the centred lift."""
    Q, P = T["Q"], T["P"]
    n = len(eq[0])
    out = [[0] * n for _ in Q]
    for k in range(n):
        nu = 0.5
        for i in range(len(Q)):
            nu = nu + float(eq[i][k]) * T["frac"][i]
        r = int(nu)
        z = [(sum(eq[i][k] * T["I"][i][j] for i in range(len(Q))) + r + ep[j][k] * T["lam"][j]) % pj
             for j, pj in enumerate(P)]
        y = [z[j] * T["pt"][j] % pj for j, pj in enumerate(P)]
        sm = 0.0
        for j in range(len(P)):
            sm = sm + float(y[j]) * T["invp"][j]
        v = int(sm + 0.5)
        for i, q in enumerate(Q):
            out[i][k] = (sum(y[j] * T["pstar_q"][j][i] for j in range(len(P))) - v * T["P_q"][i]) % q
    return out


def bfv_mul_relin_hps(p: Params, a, b, rlk, check_exact: bool = True):
    """HPS multiplication + hybrid relinearization.  a, b: [2][L][N] coefficient
    form.  With check_exact, each tensor output is compared with its definition
    round(t d / Q) on integers (d the negacyclic tensor of the centred lifts):
    the floating-point parts may differ from it by a few units, BFV noise."""
    L, n, t = p.L, p.n, p.t
    T = hps_tables(p)
    Q, P = T["Q"], T["P"]
    pmods = list(range(L + p.K, L + p.K + len(P)))
    polys = [a[0], a[1], b[0], b[1]]
    xq = [p.ntt(x, range(L)) for x in polys]
    xp = [p.ntt(hps_extend(T, x), pmods) for x in polys]

    def tensor(x, mods):
        e0, e1, e2 = [], [], []
        for i, m in enumerate(mods):
            q = p.moduli[m]
            a0, a1, b0, b1 = x[0][i], x[1][i], x[2][i], x[3][i]
            e0.append([u * v % q for u, v in zip(a0, b0)])
            e1.append([(u * v + w * z) % q for u, v, w, z in zip(a0, b1, a1, b0)])
            e2.append([u * v % q for u, v in zip(a1, b1)])
        return [e0, e1, e2]

    eq = [p.intt(e, range(L)) for e in tensor(xq, range(L))]
    ep = [p.intt(e, pmods) for e in tensor(xp, pmods)]
    res = [hps_scale(T, e_q, e_p) for e_q, e_p in zip(eq, ep)]
    if check_exact:
        Qp = T["Qp"]
        lift = [[_centered(crt([x[i][k] for i in range(L)], Q), Qp) for k in range(n)] for x in polys]
        d = [negacyclic_int_poly(lift[0], lift[2]),
             [u + v for u, v in zip(negacyclic_int_poly(lift[0], lift[3]), negacyclic_int_poly(lift[1], lift[2]))],
             negacyclic_int_poly(lift[1], lift[3])]
        for e, dd in zip(res, d):
            for k in range(n):
                want = (2 * t * dd[k] + Qp) // (2 * Qp)  # round(t d / Q), compared mod Q
                got = crt([e[i][k] for i in range(L)], Q)
                assert abs(_centered((got - want) % Qp, Qp)) <= 1 << 16, k
    ks0, ks1 = keyswitch(p, res[2], rlk, False)
    return [[[(x + y) % Q[i] for x, y in zip(res[0][i], ks0[i])] for i in range(L)],
            [[(x + y) % Q[i] for x, y in zip(res[1][i], ks1[i])] for i in range(L)]]


def negacyclic_int_poly(a: Sequence[int], b: Sequence[int]) -> List[int]:
    """Exact negacyclic product over the integers (schoolbook)."""
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


# ---------------------------------------------------------------- helpers
def crt(residues: Sequence[int], mods: Sequence[int]) -> int:
    M = math.prod(mods)
    x = 0
    for r, m in zip(residues, mods):
        h = M // m
        x += r * h * pow(h % m, -1, m)
    return x % M
