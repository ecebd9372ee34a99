"""Host model of the line cut's certified comparisons (gf-pl-slam_amd/csrc/k_cut.hip,
DESIGN.md §3): the lemmas the per-step agreement bound rests on, checked against exact
rational arithmetic (fractions.Fraction determinants, logs to 40 digits with decimal) on random,
badly scaled, near-singular and near-tie cases.

The reference decides each greedy step of estimateProjUncertainty_submodular
(src/stereoFrameHandler.cpp:1661-1764) on m^ = logdet(S + info) evaluated in floating point
(getPoseInfoOnLine's assembly, Eigen's LLT and the log of its diagonal, include/linespec.h:43-56).
The kernel decides on d (the determinant lemma) from other operands; a step is taken from d only
when every comparison clears a margin that covers
  (I)   the reference's own rounding: |m^ - logdet A| <= x / (1 - x) + 7.07 u (Lam_S + 2 tau),
        x = 6 * 15u * tau, tau = sum_i a_ii (S^-1)_ii >= tr(D A^-1 D)  [A = S + info exactly];
  (S)   a perturbation of S: |logdet(S + dS + I) - logdet(S + I)| <= e / (1 - e),
        e = sum_ik |dS_ik| sqrt((S^-1)_ii (S^-1)_kk);
  (P)   perturbed rank-one operands: |logdet(S + PP^T/v + ..) - logdet(S + P*P*^T/v* + ..)| <= N / (1 - N),
        N = sum_sides [2 eta (B + eta) / v' + (B + eta)^2 |1/v - 1/v*|], eta = sum_i e_i sqrt((S^-1)_ii);
  (RB)  running error bounds of the kernels' expression trees (gfpl_device.hpp RB), valid over
        a whole ratio range.
The -m gpu tests compare the kernels themselves with the oracle (tests/test_gpu_parity.py)."""
import math
import random
from decimal import Decimal, getcontext
from fractions import Fraction

import numpy as np
import pytest

U = 2.0 ** -53
getcontext().prec = 50


# ------------------------------------------------------------------ exact --
def det_exact(A):
    """determinant of a square matrix of Fractions (fraction-free elimination with pivoting)"""
    M = [list(r) for r in A]
    n = len(M)
    det = Fraction(1)
    for k in range(n):
        p = next((i for i in range(k, n) if M[i][k] != 0), None)
        if p is None:
            return Fraction(0)
        if p != k:
            M[k], M[p] = M[p], M[k]
            det = -det
        det *= M[k][k]
        for i in range(k + 1, n):
            f = M[i][k] / M[k][k]
            if f:
                for j in range(k, n):
                    M[i][j] -= f * M[k][j]
    return det


def log_exact(q: Fraction) -> Decimal:
    assert q > 0
    return Decimal(q.numerator).ln() - Decimal(q.denominator).ln()


def logdet_exact(A) -> Decimal:
    return log_exact(det_exact([[Fraction(float(x)) for x in r] for r in A]))


def frac_mat(A):
    return [[Fraction(float(x)) for x in r] for r in A]


def info_exact(P, v):
    """P P^T / v with Fractions"""
    Pf = [Fraction(float(x)) for x in P]
    vf = Fraction(float(v))
    return [[Pf[i] * Pf[k] / vf for k in range(6)] for i in range(6)]


def add(A, B):
    return [[A[i][k] + B[i][k] for k in range(len(A))] for i in range(len(A))]


# --------------------------------------------- the reference's evaluation --
def ref_assemble(Js, vs, Je, ve):
    """cut_assemble / getPoseInfoOnLine's [Js Je] inv(diag(vs, ve)) [Js Je]^T, float ops in order"""
    det = vs * ve - 0.0 * 0.0
    invdet = 1.0 / det
    i00, i10, i01, i11 = ve * invdet, -0.0 * invdet, -0.0 * invdet, vs * invdet
    T0 = [Js[i] * i00 + Je[i] * i10 for i in range(6)]
    T1 = [Js[i] * i01 + Je[i] * i11 for i in range(6)]
    return [[T0[i] * Js[j] + T1[i] * Je[j] for j in range(6)] for i in range(6)]


def ref_logdet(A):
    """logdet6_lower / linespec.h logdet: LLT then 2 * sum(log(diag))"""
    a = [list(map(float, r)) for r in A]
    L = [[0.0] * 6 for _ in range(6)]
    for k in range(6):
        x = a[k][k]
        for j in range(k):
            x = x - L[k][j] * L[k][j]
        if x <= 0.0:
            return float("nan")
        x = math.sqrt(x)
        L[k][k] = x
        for i in range(k + 1, 6):
            v = a[i][k]
            for j in range(k):
                v = v - L[i][j] * L[k][j]
            L[i][k] = v / x
    s = math.log(L[0][0])
    for i in range(1, 6):
        s = s + math.log(L[i][i])
    return 2.0 * s


# ------------------------------------------------------------ random cases --
def rand_spd(rng, kind):
    """6x6 SPD S of a few shapes: well conditioned, badly scaled (units), near-singular"""
    Q, _ = np.linalg.qr(rng.normal(size=(6, 6)))
    if kind == "well":
        ev = rng.uniform(0.5, 2.0, 6)
    elif kind == "ill":
        ev = 10.0 ** rng.uniform(-4, 0, 6)
    else:   # near-singular: one direction almost flat
        ev = np.concatenate([[10.0 ** rng.uniform(-9, -6)], rng.uniform(0.5, 2.0, 5)])
    S = (Q * ev) @ Q.T
    D = np.diag(10.0 ** rng.uniform(-3, 3, 6)) if kind != "well" else np.eye(6)
    S = D @ S @ D
    return (S + S.T) / 2.0


def sigma(S):
    return np.diag(np.linalg.inv(S)) * 1.01   # the kernel's s_i with a generous allowance here


def lam_bound(S):
    return sum(0.6931471805599453 * (abs(math.frexp(S[i, i])[1]) + 1) for i in range(6))


KINDS = ["well", "ill", "sing"]


@pytest.mark.parametrize("kind", KINDS)
def test_reference_llt_log_error_within_bound(kind):
    """(I): the reference's m^ against logdet of its exactly assembled matrix."""
    rng = np.random.default_rng({"well": 1, "ill": 2, "sing": 3}[kind])
    worst = 0.0
    for trial in range(40):
        S = rand_spd(rng, kind)
        sc = np.sqrt(np.diag(S))
        Js = rng.normal(size=6) * sc * rng.uniform(0.1, 10)
        Je = rng.normal(size=6) * sc * rng.uniform(0.1, 10)
        vs, ve = rng.uniform(0.1, 10.0), rng.uniform(0.1, 10.0)
        tmp = ref_assemble(list(Js), vs, list(Je), ve)
        tot = [[tmp[i][k] + S[i, k] for k in range(6)] for i in range(6)]
        m_hat = ref_logdet(tot)
        A = add(frac_mat(S), add(info_exact(Js, vs), info_exact(Je, ve)))
        M = log_exact(det_exact(A))
        a_diag = np.diag(S) + Js ** 2 / vs + Je ** 2 / ve
        tau = float(np.sum(a_diag * sigma(S)))
        x = 6 * 15 * U * tau
        if x >= 0.1:
            continue   # the kernel refuses margins there
        E = x / (1 - x) + 7.07 * U * (lam_bound(S) + 2 * tau)
        err = abs(Decimal(m_hat) - M)
        assert err <= Decimal(E), (trial, float(err), E, tau)
        worst = max(worst, float(err) / E)
    assert worst < 1.0


@pytest.mark.parametrize("kind", KINDS)
def test_s_perturbation_bound(kind):
    """(S): an entrywise-bounded change of S moves logdet(S + info) by at most e / (1 - e)."""
    rng = np.random.default_rng({"well": 11, "ill": 12, "sing": 13}[kind])
    for trial in range(30):
        S = rand_spd(rng, kind)
        sc = np.sqrt(np.diag(S))
        Ps, Pe = rng.normal(size=6) * sc, rng.normal(size=6) * sc
        vs, ve = rng.uniform(0.1, 10.0), rng.uniform(0.1, 10.0)
        sg = np.diag(np.linalg.inv(S))
        # an entry bound scaled to the diagonal, at most e ~ 1e-6
        Eb = 1e-8 * np.outer(sc, sc) * rng.uniform(0, 1, (6, 6))
        Eb = (Eb + Eb.T) / 2
        dS = Eb * rng.choice([-1.0, 1.0], (6, 6))
        dS = np.triu(dS) + np.triu(dS, 1).T
        e = float(np.sum(Eb * np.sqrt(np.outer(sg, sg)))) * 1.01
        if e >= 0.5:
            continue
        I = add(info_exact(Ps, vs), info_exact(Pe, ve))
        M0 = logdet_exact(add(frac_mat(S), I))
        M1 = log_exact(det_exact(add(add(frac_mat(S), frac_mat(dS)), I)))
        assert abs(M1 - M0) <= Decimal(e / (1 - e)), (trial, float(abs(M1 - M0)), e)


@pytest.mark.parametrize("kind", KINDS)
def test_rank_update_perturbation_bound(kind):
    """(P): perturbed rank-one terms P P^T / v on both sides."""
    rng = np.random.default_rng({"well": 21, "ill": 22, "sing": 23}[kind])
    checked = 0
    for trial in range(30):
        S = rand_spd(rng, kind)
        sc = np.sqrt(np.diag(S))
        sg = np.diag(np.linalg.inv(S))
        Lc = np.linalg.cholesky(S)
        terms = []
        N = 0.0
        Pp = []
        for side in range(2):
            P = rng.normal(size=6) * sc * rng.uniform(0.1, 3)
            v = rng.uniform(0.1, 10.0)
            e = np.abs(P) * 1e-9 * rng.uniform(0, 1, 6) + 1e-12 * sc
            ev = v * 1e-9
            dP = e * rng.uniform(-1, 1, 6)
            dv = ev * rng.uniform(-1, 1)
            B = float(np.linalg.norm(np.linalg.solve(Lc, P))) * 1.001
            eta = float(np.sum(e * np.sqrt(sg))) * 1.001
            N += 2 * eta * (B + eta) / (v - ev) + (B + eta) ** 2 * ev / ((v - ev) * (v - ev))
            Pp.append((P, v, P + dP, v + dv))
        if N >= 0.5:
            continue   # the kernel refuses margins there
        checked += 1
        A0 = frac_mat(S)
        A1 = frac_mat(S)
        for P, v, P2, v2 in Pp:
            A0 = add(A0, info_exact(P, v))
            A1 = add(A1, info_exact(P2, v2))
        d = abs(log_exact(det_exact(A1)) - log_exact(det_exact(A0)))
        assert d <= Decimal(N / (1 - N)), (trial, float(d), N)
    assert checked >= 10


# ------------------------------------------------------- running bounds --
class RB:
    """gfpl_device.hpp RB: m >= |computed|, |exact|; e >= |computed - exact|; lo lower bound"""

    def __init__(self, m, e=0.0, lo=None):
        self.m, self.e = m, e
        self.lo = m if lo is None else lo

    @staticmethod
    def c(x):
        return RB(abs(x), 0.0, abs(x))

    def __add__(self, o):
        m = self.m + o.m
        return RB(m * (1 + 4 * U), self.e + o.e + U * m, 0.0)

    __sub__ = __add__

    def __neg__(self):
        return self

    def __mul__(self, o):
        m = self.m * o.m
        return RB(m * (1 + 4 * U), self.e * o.m + self.m * o.e + U * m, self.lo * o.lo * (1 - 4 * U))

    def __truediv__(self, o):
        if not o.lo > 0:
            return RB(math.inf, math.inf, 0.0)
        m = self.m / o.lo
        return RB(m * (1 + 4 * U), self.e / o.lo + (self.m / o.lo) * (o.e / o.lo) + U * m, self.lo / o.m * (1 - 4 * U))


def se3_apply(T, P, mk):
    return [((mk(T[i][0]) * P[0] + mk(T[i][1]) * P[1]) + mk(T[i][2]) * P[2]) + mk(T[i][3]) for i in range(3)]


def pose_jac(fx, homog, g, lx, ly, mk, rmax):
    gx, gy, gz = g
    gz2 = gz * gz
    fgz2 = mk(fx) / rmax(homog, gz2)
    return [(fgz2 * lx) * gz, (fgz2 * ly) * gz, (-fgz2) * ((gx * lx) + (gy * ly)),
            (-fgz2) * ((((gx * gy) * lx) + ((gy * gy) * ly)) + ((gz * gz) * ly)),
            fgz2 * ((((gx * gx) * lx) + ((gz * gz) * lx)) + ((gx * gy) * ly)),
            fgz2 * (((gx * gz) * ly) - ((gy * gz) * lx))]


def blended_jac(T, P0, P1, c, fx, homog, lx, ly, mk, rmax, zlo=None):
    Pt = [(mk(1.0) - c) * P0[k] + c * P1[k] for k in range(3)]
    cur = se3_apply(T, Pt, mk)
    if zlo is not None:   # rb_floor
        cur[2].lo = max(cur[2].lo, zlo - cur[2].e)
    return pose_jac(fx, homog, cur, lx, ly, mk, rmax)


def test_running_error_bounds_cover_the_endpoint_jacobian():
    """(RB) over a ratio range: getPoseInfoOnLine's blended-endpoint Jacobian (se3_apply, poseJac)
    computed in doubles vs exactly, at many ratios c in [0, 1], against one RB evaluation with
    c's magnitude 1 and the depth's lower bound."""
    rng = random.Random(5)
    worst = 0.0
    for trial in range(60):
        R, _ = np.linalg.qr(np.random.default_rng(trial).normal(size=(3, 3)))
        t = [rng.uniform(-0.5, 0.5) for _ in range(3)]
        T = [[float(R[i][0]), float(R[i][1]), float(R[i][2]), t[i]] for i in range(3)]
        P0 = [rng.uniform(-3, 3), rng.uniform(-2, 2), rng.uniform(2, 9)]
        P1 = [P0[0] + rng.uniform(-1, 1), P0[1] + rng.uniform(-1, 1), P0[2] + rng.uniform(-0.5, 0.5)]
        lx, ly = rng.uniform(-1, 1), rng.uniform(-1, 1)
        fx, homog = 554.25626, 1e-7
        # depth range of the transformed segment, exact
        zf = [sum(Fraction(T[2][k]) * Fraction(P[k]) for k in range(3)) + Fraction(T[2][3]) for P in (P0, P1)]
        if zf[0] * zf[1] <= 0:
            continue
        zlo = float(min(abs(zf[0]), abs(zf[1]))) * (1 - 1e-12)
        rb = blended_jac(T, [RB.c(x) for x in P0], [RB.c(x) for x in P1], RB(1.0, 0.0, 0.0), fx, homog,
                         RB.c(lx), RB.c(ly), RB.c, lambda h, x: RB(max(abs(h), x.m), x.e, max(abs(h), x.lo)), zlo)
        for c in [0.0, 0.05, 0.35, 0.5, 0.95, 1.0, rng.random()]:
            got = blended_jac(T, P0, P1, c, fx, homog, lx, ly, float, lambda h, x: x if h < x else h)
            ex = blended_jac(T, [Fraction(x) for x in P0], [Fraction(x) for x in P1], Fraction(c), fx, homog,
                             Fraction(lx), Fraction(ly), Fraction, lambda h, x: x if Fraction(h) < x else Fraction(h))
            for i in range(6):
                err = abs(Fraction(got[i]) - ex[i])
                assert err <= Fraction(rb[i].e), (trial, c, i, float(err), rb[i].e)
                assert abs(ex[i]) <= Fraction(rb[i].m) and abs(got[i]) <= rb[i].m
                if rb[i].e > 0:
                    worst = max(worst, float(err) / rb[i].e)
    assert worst <= 1.0


# ------------------------------------------------ decisions near ties --
def test_certified_decisions_follow_the_exact_order_near_ties():
    """The margin rule: a decision is taken from computed values only when their gap exceeds
    the margin plus both values' bounds; near-ties built to 1e-13 .. 1e-7 apart are then either
    refused or ordered as the exact values are (and as the reference's m^ are)."""
    rng = np.random.default_rng(9)
    tau = 1e-9
    taken = refused = 0
    for trial in range(60):
        S = rand_spd(rng, KINDS[trial % 3])
        sc = np.sqrt(np.diag(S))
        P = rng.normal(size=6) * sc
        v = rng.uniform(0.5, 2.0)
        Pe = rng.normal(size=6) * sc
        ve = rng.uniform(0.5, 2.0)
        gap = 10.0 ** rng.uniform(-13, -7)
        # two candidates whose end variances differ by a relative `gap`
        cands = [(ve, ref_logdet([[x + y for x, y in zip(r1, r2)] for r1, r2 in
                                  zip(ref_assemble(list(P), v, list(Pe), ve0), S.tolist())]))
                 for ve0 in (ve, ve * (1 + gap))]
        M = [log_exact(det_exact(add(frac_mat(S), add(info_exact(P, v), info_exact(Pe, ve0)))))
             for ve0 in (ve, ve * (1 + gap))]
        a_diag = np.diag(S) + P ** 2 / v + Pe ** 2 / min(ve, ve * (1 + gap))
        tau_tr = float(np.sum(a_diag * sigma(S)))
        x = 6 * 15 * U * tau_tr
        E = x / (1 - x) + 7.07 * U * (lam_bound(S) + 2 * tau_tr)
        # the rule on the reference-side values: |m^ - M| <= E each, the computed gap must clear
        # the relative margin tau plus 2E
        g = cands[0][1] - cands[1][1]
        if abs(g) > math.log1p(tau) + 2 * E and E <= tau / 8:
            taken += 1
            assert (g > 0) == (M[0] > M[1]), (trial, g, float(M[0] - M[1]))
        else:
            refused += 1
    assert taken > 0 and refused > 0
