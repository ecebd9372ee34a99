// gfpl_device.hpp — device-side numerics shared by the gfx950 kernels.
//
// Every routine evaluates in the exact operation order documented in
// DESIGN.md §Numerics (pins N1-N4), compiled with -ffp-contract=off, so
// results are bit-identical to the CPU oracle's restatement: f64 + - * / and
// sqrt are IEEE correctly rounded on gfx950 (measured: tools/probe/fp_probe.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gfpl.h"

#define GFPL_DEV __device__ __forceinline__

namespace gfpl {

// ------------------------------------------------------------- bit helpers
GFPL_DEV uint32_t hiw(double x) { return (uint32_t)((uint64_t)__double_as_longlong(x) >> 32); }
GFPL_DEV uint32_t low(double x) { return (uint32_t)(uint64_t)__double_as_longlong(x); }
GFPL_DEV double with_hi(double x, uint32_t hi) {
    uint64_t u = (uint64_t)__double_as_longlong(x);
    u = ((uint64_t)hi << 32) | (u & 0xffffffffull);
    return __longlong_as_double((long long)u);
}
GFPL_DEV double from_words(uint32_t hi, uint32_t lo) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// ------------------------------------------------- fdlibm log / sin / cos
// e_log.c, k_sin.c, k_cos.c, e_rem_pio2.c (medium range) — pin N3.
// The log / sin / cos below restate the algorithms and coefficient tables of Sun fdlibm
// (e_log.c, k_sin.c, k_cos.c, e_rem_pio2.c), whose notice is preserved here:
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this software is freely granted,
//   provided that this notice is preserved.
GFPL_DEV double det_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16,
                 Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    int32_t hx = (int32_t)hiw(x);
    uint32_t lx = low(x);
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -__builtin_inf();
        if (hx < 0) return __builtin_nan("");
        k -= 54; x *= two54;
        hx = (int32_t)hiw(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    x = with_hi(x, (uint32_t)(hx | (i ^ 0x3ff00000)));
    k += (i >> 20);
    double f = x - 1.0;
    double dk;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k; return dk * ln2_hi + dk * ln2_lo;
        }
        double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k; return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    double s = f / (2.0 + f);
    dk = (double)k;
    double z = s * s;
    i = hx - 0x6147a;
    double w = z * z;
    int32_t j = 0x6b851 - hx;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    double R = t2 + t1;
    if (i > 0) {
        double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

GFPL_DEV double k_sin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    uint32_t ix = hiw(x) & 0x7fffffff;
    if (ix < 0x3e400000) { if ((int)x == 0) return x; }
    double z = x * x;
    double v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

GFPL_DEV double k_cos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    uint32_t ix = hiw(x) & 0x7fffffff;
    if (ix < 0x3e400000) { if ((int)x == 0) return 1.0; }
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y));
    double qx;
    if (ix > 0x3fe90000) qx = 0.28125;
    else qx = from_words(ix - 0x00200000, 0);
    double hz = 0.5 * z - qx;
    double a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}

#define GFPL_REM_FAIL (-2147483647 - 1)
GFPL_DEV int rem_pio2(double x, double* y) {
    const double invpio2 = 6.36619772367581382433e-01,
                 pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11,
                 pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21,
                 pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    int32_t hx = (int32_t)hiw(x);
    uint32_t ix = (uint32_t)hx & 0x7fffffff;
    if (ix <= 0x3fe921fb) { y[0] = x; y[1] = 0; return 0; }
    if (ix < 0x4002d97c) {
        double z;
        if (hx > 0) {
            z = x - pio2_1;
            if (ix != 0x3ff921fb) { y[0] = z - pio2_1t; y[1] = (z - y[0]) - pio2_1t; }
            else { z -= pio2_2; y[0] = z - pio2_2t; y[1] = (z - y[0]) - pio2_2t; }
            return 1;
        }
        z = x + pio2_1;
        if (ix != 0x3ff921fb) { y[0] = z + pio2_1t; y[1] = (z - y[0]) + pio2_1t; }
        else { z += pio2_2; y[0] = z + pio2_2t; y[1] = (z - y[0]) + pio2_2t; }
        return -1;
    }
    if (ix <= 0x413921fb) {
        double t = fabs(x);
        int32_t n = (int32_t)(t * invpio2 + 0.5);
        double fn = (double)n;
        double r = t - fn * pio2_1;
        double w = fn * pio2_1t;
        int32_t j = (int32_t)(ix >> 20);
        y[0] = r - w;
        int32_t i = j - (int32_t)((hiw(y[0]) >> 20) & 0x7ff);
        if (i > 16) {
            t = r; w = fn * pio2_2; r = t - w; w = fn * pio2_2t - ((t - r) - w); y[0] = r - w;
            i = j - (int32_t)((hiw(y[0]) >> 20) & 0x7ff);
            if (i > 49) { t = r; w = fn * pio2_3; r = t - w; w = fn * pio2_3t - ((t - r) - w); y[0] = r - w; }
        }
        y[1] = (r - y[0]) - w;
        if (hx < 0) { y[0] = -y[0]; y[1] = -y[1]; return -n; }
        return n;
    }
    return GFPL_REM_FAIL;
}

GFPL_DEV double det_sin(double x) {
    double y[2];
    uint32_t ix = hiw(x) & 0x7fffffff;
    if (ix <= 0x3fe921fb) return k_sin(x, 0.0, 0);
    if (ix >= 0x7ff00000) return x - x;
    int n = rem_pio2(x, y);
    if (n == GFPL_REM_FAIL) return __builtin_nan("");
    switch (n & 3) {
        case 0: return k_sin(y[0], y[1], 1);
        case 1: return k_cos(y[0], y[1]);
        case 2: return -k_sin(y[0], y[1], 1);
        default: return -k_cos(y[0], y[1]);
    }
}

GFPL_DEV double det_cos(double x) {
    double y[2];
    uint32_t ix = hiw(x) & 0x7fffffff;
    if (ix <= 0x3fe921fb) return k_cos(x, 0.0);
    if (ix >= 0x7ff00000) return x - x;
    int n = rem_pio2(x, y);
    if (n == GFPL_REM_FAIL) return __builtin_nan("");
    switch (n & 3) {
        case 0: return k_cos(y[0], y[1]);
        case 1: return -k_sin(y[0], y[1], 1);
        case 2: return -k_cos(y[0], y[1]);
        default: return k_sin(y[0], y[1], 1);
    }
}

GFPL_DEV double ref_max(double a, double b) { return (a < b) ? b : a; }

// ------------------------------------------------------------- Hamming
// OpenCV normHamming, cellSize 1 (NORM_HAMMING) or 2 (NORM_HAMMING2), on
// 8 dwords.  v_bcnt_u32 is exact, so this equals the SWAR form of
// include/stereoFrame.h:185-201.
template <int CELL>
GFPL_DEV int hamming8(const uint32_t* a, const uint32_t* b) {
    int d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t v = a[i] ^ b[i];
        if (CELL == 2) v = (v | (v >> 1)) & 0x55555555u;
        d += __builtin_popcount(v);
    }
    return d;
}

GFPL_DEV void load_desc(const uint8_t* p, uint32_t* d) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
    d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

// ---------------------------------------------------------- small linalg
// Row-major, inner products k-sequential (pin N2) — same association as the oracle.
GFPL_DEV void mat4_mul(const double* A, const double* B, double* C) {
    double T[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            T[i * 4 + j] = ((A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j]) + A[i * 4 + 2] * B[2 * 4 + j]) + A[i * 4 + 3] * B[3 * 4 + j];
#pragma unroll
    for (int i = 0; i < 16; ++i) C[i] = T[i];
}

GFPL_DEV void mat4_inv(const double* m, double* out) {
    double a0 = m[0] * m[5] - m[1] * m[4];
    double a1 = m[0] * m[6] - m[2] * m[4];
    double a2 = m[0] * m[7] - m[3] * m[4];
    double a3 = m[1] * m[6] - m[2] * m[5];
    double a4 = m[1] * m[7] - m[3] * m[5];
    double a5 = m[2] * m[7] - m[3] * m[6];
    double b0 = m[8] * m[13] - m[9] * m[12];
    double b1 = m[8] * m[14] - m[10] * m[12];
    double b2 = m[8] * m[15] - m[11] * m[12];
    double b3 = m[9] * m[14] - m[10] * m[13];
    double b4 = m[9] * m[15] - m[11] * m[13];
    double b5 = m[10] * m[15] - m[11] * m[14];
    double det = ((((a0 * b5 - a1 * b4) + a2 * b3) + a3 * b2) - a4 * b1) + a5 * b0;
    double inv[16];
    inv[0]  = (m[5] * b5 - m[6] * b4) + m[7] * b3;
    inv[1]  = (-(m[1] * b5) + m[2] * b4) - m[3] * b3;
    inv[2]  = (m[13] * a5 - m[14] * a4) + m[15] * a3;
    inv[3]  = (-(m[9] * a5) + m[10] * a4) - m[11] * a3;
    inv[4]  = (-(m[4] * b5) + m[6] * b2) - m[7] * b1;
    inv[5]  = (m[0] * b5 - m[2] * b2) + m[3] * b1;
    inv[6]  = (-(m[12] * a5) + m[14] * a2) - m[15] * a1;
    inv[7]  = (m[8] * a5 - m[10] * a2) + m[11] * a1;
    inv[8]  = (m[4] * b4 - m[5] * b2) + m[7] * b0;
    inv[9]  = (-(m[0] * b4) + m[1] * b2) - m[3] * b0;
    inv[10] = (m[12] * a4 - m[13] * a2) + m[15] * a0;
    inv[11] = (-(m[8] * a4) + m[9] * a2) - m[11] * a0;
    inv[12] = (-(m[4] * b3) + m[5] * b1) - m[6] * b0;
    inv[13] = (m[0] * b3 - m[1] * b1) + m[2] * b0;
    inv[14] = (-(m[12] * a3) + m[13] * a1) - m[14] * a0;
    inv[15] = (m[8] * a3 - m[9] * a1) + m[10] * a0;
    double invdet = 1.0 / det;
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * invdet;
}

GFPL_DEV void mat4_vec(const double* M, const double* v, double* o) {
    double t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) t[i] = ((M[i * 4 + 0] * v[0] + M[i * 4 + 1] * v[1]) + M[i * 4 + 2] * v[2]) + M[i * 4 + 3] * v[3];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = t[i];
}

// ---- running error bounds (Wilkinson's running error analysis, used by the line cut's
// certification).  An RB stands for a double the kernel computes from exact
// inputs: m bounds |computed| and |exact| (the value of the same expression in real
// arithmetic on the same inputs), e bounds |computed - exact|, lo (when known, else 0) bounds
// min(|computed|, |exact|) from below — needed only for divisors.  The inputs of a range of
// calls (a cut ratio c in [0, C]) enter with m = C, so the bounds hold for every c of the range.
// The same templated code runs on double (the kernel's arithmetic) and on RB (its bounds), so
// the bounds follow the kernel's expression trees exactly.  Every rounding costs u = 2^-53 of
// the result's magnitude; the bound arithmetic itself is rounded, which the callers absorb in a
// final relative slop factor.
struct RB {
    double m, e, lo;
    GFPL_DEV RB() : m(0.0), e(0.0), lo(0.0) {}
    GFPL_DEV RB(double x) : m(fabs(x)), e(0.0), lo(fabs(x)) {}
    GFPL_DEV RB(double m_, double e_, double lo_) : m(m_), e(e_), lo(lo_) {}
};
constexpr double RB_U = 0x1p-53;
GFPL_DEV RB operator+(const RB& a, const RB& b) {
    const double m = a.m + b.m;
    return RB(m * (1.0 + 4.0 * RB_U), a.e + b.e + RB_U * m, 0.0);
}
GFPL_DEV RB operator-(const RB& a, const RB& b) { return a + b; }
GFPL_DEV RB operator-(const RB& a) { return a; }
GFPL_DEV RB operator*(const RB& a, const RB& b) {
    const double m = a.m * b.m;
    return RB(m * (1.0 + 4.0 * RB_U), a.e * b.m + a.m * b.e + RB_U * m, a.lo * b.lo * (1.0 - 4.0 * RB_U));
}
GFPL_DEV RB operator/(const RB& a, const RB& b) {
    if (!(b.lo > 0.0)) return RB(__builtin_inf(), __builtin_inf(), 0.0);
    const double m = a.m / b.lo;
    return RB(m * (1.0 + 4.0 * RB_U), a.e / b.lo + (a.m / b.lo) * (b.e / b.lo) + RB_U * m,
              (a.lo / b.m) * (1.0 - 4.0 * RB_U));
}
// max is 1-Lipschitz: |max(h, x^) - max(h, x*)| <= |x^ - x*|
GFPL_DEV RB ref_max(double h, const RB& x) {
    const double ah = fabs(h);
    return RB(ah > x.m ? ah : x.m, x.e, ah > x.lo ? ah : x.lo);
}
// a divisor's known lower bound (the exact value's, lo_exact), applied to the computed one
GFPL_DEV void rb_floor(double&, double) {}
GFPL_DEV void rb_floor(RB& z, double lo_exact) {
    const double l = lo_exact - z.e;
    if (l > z.lo) z.lo = l;
}

template <typename T, typename M>
GFPL_DEV void se3_apply_t(const M* Tm, const T* P, T* o) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
        o[i] = ((T(Tm[i * 4 + 0]) * P[0] + T(Tm[i * 4 + 1]) * P[1]) + T(Tm[i * 4 + 2]) * P[2]) + T(Tm[i * 4 + 3]);
}
GFPL_DEV void se3_apply(const double* T, const double* P, double* o) { se3_apply_t<double, double>(T, P, o); }

GFPL_DEV void skew3(const double* v, double* S) {
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}

GFPL_DEV void mat3_mul(const double* A, const double* B, double* C) {
    double T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) + A[i * 3 + 2] * B[2 * 3 + j];
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}

GFPL_DEV void inverse_se3(const double* T, double* out) {
    double o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) o[i * 4 + j] = T[j * 4 + i];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        o[i * 4 + 3] = ((-T[0 * 4 + i]) * T[3] + (-T[1 * 4 + i]) * T[7]) + (-T[2 * 4 + i]) * T[11];
    o[15] = 1.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = o[i];
}

GFPL_DEV void expmap_se3(const double* x, double* T) {
    double w[3] = {x[3], x[4], x[5]}, t[3] = {x[0], x[1], x[2]};
    double theta = sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (!(theta < 0.000001)) {
        double s[9], ss[9];
        skew3(w, s);
#pragma unroll
        for (int i = 0; i < 9; ++i) s[i] = s[i] / theta;
        mat3_mul(s, s, ss);
        double st = det_sin(theta), ct = det_cos(theta);
        double omc = 1.0 - ct;
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = (I[i] + s[i] * st) + ss[i] * omc;
        double V[9];
        double tms = theta - st;
#pragma unroll
        for (int i = 0; i < 9; ++i) V[i] = (I[i] + (s[i] * omc) / theta) + (ss[i] * tms) / theta;
        double tt[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) tt[i] = (V[i * 3 + 0] * t[0] + V[i * 3 + 1] * t[1]) + V[i * 3 + 2] * t[2];
        t[0] = tt[0]; t[1] = tt[1]; t[2] = tt[2];
    }
    T[0] = R[0]; T[1] = R[1]; T[2] = R[2]; T[3] = t[0];
    T[4] = R[3]; T[5] = R[4]; T[6] = R[5]; T[7] = t[1];
    T[8] = R[6]; T[9] = R[7]; T[10] = R[8]; T[11] = t[2];
    T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}

// logdet (include/linespec.h:43-56) on a 6x6 given by its lower triangle
// L21[i*(i+1)/2 + j] (j <= i); ledger Q11 failure semantics.
GFPL_DEV int tri(int i, int j) { return i * (i + 1) / 2 + j; }

GFPL_DEV double logdet6_lower(double* a /* 21, destroyed */) {
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        double x = a[tri(k, k)];
#pragma unroll
        for (int j = 0; j < k; ++j) x = x - a[tri(k, j)] * a[tri(k, j)];
        if (x <= 0.0) break;
        x = sqrt(x);
        a[tri(k, k)] = x;
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            double v = a[tri(i, k)];
#pragma unroll
            for (int j = 0; j < k; ++j) v = v - a[tri(i, j)] * a[tri(k, j)];
            a[tri(i, k)] = v / x;
        }
    }
    double s = det_log(a[tri(0, 0)]);
#pragma unroll
    for (int i = 1; i < 6; ++i) s = s + det_log(a[tri(i, i)]);
    return 2.0 * s;
}

// The three small dense solvers below keep every matrix in registers: loops
// are fully unrolled and pivot swaps are applied through compile-time-indexed
// selects, so no runtime-indexed array spills to scratch.  The arithmetic is
// the oracle's, operation for operation (pivot choice, swap, update order).
template <typename T>
GFPL_DEV void swap_v(T& a, T& b) { T t = a; a = b; b = t; }

// LDLT solve, Eigen 3.3 semantics (see oracle ldlt_solve6).  ONE LANE only (k_pose's lane 0):
// each pivot index is made wave-uniform (readfirstlane), so a pivot swap is one scalar branch
// to the block of moves for that index instead of selects over every candidate index.
GFPL_DEV void ldlt_solve6_one_lane(const double* H, const double* g, double* x) {
    double m[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) m[i] = H[i];
    int tr[6];
    double temp[6];
    bool stop = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        if (stop) { tr[k] = k; continue; }
        int big = k;
        double bv = fabs(m[k * 7]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double v = fabs(m[i * 7]);
            if (v > bv) { bv = v; big = i; }
        }
        big = __builtin_amdgcn_readfirstlane(big);
        tr[k] = big;
#pragma unroll
        for (int c = k + 1; c < 6; ++c) {
            if (big == c) {
#pragma unroll
                for (int j = 0; j < k; ++j) swap_v(m[k * 6 + j], m[c * 6 + j]);
#pragma unroll
                for (int i = c + 1; i < 6; ++i) swap_v(m[i * 6 + k], m[i * 6 + c]);
                swap_v(m[k * 7], m[c * 7]);
#pragma unroll
                for (int i = k + 1; i < c; ++i) {
                    const double tmp = m[i * 6 + k];
                    m[i * 6 + k] = m[c * 6 + i];
                    m[c * 6 + i] = tmp;
                }
            }
        }
        if (k > 0) {
#pragma unroll
            for (int j = 0; j < k; ++j) temp[j] = m[j * 7] * m[k * 6 + j];
            double dot = m[k * 6 + 0] * temp[0];
#pragma unroll
            for (int j = 1; j < k; ++j) dot = dot + m[k * 6 + j] * temp[j];
            m[k * 7] = m[k * 7] - dot;
#pragma unroll
            for (int i = k + 1; i < 6; ++i) {
                double v = m[i * 6 + k];
#pragma unroll
                for (int j = 0; j < k; ++j) v = v - m[i * 6 + j] * temp[j];
                m[i * 6 + k] = v;
            }
        }
        const double akk = m[k * 7];
        const bool valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            tr[0] = 0;
            stop = true;
            continue;
        }
        if (k < 5 && valid) {
#pragma unroll
            for (int i = k + 1; i < 6; ++i) m[i * 6 + k] = m[i * 6 + k] / akk;
        }
    }
    double d[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) d[i] = g[i];
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int c = k + 1; c < 6; ++c)
            if (tr[k] == c) swap_v(d[k], d[c]);
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < i; ++j) d[i] = d[i] - m[i * 6 + j] * d[j];
    const double tol = 1.0 / 1.7976931348623157e308;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double di = m[i * 7];
        if (fabs(di) > tol) d[i] = d[i] / di; else d[i] = 0.0;
    }
#pragma unroll
    for (int i = 5; i >= 0; --i)
#pragma unroll
        for (int j = i + 1; j < 6; ++j) d[i] = d[i] - m[j * 6 + i] * d[j];
#pragma unroll
    for (int k = 5; k >= 0; --k)
#pragma unroll
        for (int c = k + 1; c < 6; ++c)
            if (tr[k] == c) swap_v(d[k], d[c]);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = d[i];
}

// PartialPivLU inverse (see oracle inverse6)
GFPL_DEV void inverse6(const double* A, double* out) {
    double m[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) m[i] = A[i];
    int perm[6] = {0, 1, 2, 3, 4, 5};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double pv = fabs(m[k * 6 + k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double v = fabs(m[i * 6 + k]);
            if (v > pv) { pv = v; p = i; }
        }
#pragma unroll
        for (int c = k + 1; c < 6; ++c) {
            if (p == c) {
#pragma unroll
                for (int j = 0; j < 6; ++j) swap_v(m[k * 6 + j], m[c * 6 + j]);
                swap_v(perm[k], perm[c]);
            }
        }
        const double piv = m[k * 6 + k];
        if (piv != 0.0) {
#pragma unroll
            for (int i = k + 1; i < 6; ++i) m[i * 6 + k] = m[i * 6 + k] / piv;
        }
#pragma unroll
        for (int i = k + 1; i < 6; ++i)
#pragma unroll
            for (int j = k + 1; j < 6; ++j) m[i * 6 + j] = m[i * 6 + j] - m[i * 6 + k] * m[k * 6 + j];
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        double x[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) x[i] = (perm[i] == c) ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) x[i] = x[i] - m[i * 6 + j] * x[j];
#pragma unroll
        for (int i = 5; i >= 0; --i) {
#pragma unroll
            for (int j = i + 1; j < 6; ++j) x[i] = x[i] - m[i * 6 + j] * x[j];
            x[i] = x[i] / m[i * 6 + i];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) out[i * 6 + c] = x[i];
    }
}

// adjoint_se3 (src/auxiliar.cpp:216-223): [R, skew(t) R; 0, R] (see oracle)
GFPL_DEV void adjoint_se3(const double* T, double* Ad) {
    double R[9], t[3] = {T[3], T[7], T[11]}, Sk[9], SR[9];
#pragma unroll
    for (int i = 0; i < 36; ++i) Ad[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = T[i * 4 + j];
    skew3(t, Sk);
    mat3_mul(Sk, R, SR);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            Ad[i * 6 + j] = R[i * 3 + j];
            Ad[i * 6 + 3 + j] = SR[i * 3 + j];
            Ad[(3 + i) * 6 + 3 + j] = R[i * 3 + j];
        }
}

// [C +] A X A^T for 6x6, A*X first, inner products k-sequential (see oracle sandwich6)
GFPL_DEV void sandwich6(const double* A, const double* X, const double* C, double* out) {
    double AS[36];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double s = A[i * 6 + 0] * X[0 * 6 + j];
#pragma unroll
            for (int k = 1; k < 6; ++k) s = s + A[i * 6 + k] * X[k * 6 + j];
            AS[i * 6 + j] = s;
        }
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double s = AS[i * 6 + 0] * A[j * 6 + 0];
#pragma unroll
            for (int k = 1; k < 6; ++k) s = s + AS[i * 6 + k] * A[j * 6 + k];
            out[i * 6 + j] = C ? C[i * 6 + j] + s : s;
        }
}

// Matrix6d::determinant: PartialPivLU, diagonal product left to right (see oracle det6)
GFPL_DEV double det6(const double* A) {
    double m[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) m[i] = A[i];
    int ntr = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double pv = fabs(m[k * 6 + k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double v = fabs(m[i * 6 + k]);
            if (v > pv) { pv = v; p = i; }
        }
#pragma unroll
        for (int c = k + 1; c < 6; ++c) {
            if (p == c) {
#pragma unroll
                for (int j = 0; j < 6; ++j) swap_v(m[k * 6 + j], m[c * 6 + j]);
                ++ntr;
            }
        }
        const double piv = m[k * 6 + k];
        if (piv != 0.0) {
#pragma unroll
            for (int i = k + 1; i < 6; ++i) m[i * 6 + k] = m[i * 6 + k] / piv;
        }
#pragma unroll
        for (int i = k + 1; i < 6; ++i)
#pragma unroll
            for (int j = k + 1; j < 6; ++j) m[i * 6 + j] = m[i * 6 + j] - m[i * 6 + k] * m[k * 6 + j];
    }
    double d = m[0];
#pragma unroll
    for (int i = 1; i < 6; ++i) d = d * m[i * 7];
    return (ntr & 1) ? -1.0 * d : 1.0 * d;
}

// entropy of a 6-dof Gaussian as needNewKF writes it (src/stereoFrameHandler.cpp:2315,2329)
GFPL_DEV double kf_entropy(const double* cov) {
    const double c0 = 3.0 * (1.0 + det_log(2.0 * 3.141592653589793));   // acos(-1) = pi
    return c0 + 0.5 * det_log(det6(cov));
}

// SelfAdjointEigenSolver eigenvalues -> cyclic Jacobi, ascending (see oracle eig_sym)
template <int N>
GFPL_DEV void eig_sym(const double* A, double* w) {
    double a[N * N];
#pragma unroll
    for (int i = 0; i < N * N; ++i) a[i] = A[i];
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0;
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) off = off + a[p * N + q] * a[p * N + q];
        if (!(off > 0.0)) break;
        {   // (early exit with the oracle's bits) once the off-diagonal mass is below an eighth of the
            // smallest gap under a diagonal entry, no later rotation moves a diagonal entry: each moves
            // app, aqq by t apq with |t| <= 1, the rotations keep the off-diagonal Frobenius norm (up to
            // rounding far inside the factor 8), and app -+ (less than half that gap) rounds to app.
            // Finite diagonals only (the oracle's NaN / Inf rotations spread).
            double thr = __builtin_inf();
            bool fin = true;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int e = (int)((__double_as_longlong(a[i * N + i]) >> 52) & 0x7FF);
                fin = fin && e != 0x7FF;
                // (2^(e - 1076) / 8)^2: 2^(e - 1076) is the gap below |a_ii| (0 for zero / subnormal)
                thr = fmin(thr, e == 0 ? 0.0 : ldexp(1.0, 2 * (e - 1076) - 6));
            }
            if (fin && off < thr) break;
        }
#pragma unroll
        for (int p = 0; p < N - 1; ++p)
#pragma unroll
            for (int q = p + 1; q < N; ++q) {
                const double apq = a[p * N + q];
                if (apq != 0.0) {
                    const double app = a[p * N + p], aqq = a[q * N + q];
                    const double theta = (aqq - app) / (2.0 * apq);
                    // the oracle's expressions, with two shortcuts that give their bits (the late
                    // sweeps' rotations are almost all in them): for 2^27 <= |theta| <= 1e150,
                    // theta^2 + 1 rounds to theta^2, whose correctly rounded sqrt is |theta|, so
                    // 1 / (|theta| + sqrt(.)) is 1 / (2 |theta|) = 0.5 / |theta|; and t^2 + 1 == 1
                    // makes c = 1 / sqrt(1) = 1, s = t (tests/test_oracle_known_answers.py checks both)
                    double t;
                    const double ath = fabs(theta);
                    if (ath > 1e150) t = 0.5 / theta;
                    else {
                        t = ath >= 0x1p27 ? 0.5 / ath : 1.0 / (ath + sqrt(theta * theta + 1.0));
                        if (theta < 0.0) t = -t;
                    }
                    const double tt1 = t * t + 1.0;
                    const double c = tt1 == 1.0 ? 1.0 : 1.0 / sqrt(tt1);
                    const double s = t * c;
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        if (k == p || k == q) continue;
                        const double akp = a[k * N + p], akq = a[k * N + q];
                        const double nkp = c * akp - s * akq;
                        const double nkq = s * akp + c * akq;
                        a[k * N + p] = nkp; a[p * N + k] = nkp;
                        a[k * N + q] = nkq; a[q * N + k] = nkq;
                    }
                    a[p * N + p] = app - t * apq;
                    a[q * N + q] = aqq + t * apq;
                    a[p * N + q] = 0.0; a[q * N + p] = 0.0;
                }
            }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) w[i] = a[i * N + i];
    // insertion sort, unrolled with a "still moving" flag (same result as the oracle's)
#pragma unroll
    for (int i = 1; i < N; ++i) {
        const double v = w[i];
        bool moving = true;
#pragma unroll
        for (int j = i - 1; j >= 0; --j) {
            if (moving) {
                if (w[j] > v) w[j + 1] = w[j];
                else { w[j + 1] = v; moving = false; }
            }
        }
        if (moving) w[0] = v;
    }
}

// ------------------------------------------------------------- camera
struct DevCam {
    double fx, fy, cx, cy, b;
    int width, height, n_levels;
    float scale[GFPL_MAX_LEVELS], inv_scale[GFPL_MAX_LEVELS];
    int lvl_cols[GFPL_MAX_LEVELS], lvl_rows[GFPL_MAX_LEVELS];
    long long lvl_offset[GFPL_MAX_LEVELS];
    long long pyr_bytes;
    double sigma2_pt[GFPL_MAX_LEVELS], sigma2_ln[GFPL_MAX_LEVELS];
};

GFPL_DEV void projection(const DevCam& c, const double* P, double* uv) {
    uv[0] = c.cx + (c.fx * P[0]) / P[2];
    uv[1] = c.cy + (c.fy * P[1]) / P[2];
}
GFPL_DEV void backProjection(const DevCam& c, double u, double v, double disp, double* P) {
    double bd = c.b / disp;
    P[0] = bd * (u - c.cx);
    P[1] = bd * (v - c.cy);
    P[2] = bd * c.fx;
}

// f64 a / b exactly as clang expands it for gfx950 (v_div_scale of the denominator, v_rcp and
// two Newton steps, v_div_scale of the numerator, one correction, v_div_fmas, v_div_fixup),
// with the reciprocal refinement of a denominator shared by the numerators divided by it: the
// scaled denominator v_div_scale(b, b, a) can depend on a (a = 0, a tiny, |a / b| extreme), so
// each division forms it and refines its own reciprocal unless its bits equal the shared one's —
// every quotient is the bits of `a / b` (the refinement is a function of the scaled denominator)
struct SharedDiv { double b, sb, r; };
GFPL_DEV double div_refine(double sb) {
    double r = __builtin_amdgcn_rcp(sb);
    double t = __builtin_fma(-sb, r, 1.0);
    r = __builtin_fma(r, t, r);
    t = __builtin_fma(-sb, r, 1.0);
    return __builtin_fma(r, t, r);
}
GFPL_DEV SharedDiv div_prep(double b, double a0) {
    bool f;
    const double sb = __builtin_amdgcn_div_scale(a0, b, false, &f);
    return SharedDiv{b, sb, div_refine(sb)};
}
GFPL_DEV double div_by(const SharedDiv& d, double a) {
    bool f, vcc;
    const double sb = __builtin_amdgcn_div_scale(a, d.b, false, &f);
    double r = d.r;
    if (__builtin_expect(__double_as_longlong(sb) != __double_as_longlong(d.sb), 0)) r = div_refine(sb);
    const double sa = __builtin_amdgcn_div_scale(a, d.b, true, &vcc);
    const double m = sa * r;
    const double e = __builtin_fma(-sb, m, sa);
    return __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(e, r, m, vcc), d.b, a);
}
// Jacobian of a projected residual wrt the pose, weights (lx, ly)
// (src/stereoFrameHandler.cpp:1383-1388, 1438-1443, 2150-2155, 2197-2202)
template <typename T>
GFPL_DEV void poseJac_t(const DevCam& c, double homog, const T* g, T lx, T ly, T* J) {
    T gx = g[0], gy = g[1], gz = g[2];
    T gz2 = gz * gz;
    T fgz2 = T(c.fx) / ref_max(homog, gz2);
    J[0] = (fgz2 * lx) * gz;
    J[1] = (fgz2 * ly) * gz;
    J[2] = (-fgz2) * ((gx * lx) + (gy * ly));
    J[3] = (-fgz2) * ((((gx * gy) * lx) + ((gy * gy) * ly)) + ((gz * gz) * ly));
    J[4] = fgz2 * ((((gx * gx) * lx) + ((gz * gz) * lx)) + ((gx * gy) * ly));
    J[5] = fgz2 * (((gx * gz) * ly) - ((gy * gz) * lx));
}
GFPL_DEV void poseJac(const DevCam& c, double homog, const double* g, double lx, double ly, double* J) {
    poseJac_t<double>(c, homog, g, lx, ly, J);
}

// endpoint 3x3 covariance of the stereo line gate (src/stereoFrame.cpp:707-742)
GFPL_DEV void endpointCov(const DevCam& cam, double u, double v, double disp, double* C) {
    double f = cam.fx;
    double px = u - cam.cx, py = v - cam.cy;
    double d2 = disp * disp;
    C[0] = d2 + (2.0 * px) * px;
    C[1] = (2.0 * px) * py;
    C[2] = (2.0 * f) * px;
    C[4] = d2 + (2.0 * py) * py;
    C[5] = (2.0 * f) * py;
    C[8] = (2.0 * f) * f;
    C[3] = C[1]; C[6] = C[2]; C[7] = C[5];
    double dd = d2 * d2;
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = ((C[i] * cam.b) * cam.b) / dd;
}

// getCovMat2D_3D (src/stereoFrame.cpp:1434-1446), ledger U2 (off-diagonals 0)
GFPL_DEV void covMat2D_3D(const DevCam& cam, double u, double v, double u_std, double d, double d_std, double* cov) {
    double cov2D[9] = {u_std * u_std, 0, 0, 0, u_std * u_std, 0, 0, 0, d_std * d_std};
    double b = cam.b, d_2 = d * d;
    double J[9];
    J[0] = b / d; J[3] = 0.0; J[6] = 0.0;
    J[1] = 0.0; J[4] = b / d; J[7] = 0.0;
    J[2] = ((-(u - cam.cx)) * b) / d_2;
    J[5] = ((-(v - cam.cy)) * b) / d_2;
    J[8] = ((-cam.fx) * b) / d_2;
    double JC[9];
    mat3_mul(J, cov2D, JC);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            cov[i * 3 + j] = (JC[i * 3 + 0] * J[j * 3 + 0] + JC[i * 3 + 1] * J[j * 3 + 1]) + JC[i * 3 + 2] * J[j * 3 + 2];
}

// lineSegmentOverlapStereo (src/stereoFrame.cpp:1343-1371)
GFPL_DEV double std_min(double a, double b) { return (b < a) ? b : a; }
GFPL_DEV double std_max(double a, double b) { return (a < b) ? b : a; }
GFPL_DEV double overlapStereo(double spl_obs, double epl_obs, double spl_proj, double epl_proj) {
    double sln = std_min(spl_obs, epl_obs);
    double eln = std_max(spl_obs, epl_obs);
    double spn = std_min(spl_proj, epl_proj);
    double epn = std_max(spl_proj, epl_proj);
    double length = eln - spn;
    double overlap;
    if ((epn < sln) || (spn > eln)) overlap = 0.0;
    else {
        if ((epn > eln) && (spn < sln)) overlap = eln - sln;
        else overlap = std_min(eln, epn) - std_max(sln, spn);
    }
    if (length > 0.01f) overlap = overlap / length;
    else overlap = 0.0;
    return overlap;
}

// --------------------------------------------------------- block helpers
// exclusive prefix sum of one int per thread over the block (blockDim <= 1024)
// The value at rank r (0-based) of a histogram h[0 .. nb) of small integers (nb <= 320): the first v
// with h[0] + ... + h[v] > r, or nb - 1 when the total is <= r — called by a whole wave, the result in
// every lane.  Five bins per lane, a wave prefix sum, the crossing lane scans its bins: one LDS read
// per lane instead of a one-thread loop of nb dependent reads (round 6).
__device__ __forceinline__ int wave_hist_rank(const int* h, int r, int nb) {
    const int lane = threadIdx.x & 63;
    int loc[5], sum = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const int v = lane * 5 + i;
        loc[i] = v < nb ? h[v] : 0;
        sum += loc[i];
    }
    int inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    int res = 0x7FFFFFFF;
    if (inc - sum <= r && r < inc) {
        int c = inc - sum;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            c += loc[i];
            if (c > r && res == 0x7FFFFFFF) res = lane * 5 + i;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) res = min(res, __shfl_xor(res, o, 64));
    return res == 0x7FFFFFFF ? nb - 1 : res;
}

template <int BLOCK>
GFPL_DEV int block_exclusive_scan(int v, int* lds /* >= BLOCK/64 + 1 ints */, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int w = 0; w < BLOCK / 64; ++w) { int t = lds[w]; lds[w] = s; s += t; }
        lds[BLOCK / 64] = s;
    }
    __syncthreads();
    int r = x - v + lds[wid];
    *total = lds[BLOCK / 64];
    __syncthreads();
    return r;
}

}  // namespace gfpl
