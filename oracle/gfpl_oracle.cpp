// gfpl_oracle.cpp — CPU ORACLE (test infrastructure only; see gfpl_oracle.h).
//
// Plain C++ restatement of the GF-PL-SLAM per-frame tracking path.  Reference
// citations are `file:line` into SimonsRoad/gf-pl-slam.  Build with
// -ffp-contract=off (oracle/Makefile): pin N1.
#include "gfpl_oracle.h"

#include <algorithm>
#include <array>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace {

// ===================================================================== N3 ==
// fdlibm algorithms restated with + - * / only (pin N3).
// The log / sin / cos below restate the algorithms and coefficient tables of Sun fdlibm
// (e_log.c, k_sin.c, k_cos.c, e_rem_pio2.c), whose notice is preserved here:
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this software is freely granted,
//   provided that this notice is preserved.
inline uint32_t hi_word(double x) { uint64_t u; std::memcpy(&u, &x, 8); return (uint32_t)(u >> 32); }
inline uint32_t lo_word(double x) { uint64_t u; std::memcpy(&u, &x, 8); return (uint32_t)u; }
inline double with_hi(double x, uint32_t hi) {
    uint64_t u; std::memcpy(&u, &x, 8);
    u = ((uint64_t)hi << 32) | (u & 0xffffffffull);
    std::memcpy(&x, &u, 8); return x;
}
inline double from_words(uint32_t hi, uint32_t lo) {
    uint64_t u = ((uint64_t)hi << 32) | lo; double x; std::memcpy(&x, &u, 8); return x;
}

// e_log.c
double det_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16,
                 Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    int32_t hx = (int32_t)hi_word(x);
    uint32_t lx = lo_word(x);
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -INFINITY;
        if (hx < 0) return NAN;
        k -= 54; x *= two54;
        hx = (int32_t)hi_word(x);
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

// k_sin.c
double k_sin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    uint32_t ix = hi_word(x) & 0x7fffffff;
    if (ix < 0x3e400000) { if ((int)x == 0) return x; }
    double z = x * x;
    double v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

// k_cos.c
double k_cos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    uint32_t ix = hi_word(x) & 0x7fffffff;
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

// e_rem_pio2.c, |x| <= 2^19*(pi/2) branches; returns INT_MIN beyond (NaN result).
int rem_pio2(double x, double* y) {
    const double invpio2 = 6.36619772367581382433e-01,
                 pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11,
                 pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21,
                 pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    int32_t hx = (int32_t)hi_word(x);
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
        double t = std::fabs(x);
        int32_t n = (int32_t)(t * invpio2 + 0.5);
        double fn = (double)n;
        double r = t - fn * pio2_1;
        double w = fn * pio2_1t;
        int32_t j = (int32_t)(ix >> 20);
        y[0] = r - w;
        int32_t i = j - (int32_t)((hi_word(y[0]) >> 20) & 0x7ff);
        if (i > 16) {
            t = r; w = fn * pio2_2; r = t - w; w = fn * pio2_2t - ((t - r) - w); y[0] = r - w;
            i = j - (int32_t)((hi_word(y[0]) >> 20) & 0x7ff);
            if (i > 49) { t = r; w = fn * pio2_3; r = t - w; w = fn * pio2_3t - ((t - r) - w); y[0] = r - w; }
        }
        y[1] = (r - y[0]) - w;
        if (hx < 0) { y[0] = -y[0]; y[1] = -y[1]; return -n; }
        return n;
    }
    return INT_MIN;
}

double det_sin(double x) {
    double y[2];
    uint32_t ix = hi_word(x) & 0x7fffffff;
    if (ix <= 0x3fe921fb) return k_sin(x, 0.0, 0);
    if (ix >= 0x7ff00000) return x - x;
    int n = rem_pio2(x, y);
    if (n == INT_MIN) return NAN;
    switch (n & 3) {
        case 0: return k_sin(y[0], y[1], 1);
        case 1: return k_cos(y[0], y[1]);
        case 2: return -k_sin(y[0], y[1], 1);
        default: return -k_cos(y[0], y[1]);
    }
}

double det_cos(double x) {
    double y[2];
    uint32_t ix = hi_word(x) & 0x7fffffff;
    if (ix <= 0x3fe921fb) return k_cos(x, 0.0);
    if (ix >= 0x7ff00000) return x - x;
    int n = rem_pio2(x, y);
    if (n == INT_MIN) return NAN;
    switch (n & 3) {
        case 0: return k_cos(y[0], y[1]);
        case 1: return -k_sin(y[0], y[1], 1);
        case 2: return -k_cos(y[0], y[1]);
        default: return k_sin(y[0], y[1], 1);
    }
}

// std::max as the reference uses it: (a < b) ? b : a
inline double ref_max(double a, double b) { return (a < b) ? b : a; }
// ledger U11: the reference indexes its per-level tables (mvScaleFactors,
// mvInvScaleFactors, the sigma2 of PointFeature / LineFeature) with the keypoint
// octave unchecked — UB outside the pyramid; pinned (oracle and kernels) to the
// nearest level
inline int clampl(int o, int n) { return o < 0 ? 0 : (o >= n ? n - 1 : o); }

// ============================================================ small linalg ==
// Row-major fixed-size helpers; inner products k-sequential (pin N2).
void mat4_mul(const double* A, const double* B, double* C) {
    double T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            T[i * 4 + j] = ((A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j]) + A[i * 4 + 2] * B[2 * 4 + j]) + A[i * 4 + 3] * B[3 * 4 + j];
    std::memcpy(C, T, sizeof T);
}

// Matrix4d::inverse (src/stereoFrame.cpp:1560, src/stereoFrameHandler.cpp:1635):
// cofactor expansion through 2x2 minors (pin N4).
void mat4_inv(const double* m, double* out) {
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
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * invdet;
}

// 4x4 * (v0,v1,v2,v3)
void mat4_vec(const double* M, const double* v, double* o) {
    double t[4];
    for (int i = 0; i < 4; ++i) t[i] = ((M[i * 4 + 0] * v[0] + M[i * 4 + 1] * v[1]) + M[i * 4 + 2] * v[2]) + M[i * 4 + 3] * v[3];
    std::memcpy(o, t, sizeof t);
}

// R*P + t with R = T(0:3,0:3), t = T(0:3,3)   (src/stereoFrameHandler.cpp:2135,1357)
inline void se3_apply(const double* T, const double* P, double* o) {
    for (int i = 0; i < 3; ++i)
        o[i] = ((T[i * 4 + 0] * P[0] + T[i * 4 + 1] * P[1]) + T[i * 4 + 2] * P[2]) + T[i * 4 + 3];
}

// skew (src/auxiliar.cpp:248-262)
void skew3(const double* v, double* S) {
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
void mat3_mul(const double* A, const double* B, double* C) {
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) + A[i * 3 + 2] * B[2 * 3 + j];
    std::memcpy(C, T, sizeof T);
}

// inverse_se3 (src/auxiliar.cpp:154-163)
void inverse_se3(const double* T, double* out) {
    double o[16] = {0};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) o[i * 4 + j] = T[j * 4 + i];
    for (int i = 0; i < 3; ++i)
        o[i * 4 + 3] = ((-T[0 * 4 + i]) * T[3] + (-T[1 * 4 + i]) * T[7]) + (-T[2 * 4 + i]) * T[11];
    o[15] = 1.0;
    std::memcpy(out, o, sizeof o);
}

// expmap_se3 (src/auxiliar.cpp:165-182); x = [t; w]
void expmap_se3(const double* x, double* T) {
    double w[3] = {x[3], x[4], x[5]}, t[3] = {x[0], x[1], x[2]};
    double theta = std::sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (!(theta < 0.000001)) {
        double s[9], ss[9];
        skew3(w, s);
        for (int i = 0; i < 9; ++i) s[i] = s[i] / theta;
        mat3_mul(s, s, ss);
        double st = det_sin(theta), ct = det_cos(theta);
        double omc = 1.0 - ct;                       // (1.0f-cos(theta))
        double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        for (int i = 0; i < 9; ++i) R[i] = (I[i] + s[i] * st) + ss[i] * omc;
        double V[9];
        double tms = theta - st;
        for (int i = 0; i < 9; ++i) V[i] = (I[i] + (s[i] * omc) / theta) + (ss[i] * tms) / theta;
        double tt[3];
        for (int i = 0; i < 3; ++i) tt[i] = (V[i * 3 + 0] * t[0] + V[i * 3 + 1] * t[1]) + V[i * 3 + 2] * t[2];
        t[0] = tt[0]; t[1] = tt[1]; t[2] = tt[2];
    }
    double o[16] = {R[0], R[1], R[2], t[0], R[3], R[4], R[5], t[1], R[6], R[7], R[8], t[2], 0, 0, 0, 1};
    std::memcpy(T, o, sizeof o);
}

// logdet (include/linespec.h:43-56): LLT<MatrixXd> lower, unblocked path
// (size < 32), no failure check (ledger Q11): on a non-positive pivot at k the
// factorisation stops and diag entries k..5 keep their input values.
double logdet6(const double* M) {
    double a[36];
    std::memcpy(a, M, sizeof a);
    for (int k = 0; k < 6; ++k) {
        double x = a[k * 6 + k];
        for (int j = 0; j < k; ++j) x = x - a[k * 6 + j] * a[k * 6 + j];
        if (x <= 0.0) break;
        x = std::sqrt(x);
        a[k * 6 + k] = x;
        for (int i = k + 1; i < 6; ++i) {
            double v = a[i * 6 + k];
            for (int j = 0; j < k; ++j) v = v - a[i * 6 + j] * a[k * 6 + j];
            a[i * 6 + k] = v / x;
        }
    }
    double s = det_log(a[0]);
    for (int i = 1; i < 6; ++i) s = s + det_log(a[i * 6 + i]);
    return 2.0 * s;
}

// LDLT<Matrix6d>::solve (src/stereoFrameHandler.cpp:2045-2046): Eigen 3.3
// ldlt_inplace<Lower>::unblocked + _solve_impl (pin N4).
void ldlt_solve6(const double* H, const double* g, double* x) {
    double m[36];
    std::memcpy(m, H, sizeof m);
    int tr[6];
    double temp[6];
    for (int k = 0; k < 6; ++k) {
        int big = k;
        double bv = std::fabs(m[k * 6 + k]);
        for (int i = k + 1; i < 6; ++i) {
            double v = std::fabs(m[i * 6 + i]);
            if (v > bv) { bv = v; big = i; }
        }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; ++j) std::swap(m[k * 6 + j], m[big * 6 + j]);
            for (int i = big + 1; i < 6; ++i) std::swap(m[i * 6 + k], m[i * 6 + big]);
            std::swap(m[k * 6 + k], m[big * 6 + big]);
            for (int i = k + 1; i < big; ++i) {
                double tmp = m[i * 6 + k];
                m[i * 6 + k] = m[big * 6 + i];
                m[big * 6 + i] = tmp;
            }
        }
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = m[j * 6 + j] * m[k * 6 + j];
            double dot = m[k * 6 + 0] * temp[0];
            for (int j = 1; j < k; ++j) dot = dot + m[k * 6 + j] * temp[j];
            m[k * 6 + k] = m[k * 6 + k] - dot;
            for (int i = k + 1; i < 6; ++i) {
                double v = m[i * 6 + k];
                for (int j = 0; j < k; ++j) v = v - m[i * 6 + j] * temp[j];
                m[i * 6 + k] = v;
            }
        }
        double akk = m[k * 6 + k];
        bool valid = std::fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            for (int j = 0; j < 6; ++j) tr[j] = j;
            break;
        }
        if (k < 5 && valid)
            for (int i = k + 1; i < 6; ++i) m[i * 6 + k] = m[i * 6 + k] / akk;
    }
    double d[6];
    for (int i = 0; i < 6; ++i) d[i] = g[i];
    for (int k = 0; k < 6; ++k) std::swap(d[k], d[tr[k]]);
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < i; ++j) d[i] = d[i] - m[i * 6 + j] * d[j];
    const double tol = 1.0 / DBL_MAX;
    for (int i = 0; i < 6; ++i) {
        double di = m[i * 6 + i];
        if (std::fabs(di) > tol) d[i] = d[i] / di; else d[i] = 0.0;
    }
    for (int i = 5; i >= 0; --i)
        for (int j = i + 1; j < 6; ++j) d[i] = d[i] - m[j * 6 + i] * d[j];
    for (int k = 5; k >= 0; --k) std::swap(d[k], d[tr[k]]);
    std::memcpy(x, d, sizeof d);
}

// Matrix6d::inverse (src/stereoFrameHandler.cpp:2054): PartialPivLU (pin N4)
void inverse6(const double* A, double* out) {
    double m[36];
    std::memcpy(m, A, sizeof m);
    int perm[6] = {0, 1, 2, 3, 4, 5};
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double pv = std::fabs(m[k * 6 + k]);
        for (int i = k + 1; i < 6; ++i) {
            double v = std::fabs(m[i * 6 + k]);
            if (v > pv) { pv = v; p = i; }
        }
        if (p != k) {
            for (int j = 0; j < 6; ++j) std::swap(m[k * 6 + j], m[p * 6 + j]);
            std::swap(perm[k], perm[p]);
        }
        double piv = m[k * 6 + k];
        if (piv != 0.0)
            for (int i = k + 1; i < 6; ++i) m[i * 6 + k] = m[i * 6 + k] / piv;
        for (int i = k + 1; i < 6; ++i)
            for (int j = k + 1; j < 6; ++j) m[i * 6 + j] = m[i * 6 + j] - m[i * 6 + k] * m[k * 6 + j];
    }
    double inv[36];
    for (int c = 0; c < 6; ++c) {
        double x[6];
        for (int i = 0; i < 6; ++i) x[i] = (perm[i] == c) ? 1.0 : 0.0;
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < i; ++j) x[i] = x[i] - m[i * 6 + j] * x[j];
        for (int i = 5; i >= 0; --i) {
            for (int j = i + 1; j < 6; ++j) x[i] = x[i] - m[i * 6 + j] * x[j];
            x[i] = x[i] / m[i * 6 + i];
        }
        for (int i = 0; i < 6; ++i) inv[i * 6 + c] = x[i];
    }
    std::memcpy(out, inv, sizeof inv);
}

// SelfAdjointEigenSolver eigenvalues (src/stereoFrame.cpp:745-748,
// src/stereoFrameHandler.cpp:1997): cyclic Jacobi, ascending (pin N4).
void eig_sym(const double* A, int n, double* w) {
    double a[36];
    for (int i = 0; i < n * n; ++i) a[i] = A[i];
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off = off + a[p * n + q] * a[p * n + q];
        if (!(off > 0.0)) break;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                double apq = a[p * n + q];
                if (apq == 0.0) continue;
                double app = a[p * n + p], aqq = a[q * n + q];
                double theta = (aqq - app) / (2.0 * apq);
                double t;
                if (std::fabs(theta) > 1e150) t = 0.5 / theta;
                else {
                    t = 1.0 / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                    if (theta < 0.0) t = -t;
                }
                double c = 1.0 / std::sqrt(t * t + 1.0);
                double s = t * c;
                for (int k = 0; k < n; ++k) {
                    if (k == p || k == q) continue;
                    double akp = a[k * n + p], akq = a[k * n + q];
                    double nkp = c * akp - s * akq;
                    double nkq = s * akp + c * akq;
                    a[k * n + p] = nkp; a[p * n + k] = nkp;
                    a[k * n + q] = nkq; a[q * n + k] = nkq;
                }
                a[p * n + p] = app - t * apq;
                a[q * n + q] = aqq + t * apq;
                a[p * n + q] = 0.0; a[q * n + p] = 0.0;
            }
    }
    for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
    for (int i = 1; i < n; ++i) {
        double v = w[i];
        int j = i - 1;
        while (j >= 0 && w[j] > v) { w[j + 1] = w[j]; --j; }
        w[j + 1] = v;
    }
}

// adjoint_se3 (src/auxiliar.cpp:216-223): [R, skew(t) R; 0, R]
void adjoint_se3(const double* T, double* Ad) {
    double R[9], t[3] = {T[3], T[7], T[11]}, S[9], SR[9];
    for (int i = 0; i < 36; ++i) Ad[i] = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = T[i * 4 + j];
    skew3(t, S);
    mat3_mul(S, R, SR);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            Ad[i * 6 + j] = R[i * 3 + j];
            Ad[i * 6 + 3 + j] = SR[i * 3 + j];
            Ad[(3 + i) * 6 + 3 + j] = R[i * 3 + j];
        }
}

// [C +] A X A^T for 6x6 (Eigen: the product A*X into a temporary, then * A^T;
// inner products k-sequential, pin N2; C + product as in `covT1 + adj*cov*adj^T`)
void sandwich6(const double* A, const double* X, const double* C, double* out) {
    double AS[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double s = A[i * 6 + 0] * X[0 * 6 + j];
            for (int k = 1; k < 6; ++k) s = s + A[i * 6 + k] * X[k * 6 + j];
            AS[i * 6 + j] = s;
        }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double s = AS[i * 6 + 0] * A[j * 6 + 0];
            for (int k = 1; k < 6; ++k) s = s + AS[i * 6 + k] * A[j * 6 + k];
            out[i * 6 + j] = C ? C[i * 6 + j] + s : s;
        }
}

// unccomp_se3 (src/auxiliar.cpp:233-238): covT1 + adj(T1) covTinc adj(T1)^T
void unccomp_se3(const double* T1, const double* cov1, const double* covInc, double* out) {
    double Ad[36];
    adjoint_se3(T1, Ad);
    sandwich6(Ad, covInc, cov1, out);
}

// Matrix6d::determinant (Eigen 3.3, size > 4: PartialPivLU): the factorisation of
// inverse6, det = (-1)^transpositions * (((((d0 d1) d2) d3) d4) d5) — the
// diagonal product pinned left to right (the reference's vectorised redux order
// is machine-dependent)
double det6(const double* A) {
    double m[36];
    std::memcpy(m, A, sizeof m);
    int ntr = 0;
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double pv = std::fabs(m[k * 6 + k]);
        for (int i = k + 1; i < 6; ++i) {
            double v = std::fabs(m[i * 6 + k]);
            if (v > pv) { pv = v; p = i; }
        }
        if (p != k) {
            for (int j = 0; j < 6; ++j) std::swap(m[k * 6 + j], m[p * 6 + j]);
            ++ntr;
        }
        double piv = m[k * 6 + k];
        if (piv != 0.0)
            for (int i = k + 1; i < 6; ++i) m[i * 6 + k] = m[i * 6 + k] / piv;
        for (int i = k + 1; i < 6; ++i)
            for (int j = k + 1; j < 6; ++j) m[i * 6 + j] = m[i * 6 + j] - m[i * 6 + k] * m[k * 6 + j];
    }
    double d = m[0];
    for (int i = 1; i < 6; ++i) d = d * m[i * 7];
    return (ntr & 1) ? -1.0 * d : 1.0 * d;
}

// entropy of a 6-dof Gaussian as needNewKF writes it: 3(1 + log(2 acos(-1))) + 0.5 log det
double kf_entropy(const double* cov) {
    const double c0 = 3.0 * (1.0 + det_log(2.0 * 3.141592653589793));   // acos(-1) = pi
    return c0 + 0.5 * det_log(det6(cov));
}

// is_finite (src/auxiliar.cpp:475-477)
bool is_finite16(const double* T) {
    for (int i = 0; i < 16; ++i) { double d = T[i] - T[i]; if (!(d == d)) return false; }
    return true;
}

// ================================================================ matching ==
typedef std::array<uint8_t, 32> Desc;

// descriptorDistance (include/stereoFrame.h:185-201) and OpenCV normHamming
// cellSize 1 / 2 (NORM_HAMMING2 counts non-zero 2-bit cells).
int hamming(const uint8_t* a, const uint8_t* b, int cell) {
    int d = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        if (cell == 2) v = (v | (v >> 1)) & 0x55555555u;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        d += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return d;
}

struct DMatch { int queryIdx, trainIdx; float distance; };
typedef std::array<DMatch, 2> Knn2;

// BFMatcher::knnMatch(k=2) via cv::batchDistance's insertion rule (ledger T1):
// d < dist[K-1] then shift while dist[k] > d -> ties keep the lower train index.
std::vector<Knn2> knn2(const std::vector<Desc>& q, const std::vector<Desc>& t, int cell) {
    std::vector<Knn2> out(q.size());
    for (size_t i = 0; i < q.size(); ++i) {
        int dist[2] = {INT_MAX, INT_MAX}, idx[2] = {-1, -1};
        for (size_t j = 0; j < t.size(); ++j) {
            int d = hamming(q[i].data(), t[j].data(), cell);
            if (d < dist[1]) {
                int k = 0;
                for (k = 0; k >= 0 && dist[k] > d; --k) { idx[k + 1] = idx[k]; dist[k + 1] = dist[k]; }
                idx[k + 1] = (int)j; dist[k + 1] = d;
            }
        }
        out[i][0] = {(int)i, idx[0], (float)dist[0]};
        out[i][1] = {(int)i, idx[1], (float)dist[1]};
    }
    return out;
}

// lineDescriptorMAD (src/stereoFrame.cpp:1287-1313): only nn12_mad is used by
// the callers; nn_dist_median is uninitialised in the reference (ledger U1:
// pinned to 0.0), so the deviations are fabsf(float(d1-d0)).
double lineDescriptorMAD_nn12(const std::vector<Knn2>& m) {
    std::vector<float> v(m.size());
    const double nn_dist_median = 0.0;   // U1
    for (size_t j = 0; j < m.size(); ++j)
        v[j] = std::fabs((float)((double)(m[j][1].distance - m[j][0].distance) - nn_dist_median));
    std::sort(v.begin(), v.end());
    return 1.4826 * (double)v[v.size() / 2];
}

// lineDescriptorBudgetThres (src/stereoFrame.cpp:1329-1341)
double lineDescriptorBudgetThres(const std::vector<Knn2>& m, int max_num) {
    std::vector<float> v(m.size());
    for (size_t j = 0; j < m.size(); ++j) v[j] = m[j][0].distance;
    std::sort(v.begin(), v.end());
    size_t bi = std::min((size_t)max_num, v.size()) - 1;
    return (double)v[bi];
}

// lineSegmentOverlapStereo (src/stereoFrame.cpp:1343-1371), ledger Q9
double overlapStereo(double spl_obs, double epl_obs, double spl_proj, double epl_proj) {
    double sln = std::min(spl_obs, epl_obs);
    double eln = std::max(spl_obs, epl_obs);
    double spn = std::min(spl_proj, epl_proj);
    double epn = std::max(spl_proj, epl_proj);
    double length = eln - spn;
    double overlap;
    if ((epn < sln) || (spn > eln)) overlap = 0.0;
    else {
        if ((epn > eln) && (spn < sln)) overlap = eln - sln;
        else overlap = std::min(eln, epn) - std::max(sln, spn);
    }
    if (length > 0.01f) overlap = overlap / length;
    else overlap = 0.0;
    return overlap;
}

// ================================================================== state ==
struct Cam {
    int width, height;
    double fx, fy, cx, cy, b;
    int nlev;
    float scale[GFPL_MAX_LEVELS], inv[GFPL_MAX_LEVELS];
    int cols[GFPL_MAX_LEVELS], rows[GFPL_MAX_LEVELS];
    int64_t off[GFPL_MAX_LEVELS];
    double sigma2_pt[GFPL_MAX_LEVELS], sigma2_ln[GFPL_MAX_LEVELS];
};

struct PointF {
    int idx = 0;
    double pl[2] = {0, 0}, pl_obs[2] = {0, 0};
    double disp = 0;
    double P[3] = {0, 0, 0};
    bool inlier = true;
    int level = 0;
    double sigma2 = 1.0;
    bool frame_matched = false;
};

struct LineF {
    int idx = 0;
    double spl[2] = {0, 0}, epl[2] = {0, 0}, spl_obs[2] = {0, 0}, epl_obs[2] = {0, 0};
    double sdisp = 0, edisp = 0, angle = 0, sdisp_obs = 0, edisp_obs = 0;
    double sP[3] = {0, 0, 0}, eP[3] = {0, 0, 0}, le[3] = {0, 0, 0}, le_obs[3] = {0, 0, 0};
    bool inlier = true;
    int level = 0;
    double sigma2 = 1.0;
    double covS[9] = {0}, covE[9] = {0};
    double cut[2] = {0, 0};
    double invCov[36] = {0};
};

struct Frame {
    double time_stamp = 0;
    double Tfw[16], DT[16], Tfw_cov[36], DT_cov[36], DT_cov_eig[6];
    double err_norm = 0;
    std::vector<PointF> pt;
    std::vector<LineF> ls;
    std::vector<Desc> pdesc, ldesc;
    // injected detections (views into the caller's host batch)
    const gfpl_frames* in = nullptr;
    gfpl_frames in_store{};   // begin_frame keeps a copy: the caller's struct may be a temporary
    int seq = 0;
    Frame() {
        for (int i = 0; i < 16; ++i) Tfw[i] = DT[i] = (i % 5 == 0) ? 1.0 : 0.0;
        for (int i = 0; i < 36; ++i) Tfw_cov[i] = DT_cov[i] = 0.0;
        for (int i = 0; i < 6; ++i) DT_cov_eig[i] = 0.0;
    }
    int nkl() const { return in->n_kp_l[seq]; }
    int nkr() const { return in->n_kp_r[seq]; }
    const gfpl_keypoint& kpl(int i) const { return in->kp_l[(size_t)seq * in->kp_cap + i]; }
    const gfpl_keypoint& kpr(int i) const { return in->kp_r[(size_t)seq * in->kp_cap + i]; }
    const uint8_t* pdl(int i) const { return in->pdesc_l + ((size_t)seq * in->kp_cap + i) * 32; }
    const uint8_t* pdr(int i) const { return in->pdesc_r + ((size_t)seq * in->kp_cap + i) * 32; }
    int nll() const { return in->n_kl_l[seq]; }
    int nlr() const { return in->n_kl_r[seq]; }
    const gfpl_keyline& kll(int i) const { return in->kl_l[(size_t)seq * in->kl_cap + i]; }
    const gfpl_keyline& klr(int i) const { return in->kl_r[(size_t)seq * in->kl_cap + i]; }
    const uint8_t* ldl(int i) const { return in->ldesc_l + ((size_t)seq * in->kl_cap + i) * 32; }
    const uint8_t* ldr(int i) const { return in->ldesc_r + ((size_t)seq * in->kl_cap + i) * 32; }
};

std::vector<Desc> collect(const uint8_t* (Frame::*f)(int) const, const Frame& fr, int n) {
    std::vector<Desc> v(n);
    for (int i = 0; i < n; ++i) std::memcpy(v[i].data(), (fr.*f)(i), 32);
    return v;
}

}  // namespace

// Line-cut work counters and duplicate-evaluation scans: analysis only, compiled in with
// -DGFPL_ORACLE_CUT_STATS (off in liboracle.so, which is also the timed CPU baseline: shared
// counters bumped from every worker thread and the linear duplicate scans cost more than the
// search itself at 16 threads).
#ifdef GFPL_ORACLE_CUT_STATS
static int64_t g_cut_stats[8];
// per line: the smallest metric gap a step decision rests on (histogram by decade, 1e-16 .. 1e3)
static int64_t g_cut_gap_hist[20];
// moves by (sign of the start-ratio change + 1) * 3 + (sign of the end-ratio change + 1); [9]: a
// single-ratio move right after one on the same ratio in the same direction; [10]: lines
static int64_t g_cut_moves[11];
static std::string g_cut_paths;   // per line: the move classes, one character each ('0' + class, 'S' stay)
#define CUT_STAT(stmt) do { stmt; } while (0)
#else
#define CUT_STAT(stmt) do { } while (0)
#endif

struct gfplo_handler {
    Cam cam;
    gfpl_config cfg;
    Frame* prev = nullptr;
    Frame* curr = nullptr;
    std::vector<int> matched_pt, matched_ls;
    int n_inliers = 0, n_inliers_pt = 0, n_inliers_ls = 0;
    int numFrameLoss = 0;
    // keyframe decision (include/stereoFrameHandler.h:147-153)
    int numFrameSinceKeyframe = 0;
    bool prev_f_iskf = true;
    double entropy_first_prevKF = 0.0, entropy_ratio = 0.0;
    double T_prevKF[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    double cov_prevKF_currF[36] = {0};
    int need_new_kf = 0;

    // needNewKF (src/stereoFrameHandler.cpp:2309-2349)
    bool needNewKF() {
        if (prev_f_iskf) {
            entropy_first_prevKF = kf_entropy(curr->DT_cov);
            prev_f_iskf = false;
        }
        double adj[36], Ti[16], adjTinv[36], covDTinv[36], acc[36];
        adjoint_se3(T_prevKF, adj);
        inverse_se3(curr->DT, Ti);            // uncTinv_se3 (src/auxiliar.cpp:225-231)
        adjoint_se3(Ti, adjTinv);
        sandwich6(adjTinv, curr->DT_cov, nullptr, covDTinv);
        sandwich6(adj, covDTinv, cov_prevKF_currF, acc);
        std::memcpy(cov_prevKF_currF, acc, sizeof acc);
        const double entropy_curr = kf_entropy(cov_prevKF_currF);
        entropy_ratio = entropy_curr / entropy_first_prevKF;
        bool zero_cov = true, ident = true;
        for (int i = 0; i < 36; ++i) zero_cov = zero_cov && curr->DT_cov[i] == 0.0;
        for (int i = 0; i < 16; ++i) ident = ident && curr->DT[i] == ((i % 5 == 0) ? 1.0 : 0.0);
        need_new_kf = (numFrameSinceKeyframe > cfg.max_kf_num_frames || entropy_ratio < cfg.min_entropy_ratio ||
                       std::isnan(entropy_ratio) || std::isinf(entropy_ratio) || (zero_cov && ident)) ? 1 : 0;
        return need_new_kf != 0;
    }

    // currFrameIsKF (src/stereoFrameHandler.cpp:2351-2379)
    void currFrameIsKF() {
        numFrameSinceKeyframe = 0;
        for (size_t i = 0; i < curr->pt.size(); ++i) curr->pt[i].idx = (int)i;
        for (size_t i = 0; i < curr->ls.size(); ++i) curr->ls[i].idx = (int)i;
        for (int i = 0; i < 16; ++i) curr->Tfw[i] = (i % 5 == 0) ? 1.0 : 0.0;
        for (int i = 0; i < 36; ++i) curr->Tfw_cov[i] = (i % 7 == 0) ? 1.0 : 0.0;
        std::memcpy(T_prevKF, curr->Tfw, sizeof T_prevKF);
        for (int i = 0; i < 36; ++i) cov_prevKF_currF[i] = 0.0;
        prev_f_iskf = true;
    }

    // ----------------------------------------------------------- camera --
    // PinholeStereoCamera::projection / backProjection / getDisparity
    // (src/pinholeStereoCamera.cpp:133-141,159-170), ledger Q8 (fx only in back-projection)
    void projection(const double* P, double* uv) const {
        uv[0] = cam.cx + (cam.fx * P[0]) / P[2];
        uv[1] = cam.cy + (cam.fy * P[1]) / P[2];
    }
    void backProjection(double u, double v, double disp, double* P) const {
        double bd = cam.b / disp;
        P[0] = bd * (u - cam.cx);
        P[1] = bd * (v - cam.cy);
        P[2] = bd * cam.fx;
    }
    double getDisparity(double pZ) const { return (cam.fx * cam.b) / pZ; }

    // ------------------------------------------- extractInitialStereoFeatures
    // src/stereoFrame.cpp:173-336 (detection injected)
    void extractInitialStereoFeatures(Frame& f) {
        f.pt.clear(); f.pdesc.clear();
        int N = f.nkl(), Nr = f.nkr();
        if (N > 0 && Nr > 0 && N >= 2 && Nr >= 2) {   // U4 guard
            std::vector<Desc> dl = collect(&Frame::pdl, f, N), dr = collect(&Frame::pdr, f, Nr);
            std::vector<Knn2> lr = knn2(dl, dr, 1), rl = knn2(dr, dl, 1);
            int pt_idx = 0;
            for (int i = 0; i < N; ++i) {
                int lr_qdx = lr[i][0].queryIdx, lr_tdx = lr[i][0].trainIdx;
                int rl_tdx = rl[lr_tdx][0].trainIdx;
                double dist_12 = (double)(lr[i][0].distance / lr[i][1].distance);
                if (lr_qdx == rl_tdx && dist_12 <= cfg.max_ratio_12_p) {
                    const gfpl_keypoint& kl = f.kpl(lr_qdx);
                    const gfpl_keypoint& kr = f.kpr(lr_tdx);
                    if ((double)std::fabs(kl.y - kr.y) <= cfg.max_dist_epip) {
                        double disp_ = (double)(kl.x - kr.x);
                        if (disp_ >= cfg.min_disp) {
                            PointF p;
                            p.pl[0] = kl.x; p.pl[1] = kl.y;
                            p.disp = disp_;
                            backProjection(p.pl[0], p.pl[1], disp_, p.P);
                            p.idx = pt_idx; p.level = kl.octave; p.sigma2 = cam.sigma2_pt[clampl(kl.octave, cam.nlev)]; p.inlier = true;
                            f.pt.push_back(p);
                            f.pdesc.push_back(dl[lr_qdx]);
                            ++pt_idx;
                        }
                    }
                }
            }
        }
        f.ls.clear(); f.ldesc.clear();
        int NL = f.nll(), NR = f.nlr();
        if (NL >= 2 && NR >= 2) {   // U4 guard
            std::vector<Desc> dl = collect(&Frame::ldl, f, NL), dr = collect(&Frame::ldr, f, NR);
            std::vector<Knn2> lr = knn2(dl, dr, 1), rl = knn2(dr, dl, 1);
            double nn12_dist_th = lineDescriptorMAD_nn12(lr) * cfg.desc_th_l;
            int n_matches = std::min(NL, NR);   // Q5
            int ls_idx = 0;
            for (int i = 0; i < n_matches; ++i) {
                int lr_qdx = lr[i][0].queryIdx, lr_tdx = lr[i][0].trainIdx;
                int rl_tdx = rl[lr_tdx][0].trainIdx;
                double dist_12 = (double)(lr[i][1].distance - lr[i][0].distance);
                if (lr_qdx == rl_tdx && dist_12 > nn12_dist_th) {
                    LineF L;
                    if (triangulate(f, lr_qdx, lr_tdx, /*initial=*/true, &L)) {
                        L.idx = ls_idx++;
                        f.ls.push_back(L);
                        f.ldesc.push_back(dl[lr_qdx]);
                    }
                }
            }
        }
    }

    // Line triangulation shared by the initial (src/stereoFrame.cpp:301-330)
    // and per-frame (:684-760) branches.  Returns whether the line is kept.
    bool triangulate(const Frame& f, int lq, int rt, bool initial, LineF* out) {
        const gfpl_keyline& a = f.kll(lq);
        const gfpl_keyline& c = f.klr(rt);
        double sp_l[3] = {a.sx, a.sy, 1.0}, ep_l[3] = {a.ex, a.ey, 1.0};
        double le_l[3] = {sp_l[1] * ep_l[2] - sp_l[2] * ep_l[1], sp_l[2] * ep_l[0] - sp_l[0] * ep_l[2],
                          sp_l[0] * ep_l[1] - sp_l[1] * ep_l[0]};
        double nrm = std::sqrt(le_l[0] * le_l[0] + le_l[1] * le_l[1]);
        le_l[0] = le_l[0] / nrm; le_l[1] = le_l[1] / nrm; le_l[2] = le_l[2] / nrm;
        double sp_r[3] = {c.sx, c.sy, 1.0}, ep_r[3] = {c.ex, c.ey, 1.0};
        double le_r[3] = {sp_r[1] * ep_r[2] - sp_r[2] * ep_r[1], sp_r[2] * ep_r[0] - sp_r[0] * ep_r[2],
                          sp_r[0] * ep_r[1] - sp_r[1] * ep_r[0]};
        double overlap = overlapStereo(sp_l[1], ep_l[1], sp_r[1], ep_r[1]);
        double spx = (-(le_r[2] + le_r[1] * (double)a.sy)) / le_r[0];
        double epx = (-(le_r[2] + le_r[1] * (double)a.ey)) / le_r[0];
        double disp_s = (double)a.sx - spx;
        double disp_e = (double)a.ex - epx;
        double horiz = initial ? (double)std::fabs((float)le_r[0]) : (double)std::fabs((float)le_l[0]);
        if (!(disp_s >= cfg.min_disp && disp_e >= cfg.min_disp && horiz > cfg.line_horiz_th &&
              overlap > cfg.stereo_overlap_th))
            return false;
        LineF L;
        L.spl[0] = sp_l[0]; L.spl[1] = sp_l[1];
        L.epl[0] = ep_l[0]; L.epl[1] = ep_l[1];
        L.sdisp = disp_s; L.edisp = disp_e;
        backProjection(sp_l[0], sp_l[1], disp_s, L.sP);
        backProjection(ep_l[0], ep_l[1], disp_e, L.eP);
        L.le[0] = le_l[0]; L.le[1] = le_l[1]; L.le[2] = le_l[2];
        L.angle = (double)a.angle;
        L.level = a.octave;
        L.sigma2 = cam.sigma2_ln[clampl(a.octave, GFPL_MAX_LEVELS)];
        L.inlier = true;
        if (!initial) {
            // endpoint covariance gate (src/stereoFrame.cpp:707-751)
            double cS[9], cE[9];
            endpointCov(sp_l[0], sp_l[1], disp_s, cS);
            endpointCov(ep_l[0], ep_l[1], disp_e, cE);
            double wS[3], wE[3];
            eig_sym(cS, 3, wS);
            eig_sym(cE, 3, wE);
            double max_eig = std::max(wS[2], wE[2]);
            if (!(max_eig < cfg.line_cov_th)) return false;
            L.idx = -1;
        }
        *out = L;
        return true;
    }

    void endpointCov(double u, double v, double disp, double* C) const {
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
        for (int i = 0; i < 9; ++i) C[i] = ((C[i] * cam.b) * cam.b) / dd;
    }

    // --------------------------------------- subPixelStereoRefine_ORBSLAM --
    // src/stereoFrame.cpp:340-404 (ledger Q1: both patches from the RIGHT pyramid)
    void subPixel(const Frame& f, const gfpl_keypoint& kpL, const gfpl_keypoint& kpR,
                  float& disparity, float& bestuR) const {
        disparity = -1;
        bestuR = kpR.x;
        const float uR0 = kpR.x;
        const int o = clampl(kpL.octave, cam.nlev);
        const float scaleFactor = cam.inv[o];
        const float scaleduL = std::round(kpL.x * scaleFactor);
        const float scaledvL = std::round(kpL.y * scaleFactor);
        const float scaleduR0 = std::round(uR0 * scaleFactor);
        const int w = 5, L = 5;
        const int cols = cam.cols[o], rows = cam.rows[o];
        const uint8_t* img = f.in->pyr_r + pyr_off(f) + cam.off[o];
        const float iniu = scaleduR0 + L - w;
        const float endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= cols) return;
        // U8 guard: windows outside the level image are rejected (the reference asserts)
        int vL = (int)scaledvL, uL = (int)scaleduL, uR = (int)scaleduR0;
        if (vL - w < 0 || vL + w >= rows || uL - w < 0 || uL + w >= cols || uR - L - w < 0 || uR + L + w >= cols) return;
        float IL[121];
        float cL = (float)img[(size_t)vL * cols + uL];
        for (int r = 0; r < 11; ++r)
            for (int c = 0; c < 11; ++c) IL[r * 11 + c] = (float)img[(size_t)(vL - w + r) * cols + (uL - w + c)] - cL;
        int bestDist = INT_MAX;
        int bestincR = 0;
        float vDists[11];
        for (int incR = -L; incR <= L; ++incR) {
            int uc = uR + incR;
            float cR = (float)img[(size_t)vL * cols + uc];
            double acc = 0.0;
            for (int r = 0; r < 11; ++r)
                for (int c = 0; c < 11; ++c) {
                    float ir = (float)img[(size_t)(vL - w + r) * cols + (uc - w + c)] - cR;
                    acc += (double)std::fabs(IL[r * 11 + c] - ir);
                }
            float dist = (float)acc;
            if (dist < (float)bestDist) { bestDist = (int)dist; bestincR = incR; }
            vDists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) return;
        const float dist1 = vDists[L + bestincR - 1];
        const float dist2 = vDists[L + bestincR];
        const float dist3 = vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) return;
        bestuR = cam.scale[o] * ((float)scaleduR0 + (float)bestincR + deltaR);
        disparity = (kpL.x - bestuR);
    }
    int64_t pyr_off(const Frame& f) const { return (int64_t)f.seq * pyr_bytes; }
    int64_t pyr_bytes = 0;

    // ------------------------------------ extractStereoFeatures_ORBSLAM pts
    // src/stereoFrame.cpp:453-630
    void stereoPoints(Frame& f) {
        f.pt.clear(); f.pdesc.clear();
        int N = f.nkl(), Nr = f.nkr();
        if (N == 0 || Nr == 0) return;
        const int thOrbDist = 80;
        const int nRows = cam.height;
        std::vector<std::vector<int>> vRowIndices(nRows);
        for (int iR = 0; iR < Nr; ++iR) {
            const gfpl_keypoint& kp = f.kpr(iR);
            const float kpY = kp.y;
            const float r = 2.0f * cam.scale[clampl(kp.octave, cam.nlev)];
            const int maxr = (int)std::ceil(kpY + r);
            const int minr = (int)std::floor(kpY - r);
            for (int yi = minr; yi <= maxr; ++yi)
                if (yi >= 0 && yi < nRows) vRowIndices[yi].push_back(iR);   // U9 guard
        }
        const float minD = 0;
        const float maxD = (float)cam.fx;
        const float mbf = (float)(cam.fx * cam.b);
        std::vector<float> mvDepth(N, -1.0f);
        std::vector<std::pair<int, int>> vDistIdx;
        for (int iL = 0; iL < N; ++iL) {
            const gfpl_keypoint& kpL = f.kpl(iL);
            const int levelL = kpL.octave;
            const float vL = kpL.y, uL = kpL.x;
            if (!(vL >= 0.0f) || (size_t)vL >= (size_t)nRows) continue;   // U9 guard
            const std::vector<int>& cand = vRowIndices[(size_t)vL];
            if (cand.empty()) continue;
            const float minU = uL - maxD;
            const float maxU = uL - minD;
            if (maxU < 0) continue;
            int bestDist = 100;
            int bestIdxR = 0;
            for (size_t iC = 0; iC < cand.size(); ++iC) {
                const int iR = cand[iC];
                const gfpl_keypoint& kpR = f.kpr(iR);
                if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
                const float uR = kpR.x;
                if (uR >= minU && uR <= maxU) {
                    const int dist = hamming(f.pdl(iL), f.pdr(iR), 1);
                    if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
                }
            }
            if (bestDist < thOrbDist) {
                float disparity, bestuR;
                subPixel(f, kpL, f.kpr(bestIdxR), disparity, bestuR);
                if (disparity >= minD && disparity < maxD) {
                    if (disparity <= 0) { disparity = 0.01f; bestuR = (float)((double)uL - 0.01); }
                    mvDepth[iL] = mbf / disparity;
                    vDistIdx.push_back(std::make_pair(bestDist, iL));
                }
            }
        }
        if (vDistIdx.empty()) return;   // U5 guard
        std::sort(vDistIdx.begin(), vDistIdx.end());
        const float median = (float)vDistIdx[vDistIdx.size() / 2].first;
        const float thDist = 1.5f * 1.4f * median;
        int pt_idx = 0;
        for (size_t i = 0; i < vDistIdx.size(); ++i) {
            if ((float)vDistIdx[i].first >= thDist) break;
            int iL = vDistIdx[i].second;
            const gfpl_keypoint& kpL = f.kpl(iL);
            PointF p;
            p.pl[0] = kpL.x; p.pl[1] = kpL.y;
            float disparity = mbf / mvDepth[iL];   // Q6 float round trip
            if (disparity < 0) continue;
            p.disp = (double)disparity;
            backProjection(p.pl[0], p.pl[1], p.disp, p.P);
            p.idx = pt_idx; p.level = kpL.octave; p.sigma2 = cam.sigma2_pt[clampl(kpL.octave, cam.nlev)]; p.inlier = true;
            f.pt.push_back(p);
            Desc d; std::memcpy(d.data(), f.pdl(iL), 32);
            f.pdesc.push_back(d);
            ++pt_idx;
        }
    }

    // ------------------------------------ extractStereoFeatures_ORBSLAM lines
    // src/stereoFrame.cpp:633-767
    void stereoLines(Frame& f) {
        f.ls.clear(); f.ldesc.clear();
        int NL = f.nll(), NR = f.nlr();
        if (NL < 2 || NR < 2) return;   // empty -> reference skips; 1 row -> U4 guard
        std::vector<Desc> dl = collect(&Frame::ldl, f, NL), dr = collect(&Frame::ldr, f, NR);
        std::vector<Knn2> lr = knn2(dl, dr, 2), rl = knn2(dr, dl, 2);   // Q7 HAMMING2
        double nn12_dist_th = lineDescriptorMAD_nn12(lr) * cfg.desc_th_l;
        int n_matches = std::min(NL, NR);   // Q5
        for (int i = 0; i < n_matches; ++i) {
            int lr_qdx = lr[i][0].queryIdx, lr_tdx = lr[i][0].trainIdx;
            int rl_tdx = rl[lr_tdx][0].trainIdx;
            double dist_12 = (double)(lr[i][1].distance - lr[i][0].distance);
            if (lr_qdx == rl_tdx && dist_12 > nn12_dist_th) {
                LineF L;
                if (triangulate(f, lr_qdx, lr_tdx, /*initial=*/false, &L)) {
                    f.ls.push_back(L);
                    f.ldesc.push_back(dl[lr_qdx]);
                }
            }
        }
    }

    // -------------------------------------------- estimateStereoUncertainty
    // src/stereoFrame.cpp:1448-1484 + getCovMat2D_3D :1434-1446 + getJacob2D_3D :1375-1392
    void covMat2D_3D(double u, double v, double u_std, double d, double d_std, double* cov) const {
        double cov2D[9] = {u_std * u_std, 0, 0, 0, u_std * u_std, 0, 0, 0, d_std * d_std};   // U2: off-diagonals 0
        double b = cam.b, d_2 = d * d;
        double J[9];
        J[0] = b / d;  J[3] = 0.0; J[6] = 0.0;
        J[1] = 0.0;    J[4] = b / d; J[7] = 0.0;
        J[2] = ((-(u - cam.cx)) * b) / d_2;
        J[5] = ((-(v - cam.cy)) * b) / d_2;
        J[8] = ((-cam.fx) * b) / d_2;
        double JC[9];
        mat3_mul(J, cov2D, JC);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                cov[i * 3 + j] = (JC[i * 3 + 0] * J[j * 3 + 0] + JC[i * 3 + 1] * J[j * 3 + 1]) + JC[i * 3 + 2] * J[j * 3 + 2];
    }
    void estimateStereoUncertainty(Frame& f) {
        for (LineF& L : f.ls) {
            double spl_std = 1.0, epl_std = 1.0, sdisp_std, edisp_std;
            if (std::fabs(L.le[0]) > 0.15) {
                sdisp_std = cfg.ratio_disp_std * L.sdisp;
                edisp_std = cfg.ratio_disp_std * L.edisp;
            } else {
                sdisp_std = cfg.ratio_disp_std_hor * L.sdisp;
                edisp_std = cfg.ratio_disp_std_hor * L.edisp;
            }
            covMat2D_3D(L.spl[0], L.spl[1], spl_std, L.sdisp, sdisp_std, L.covS);
            covMat2D_3D(L.epl[0], L.epl[1], epl_std, L.edisp, edisp_std, L.covE);
        }
    }

    // ------------------------------------------------ crossFrameMatching points
    // predictFramePose (src/stereoFrameHandler.cpp:153-157) + points part of
    // crossFrameMatching_Hybrid (:451-603) + projectPrev3DPoint (src/stereoFrame.cpp:1550-1570)
    void predictFramePose() { mat4_mul(prev->Tfw, prev->DT, curr->Tfw); }

    void crossPoints() {
        matched_pt.clear();
        Frame& P = *prev;
        Frame& C = *curr;
        if (C.pt.empty() || P.pt.empty()) return;
        for (auto& p : P.pt) p.frame_matched = false;
        for (auto& p : C.pt) p.frame_matched = false;
        double Tinv[16];
        mat4_inv(C.Tfw, Tinv);
        const float radius = (float)cfg.point_match_radius;
        // multimap<curr idx, (prev idx, dist)>; values of a key kept in insertion order
        std::map<int, std::vector<std::pair<int, float>>> pair_frame;
        for (int q = 0; q < (int)P.pt.size(); ++q) {
            // radiusMatch row q (ledger T1: <= maxDistance)
            std::vector<std::pair<int, float>> row;
            for (int t = 0; t < (int)C.pt.size(); ++t) {
                float d = (float)hamming(P.pdesc[q].data(), C.pdesc[t].data(), 1);
                if (d <= radius) row.push_back(std::make_pair(t, d));
            }
            if (row.empty()) continue;
            if (P.pt[q].frame_matched) continue;
            double v[4] = {P.pt[q].P[0], P.pt[q].P[1], P.pt[q].P[2], 1.0};
            mat4_vec(P.Tfw, v, v);
            mat4_vec(Tinv, v, v);
            double uv[2];
            projection(v, uv);
            for (auto& tc : row) {
                int t = tc.first;
                double dx = uv[0] - C.pt[t].pl[0], dy = uv[1] - C.pt[t].pl[1];
                if (std::sqrt(dx * dx + dy * dy) > cfg.proj_gate_px) continue;
                pair_frame[t].push_back(std::make_pair(q, tc.second));
            }
        }
        // resolution: distinct keys ascending (ledger U3), strict min dist -> first inserted
        for (auto& kv : pair_frame) {
            float min_value = 1e+7f;
            int mq = 0;
            for (auto& qv : kv.second)
                if (qv.second < min_value) { min_value = qv.second; mq = qv.first; }
            int t = kv.first;
            PointF& pp = P.pt[mq];
            pp.pl_obs[0] = C.pt[t].pl[0]; pp.pl_obs[1] = C.pt[t].pl[1];
            pp.inlier = true;
            matched_pt.push_back(mq);   // Q12: duplicates allowed
            C.pt[t].idx = pp.idx;
            pp.frame_matched = true;
            C.pt[t].frame_matched = true;
            if ((int)matched_pt.size() >= cfg.max_point_match_num) break;
        }
    }

    // --------------------------------------------------- crossFrameMatching lines
    // src/stereoFrameHandler.cpp:605-690
    void crossLines() {
        matched_ls.clear();
        Frame& P = *prev;
        Frame& C = *curr;
        if (C.ls.empty() || P.ls.empty()) return;
        if (C.ls.size() < 2 || P.ls.size() < 2) return;   // U4 guard
        std::vector<Knn2> l12 = knn2(P.ldesc, C.ldesc, 1), l21 = knn2(C.ldesc, P.ldesc, 1);
        double nn12_dist_th = lineDescriptorMAD_nn12(l12) * cfg.desc_th_l;
        double budget = lineDescriptorBudgetThres(l12, cfg.max_line_match_num);
        for (int i = 0; i < (int)l12.size(); ++i) {
            int lr_qdx = l12[i][0].queryIdx, lr_tdx = l12[i][0].trainIdx;
            int rl_tdx = l21[lr_tdx][0].trainIdx;
            if ((double)l12[i][0].distance > 1.2 * budget) continue;
            double dist_12 = (double)(l12[i][1].distance - l12[i][0].distance);
            if (lr_qdx == rl_tdx && dist_12 > nn12_dist_th) {
                LineF& L = P.ls[lr_qdx];
                const LineF& M = C.ls[lr_tdx];
                L.sdisp_obs = M.sdisp; L.edisp_obs = M.edisp;
                L.spl_obs[0] = M.spl[0]; L.spl_obs[1] = M.spl[1];
                L.epl_obs[0] = M.epl[0]; L.epl_obs[1] = M.epl[1];
                for (int k = 0; k < 3; ++k) L.le_obs[k] = M.le[k];
                L.inlier = true;
                matched_ls.push_back(lr_qdx);
                C.ls[lr_tdx].idx = L.idx;
            }
            if ((int)matched_ls.size() >= cfg.max_line_match_num) break;
        }
    }

    void finishCounts() {
        n_inliers_pt = (int)matched_pt.size();
        n_inliers_ls = (int)matched_ls.size();
        n_inliers = n_inliers_pt + n_inliers_ls;
    }

    // ------------------------------------------------------ line-cut helpers
    // getJacob3D_2D (src/stereoFrame.cpp:1394-1412)
    void jacob3D_2D(double px, double py, double pz, double* J) const {
        double f = cam.fx, b = cam.b, pz_2 = pz * pz;
        J[0] = f / pz; J[3] = 0.0; J[6] = 0.0;
        J[1] = 0.0; J[4] = f / pz; J[7] = 0.0;
        J[2] = ((-f) * px) / pz_2;
        J[5] = ((-f) * py) / pz_2;
        J[8] = ((-f) * b) / pz_2;
    }

    // Jacobian of a projected residual wrt the pose (src/stereoFrameHandler.cpp:1383-1388,
    // 1438-1443, 2150-2155, 2197-2202) with weights (lx, ly) = line coeffs or error.
    void poseJac(const double* g, double lx, double ly, double* J) const {
        double gx = g[0], gy = g[1], gz = g[2];
        double gz2 = gz * gz;
        double fgz2 = cam.fx / ref_max(cfg.homog_th, gz2);
        J[0] = (fgz2 * lx) * gz;
        J[1] = (fgz2 * ly) * gz;
        J[2] = (-fgz2) * ((gx * lx) + (gy * ly));
        J[3] = (-fgz2) * ((((gx * gy) * lx) + ((gy * gy) * ly)) + ((gz * gz) * ly));
        J[4] = fgz2 * ((((gx * gx) * lx) + ((gz * gz) * lx)) + ((gx * gy) * ly));
        J[5] = fgz2 * (((gx * gz) * ly) - ((gy * gz) * lx));
    }

    // projected residual variance of one cut endpoint (src/stereoFrameHandler.cpp:1356-1369)
    double endpointVar(const double* DT_inv, const double* Jl, const double* Pt, const double* cov) const {
        double Jdt[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Jdt[i * 3 + j] = DT_inv[i * 4 + j];
        double cur[3];
        se3_apply(DT_inv, Pt, cur);
        double Jp[9];
        jacob3D_2D(cur[0], cur[1], cur[2], Jp);
        // ((((Jp2 * Jdt) * cov) * Jdt^T) * Jp2^T)
        double T1[6], T2[6], T3[6], M[4];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j)
                T1[i * 3 + j] = (Jp[i * 3 + 0] * Jdt[0 * 3 + j] + Jp[i * 3 + 1] * Jdt[1 * 3 + j]) + Jp[i * 3 + 2] * Jdt[2 * 3 + j];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j)
                T2[i * 3 + j] = (T1[i * 3 + 0] * cov[0 * 3 + j] + T1[i * 3 + 1] * cov[1 * 3 + j]) + T1[i * 3 + 2] * cov[2 * 3 + j];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j)
                T3[i * 3 + j] = (T2[i * 3 + 0] * Jdt[j * 3 + 0] + T2[i * 3 + 1] * Jdt[j * 3 + 1]) + T2[i * 3 + 2] * Jdt[j * 3 + 2];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j)
                M[i * 2 + j] = (T3[i * 3 + 0] * Jp[j * 3 + 0] + T3[i * 3 + 1] * Jp[j * 3 + 1]) + T3[i * 3 + 2] * Jp[j * 3 + 2];
        double r0 = Jl[0] * M[0] + Jl[1] * M[2];
        double r1 = Jl[0] * M[1] + Jl[1] * M[3];
        return r0 * Jl[0] + r1 * Jl[1];
    }

    // getPoseInfoOnLine (src/stereoFrameHandler.cpp:1342-1411)
    void poseInfoOnLine(const double* DT_inv, const double* Jl, const LineF& L, const double* cut, double* info) const {
        double sPt[3], ePt[3];
        for (int k = 0; k < 3; ++k) {
            sPt[k] = (1 - cut[0]) * L.sP[k] + cut[0] * L.eP[k];
            ePt[k] = (1 - cut[1]) * L.eP[k] + cut[1] * L.sP[k];
        }
        double a0 = (1 - cut[0]) * (1 - cut[0]), c0 = cut[0] * cut[0];
        double a1 = (1 - cut[1]) * (1 - cut[1]), c1 = cut[1] * cut[1];
        double covSt[9], covEt[9];
        for (int i = 0; i < 9; ++i) {
            covSt[i] = a0 * L.covS[i] + c0 * L.covE[i];
            covEt[i] = a1 * L.covE[i] + c1 * L.covS[i];
        }
        double vs = endpointVar(DT_inv, Jl, sPt, covSt);
        double ve = endpointVar(DT_inv, Jl, ePt, covEt);
        // cov_r.inverse(): Eigen 2x2 cofactor / invdet (ledger Q10)
        double det = vs * ve - 0.0 * 0.0;
        double invdet = 1.0 / det;
        double i00 = ve * invdet, i10 = -0.0 * invdet, i01 = -0.0 * invdet, i11 = vs * invdet;
        double curS[3], curE[3];
        se3_apply(DT_inv, sPt, curS);
        se3_apply(DT_inv, ePt, curE);
        double Js[6], Je[6];
        poseJac(curS, Jl[0], Jl[1], Js);
        poseJac(curE, Jl[0], Jl[1], Je);
        double T0[6], T1[6];
        for (int i = 0; i < 6; ++i) {
            T0[i] = Js[i] * i00 + Je[i] * i10;
            T1[i] = Js[i] * i01 + Je[i] * i11;
        }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) info[i * 6 + j] = T0[i] * Js[j] + T1[i] * Je[j];
    }

    // getPoseInfoPoint (src/stereoFrameHandler.cpp:1414-1447)
    void poseInfoPoint(const double* DT_inv, const PointF& p, double* info) const {
        double cur[3];
        se3_apply(DT_inv, p.P, cur);
        double uv[2];
        projection(cur, uv);
        double dx = uv[0] - p.pl_obs[0], dy = uv[1] - p.pl_obs[1];
        double J[6];
        poseJac(cur, dx, dy, J);
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) info[i * 6 + j] = J[i] * J[j];
    }

    // updateEndPointByRatio (src/stereoFrameHandler.cpp:1451-1470), ledger Q4
    void updateEndPointByRatio(LineF& L) const {
        if (std::fabs(L.cut[0]) < 0.0001 && std::fabs(L.cut[1]) < 0.0001) return;
        if (std::fabs(L.cut[0]) > 0.0001) {
            double s[3];
            for (int k = 0; k < 3; ++k) s[k] = (1 - L.cut[0]) * L.sP[k] + L.cut[0] * L.eP[k];
            std::memcpy(L.sP, s, sizeof s);
            projection(L.sP, L.spl);
            L.sdisp = getDisparity(L.sP[2]);
        }
        if (std::fabs(L.cut[1]) > 0.0001) {
            double e[3];
            for (int k = 0; k < 3; ++k) e[k] = (1 - L.cut[1]) * L.eP[k] + L.cut[1] * L.sP[k];
            std::memcpy(L.eP, e, sizeof e);
            projection(L.eP, L.epl);
            L.edisp = getDisparity(L.eP[2]);
        }
    }

    // estimateProjUncertainty_submodular (src/stereoFrameHandler.cpp:1618-1764)
    void lineCut() {
        if (matched_ls.empty()) return;
        const double s = cfg.cut_step;
        const double nb[8][2] = {{s, 0}, {-s, 0}, {0, s}, {0, -s}, {s, s}, {s, -s}, {-s, s}, {-s, -s}};
        double Tinv[16], DT_inv[16];
        mat4_inv(curr->Tfw, Tinv);
        mat4_mul(Tinv, prev->Tfw, DT_inv);
        double sum[36] = {0};
        for (int li : matched_ls) {
            LineF& L = prev->ls[li];
            double Jl[2] = {L.le_obs[0], L.le_obs[1]};
            L.cut[0] = 0; L.cut[1] = 0;
            poseInfoOnLine(DT_inv, Jl, L, L.cut, L.invCov);
            for (int i = 0; i < 36; ++i) sum[i] = sum[i] + L.invCov[i];
        }
        for (int pi : matched_pt) {
            double tmp[36];
            poseInfoPoint(DT_inv, prev->pt[pi], tmp);
            for (int i = 0; i < 36; ++i) sum[i] = sum[i] + tmp[i];
        }
#ifdef GFPL_ORACLE_CUT_STATS
        bool prev_moved = true;
        double sum_before[36];
#endif
        for (int li : matched_ls) {
            LineF& L = prev->ls[li];
            double Jl[2] = {L.le_obs[0], L.le_obs[1]};
            double metric_back = logdet6(sum);
#ifdef GFPL_ORACLE_CUT_STATS
            g_cut_stats[0]++;   // lines
            if (!prev_moved) {
                bool same = true;
                for (int i = 0; i < 36; ++i) same = same && (sum[i] == sum_before[i]);
                if (!same) g_cut_stats[5]++;   // setup logdet really needed
            }
            std::memcpy(sum_before, sum, sizeof sum);
            std::vector<std::pair<uint64_t, uint64_t>> seen, last_step, this_step;
            double line_gap = 1e300;
            int prev_mc = -1;
            g_cut_moves[10]++;
#endif
            [[maybe_unused]] bool moved = false;
            for (int i = 0; i < 36; ++i) sum[i] = sum[i] - L.invCov[i];
            while (L.cut[0] + L.cut[1] <= 1.0) {
                bool hit = false;
                double cand[2] = {0, 0};
                double cand_info[36];
                double metric_init = metric_back;
                CUT_STAT(g_cut_stats[1]++);   // steps
#ifdef GFPL_ORACLE_CUT_STATS
                double mv[8];
                int nv = 0;
#endif
#ifdef GFPL_ORACLE_CUT_STATS
                this_step.clear();
#endif
                for (int j = 0; j < 8; ++j) {
                    double rt[2] = {L.cut[0] + nb[j][0], L.cut[1] + nb[j][1]};
                    if (rt[0] + rt[1] > 1.0) continue;
                    if (rt[0] < cfg.cut_rng[0] || rt[0] > cfg.cut_rng[1]) continue;
                    if (rt[1] < cfg.cut_rng[0] || rt[1] > cfg.cut_rng[1]) continue;
#ifdef GFPL_ORACLE_CUT_STATS
                    g_cut_stats[2]++;   // valid evaluations
                    uint64_t k0, k1;
                    std::memcpy(&k0, &rt[0], 8); std::memcpy(&k1, &rt[1], 8);
                    bool dup = false;
                    for (auto& pr : seen) dup = dup || (pr.first == k0 && pr.second == k1);
                    if (!dup) { seen.push_back({k0, k1}); g_cut_stats[3]++; }   // distinct evaluations
                    // history limited to the previous step's evaluations
                    bool dup1 = false;
                    for (auto& pr : last_step) dup1 = dup1 || (pr.first == k0 && pr.second == k1);
                    if (!dup1) g_cut_stats[6]++;
                    this_step.push_back({k0, k1});
#endif
                    double tmp[36], tot[36];
                    poseInfoOnLine(DT_inv, Jl, L, rt, tmp);
                    for (int i = 0; i < 36; ++i) tot[i] = tmp[i] + sum[i];
                    double m = logdet6(tot);
#ifdef GFPL_ORACLE_CUT_STATS
                    mv[nv++] = m;
#endif
                    if (m > metric_init) {
                        metric_init = m;
                        cand[0] = rt[0]; cand[1] = rt[1];
                        std::memcpy(cand_info, tmp, sizeof tmp);
                        hit = true;
                    }
                }
#ifdef GFPL_ORACLE_CUT_STATS
                last_step = this_step;
                {   // the gaps the decision rests on: winner vs every other value and vs the centre
                    const double top = hit ? metric_init : metric_back;
                    double g = 1e300;
                    for (int i = 0; i < nv; ++i)
                        if (mv[i] != top) g = std::min(g, std::fabs(top - mv[i]));
                    if (hit) g = std::min(g, std::fabs(top - metric_back));
                    line_gap = std::min(line_gap, g);
                }
#endif
#ifdef GFPL_ORACLE_CUT_STATS
                if (hit) {
                    const int s0 = (cand[0] > L.cut[0]) - (cand[0] < L.cut[0]), s1 = (cand[1] > L.cut[1]) - (cand[1] < L.cut[1]);
                    const int mc = (s0 + 1) * 3 + (s1 + 1);
                    g_cut_moves[mc]++;
                    g_cut_paths.push_back((char)('0' + mc));
                    if ((s0 == 0) != (s1 == 0) && mc == prev_mc) g_cut_moves[9]++;
                    prev_mc = mc;
                }
#endif
                if (hit) {
                    CUT_STAT(if (cand[0] < L.cut[0] || cand[1] < L.cut[1]) g_cut_stats[7]++);   // a ratio moved back
                    L.cut[0] = cand[0]; L.cut[1] = cand[1];
                    std::memcpy(L.invCov, cand_info, sizeof cand_info);
                    metric_back = metric_init;
                    moved = true;
                } else break;
            }
#ifdef GFPL_ORACLE_CUT_STATS
            g_cut_paths.push_back('\n');
#endif
            CUT_STAT(if (!moved) g_cut_stats[4]++);   // lines that never moved
#ifdef GFPL_ORACLE_CUT_STATS
            {
                int b = line_gap > 0 ? (int)std::floor(std::log10(line_gap)) + 16 : 0;
                g_cut_gap_hist[std::max(0, std::min(19, b))]++;
            }
#endif
            CUT_STAT(prev_moved = moved);
            updateEndPointByRatio(L);
            for (int i = 0; i < 36; ++i) sum[i] = sum[i] + L.invCov[i];
        }
    }

    // ------------------------------------------------------------ pose ---
    // optimizeFunctions (src/stereoFrameHandler.cpp:2118-2245)
    void optimizeFunctions(const double* DT, double* H, double* g, double& e) const {
        double Hp[36] = {0}, Hl[36] = {0}, gp[6] = {0}, gl[6] = {0};
        double ep = 0.0, el = 0.0;
        int Np = 0, Nl = 0;
        for (int pi : matched_pt) {
            const PointF& p = prev->pt[pi];
            if (!p.inlier) continue;
            double Pc[3];
            se3_apply(DT, p.P, Pc);
            double uv[2];
            projection(Pc, uv);
            double ex = uv[0] - p.pl_obs[0], ey = uv[1] - p.pl_obs[1];
            double n = std::sqrt(ex * ex + ey * ey);
            double J[6];
            poseJac(Pc, ex, ey, J);
            double m = ref_max(cfg.homog_th, n);
            for (int i = 0; i < 6; ++i) J[i] = J[i] / m;
            double w = 1.0 / (1.0 + (n * n) * p.sigma2);
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) Hp[i * 6 + j] = Hp[i * 6 + j] + (J[i] * J[j]) * w;
            for (int i = 0; i < 6; ++i) gp[i] = gp[i] + (J[i] * n) * w;
            ep = ep + (n * n) * w;
            ++Np;
        }
        for (int li : matched_ls) {
            const LineF& L = prev->ls[li];
            if (!L.inlier) continue;
            double sc[3], ec[3], su[2], eu[2];
            se3_apply(DT, L.sP, sc);
            projection(sc, su);
            se3_apply(DT, L.eP, ec);
            projection(ec, eu);
            const double* lo = L.le_obs;
            double ds = (lo[0] * su[0] + lo[1] * su[1]) + lo[2];
            double de = (lo[0] * eu[0] + lo[1] * eu[1]) + lo[2];
            double n = std::sqrt(ds * ds + de * de);
            double Js[6], Je[6], J[6];
            poseJac(sc, lo[0], lo[1], Js);
            poseJac(ec, lo[0], lo[1], Je);
            double m = ref_max(cfg.homog_th, n);
            for (int i = 0; i < 6; ++i) J[i] = (Js[i] * ds + Je[i] * de) / m;
            double w = 1.0 / (1.0 + (n * n) * L.sigma2);
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) Hl[i * 6 + j] = Hl[i * 6 + j] + (J[i] * J[j]) * w;
            for (int i = 0; i < 6; ++i) gl[i] = gl[i] + (J[i] * n) * w;
            el = el + (n * n) * w;
            ++Nl;
        }
        for (int i = 0; i < 36; ++i) H[i] = Hp[i] + Hl[i];
        for (int i = 0; i < 6; ++i) g[i] = gp[i] + gl[i];
        e = ep + el;
        e = e / (double)(Nl + Np);
    }

    // gaussNewtonOptimization (src/stereoFrameHandler.cpp:2032-2056)
    void gaussNewton(double* DT, double* DT_cov, double& err_, int max_iters) const {
        double H[36] = {0}, g[6], inc[6];
        double err = 0.0, err_prev = 999999999.9;
        for (int it = 0; it < max_iters; ++it) {
            optimizeFunctions(DT, H, g, err);
            if ((std::fabs(err - err_prev) < cfg.min_error_change) || (err < cfg.min_error)) break;
            ldlt_solve6(H, g, inc);
            double E[16], Ei[16];
            expmap_se3(inc, E);
            inverse_se3(E, Ei);
            mat4_mul(DT, Ei, DT);
            double nrm = std::sqrt(((((inc[0] * inc[0] + inc[1] * inc[1]) + inc[2] * inc[2]) + inc[3] * inc[3]) + inc[4] * inc[4]) + inc[5] * inc[5]);
            if (nrm < DBL_EPSILON) break;
            err_prev = err;
        }
        inverse6(H, DT_cov);   // Q13: last evaluated H
        err_ = err;
    }

    // vector_stdv_mad (src/auxiliar.cpp:521-537)
    static double stdv_mad(std::vector<double> r) {
        if (r.empty()) return 0.0;
        int n = (int)r.size();
        std::sort(r.begin(), r.end());
        double median = r[n / 2];
        for (int i = 0; i < n; ++i) r[i] = (double)std::fabs((float)(r[i] - median));
        std::sort(r.begin(), r.end());
        return 1.4826 * r[n / 2];
    }

    // removeOutliers (src/stereoFrameHandler.cpp:2058-2116)
    void removeOutliers(const double* DT) {
        std::vector<double> rp, rl;
        for (int pi : matched_pt) {
            const PointF& p = prev->pt[pi];
            double Pc[3], uv[2];
            se3_apply(DT, p.P, Pc);
            projection(Pc, uv);
            double ex = uv[0] - p.pl_obs[0], ey = uv[1] - p.pl_obs[1];
            rp.push_back(std::sqrt(ex * ex + ey * ey) * std::sqrt(p.sigma2));
        }
        for (int li : matched_ls) {
            const LineF& L = prev->ls[li];
            double sc[3], ec[3], su[2], eu[2];
            se3_apply(DT, L.sP, sc);
            se3_apply(DT, L.eP, ec);
            projection(sc, su);
            projection(ec, eu);
            const double* lo = L.le_obs;
            double e0 = (lo[0] * su[0] + lo[1] * su[1]) + lo[2];
            double e1 = (lo[0] * eu[0] + lo[1] * eu[1]) + lo[2];
            rl.push_back(std::sqrt(e0 * e0 + e1 * e1) * std::sqrt(L.sigma2));
        }
        double th_p = cfg.inlier_k * stdv_mad(rp);
        double th_l = cfg.inlier_k * stdv_mad(rl);
        for (size_t k = 0; k < matched_pt.size(); ++k)
            if (rp[k] > th_p) { prev->pt[matched_pt[k]].inlier = false; --n_inliers; --n_inliers_pt; }
        for (size_t k = 0; k < matched_ls.size(); ++k)
            if (rl[k] > th_l) { prev->ls[matched_ls[k]].inlier = false; --n_inliers; --n_inliers_ls; }
    }

    // optimizePose(Matrix4d DT_ini) (src/stereoFrameHandler.cpp:1939-2030)
    void optimizePose(const double* DT_ini) {
        double DT_cov[36], DT[16], DT_[16];
        double err = 0.0;
        std::memcpy(DT, DT_ini, sizeof DT);
        std::memcpy(DT_cov, prev->DT_cov, sizeof DT_cov);
        auto reset = [&]() {
            for (int i = 0; i < 16; ++i) DT[i] = (i % 5 == 0) ? 1.0 : 0.0;
            for (int i = 0; i < 36; ++i) DT_cov[i] = 0.0;
        };
        if (n_inliers > cfg.min_features) {
            std::memcpy(DT_, DT, sizeof DT);
            gaussNewton(DT_, DT_cov, err, cfg.max_iters);
            if (is_finite16(DT_)) {
                removeOutliers(DT_);
                if (n_inliers > cfg.min_features) gaussNewton(DT, DT_cov, err, cfg.max_iters_ref);   // Q3
                else reset();
            } else reset();
        } else reset();
        Frame& C = *curr;
        if (is_finite16(DT)) {
            inverse_se3(DT, C.DT);
            double tn = std::sqrt((C.DT[3] * C.DT[3] + C.DT[7] * C.DT[7]) + C.DT[11] * C.DT[11]);
            if (tn < cfg.motion_step_th * (C.time_stamp - prev->time_stamp)) {
                mat4_mul(prev->Tfw, C.DT, C.Tfw);
                std::memcpy(C.DT_cov, DT_cov, sizeof DT_cov);
                eig_sym(DT_cov, 6, C.DT_cov_eig);
                unccomp_se3(prev->Tfw, prev->Tfw_cov, DT_cov, C.Tfw_cov);
                C.err_norm = err;
            } else {
                for (int i = 0; i < 16; ++i) C.DT[i] = (i % 5 == 0) ? 1.0 : 0.0;
                std::memcpy(C.Tfw, prev->Tfw, sizeof C.Tfw);
                std::memcpy(C.Tfw_cov, prev->Tfw_cov, sizeof C.Tfw_cov);
                std::memcpy(C.DT_cov, DT_cov, sizeof DT_cov);
                eig_sym(DT_cov, 6, C.DT_cov_eig);
                C.err_norm = -1.0;
            }
            numFrameLoss = 0;
        } else {
            for (int i = 0; i < 16; ++i) C.DT[i] = (i % 5 == 0) ? 1.0 : 0.0;
            std::memcpy(C.Tfw, prev->Tfw, sizeof C.Tfw);
            std::memcpy(C.Tfw_cov, prev->Tfw_cov, sizeof C.Tfw_cov);
            std::memcpy(C.DT_cov, DT_cov, sizeof DT_cov);
            eig_sym(DT_cov, 6, C.DT_cov_eig);
            C.err_norm = -1.0;
            ++numFrameLoss;
        }
    }
};

// ======================================================================= C ABI
namespace {
int init_cam(Cam& c, const gfpl_camera* cam, const gfpl_config* cfg) {
    c.width = cam->width; c.height = cam->height;
    c.fx = cam->fx; c.fy = cam->fy; c.cx = cam->cx; c.cy = cam->cy; c.b = cam->b;
    c.nlev = cfg->orb_n_levels;
    if (c.nlev < 1 || c.nlev > GFPL_MAX_LEVELS) return GFPL_E_INVALID;
    // ORBextractor ctor (src/ORBextractor.cc:410-431): float factor, double member
    const double sfm = (double)(float)cfg->orb_scale_factor;
    c.scale[0] = 1.0f;
    for (int i = 1; i < c.nlev; ++i) c.scale[i] = (float)((double)c.scale[i - 1] * sfm);
    for (int i = 0; i < c.nlev; ++i) c.inv[i] = 1.0f / c.scale[i];
    for (int i = 0; i < c.nlev; ++i) {
        // ComputePyramid sizes (src/ORBextractor.cc:1111-1113): cvRound((float)cols*scale)
        c.cols[i] = (int)std::lrint((double)((float)c.width * c.inv[i]));
        c.rows[i] = (int)std::lrint((double)((float)c.height * c.inv[i]));
        if (c.cols[i] != cam->lvl_cols[i] || c.rows[i] != cam->lvl_rows[i]) return GFPL_E_INVALID;
        c.off[i] = cam->lvl_offset[i];
        if (std::memcmp(&c.scale[i], &cam->scale[i], 4) || std::memcmp(&c.inv[i], &cam->inv_scale[i], 4))
            return GFPL_E_INVALID;
    }
    // PointFeature / LineFeature sigma2 (src/stereoFeatures.cpp:41-47,96-101)
    for (int l = 0; l < GFPL_MAX_LEVELS; ++l) {
        double s = 1.0;
        for (int i = 0; i < l + 1; ++i) s *= cfg->orb_scale_factor;
        c.sigma2_pt[l] = 1.f / (s * s);
        double t = 1.0;
        for (int i = 0; i < l + 1; ++i) t *= cfg->lsd_scale;
        c.sigma2_ln[l] = 1.f / (t * t);
    }
    return 0;
}

void put2(double* d, const double* s) { d[0] = s[0]; d[1] = s[1]; }
void put3(double* d, const double* s) { d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; }

void frame_to_host(const Frame& f, gfpl_frame_host* o) {
    o->n_pt = (int)f.pt.size();
    o->n_ls = (int)f.ls.size();
    for (size_t i = 0; i < f.pt.size(); ++i) {
        const PointF& p = f.pt[i];
        if (o->pt_pl) put2(o->pt_pl + 2 * i, p.pl);
        if (o->pt_pl_obs) put2(o->pt_pl_obs + 2 * i, p.pl_obs);
        if (o->pt_disp) o->pt_disp[i] = p.disp;
        if (o->pt_P) put3(o->pt_P + 3 * i, p.P);
        if (o->pt_sigma2) o->pt_sigma2[i] = p.sigma2;
        if (o->pt_idx) o->pt_idx[i] = p.idx;
        if (o->pt_level) o->pt_level[i] = p.level;
        if (o->pt_inlier) o->pt_inlier[i] = p.inlier ? 1 : 0;
        if (o->pdesc) std::memcpy(o->pdesc + 32 * i, f.pdesc[i].data(), 32);
    }
    for (size_t i = 0; i < f.ls.size(); ++i) {
        const LineF& L = f.ls[i];
        if (o->ls_spl) put2(o->ls_spl + 2 * i, L.spl);
        if (o->ls_epl) put2(o->ls_epl + 2 * i, L.epl);
        if (o->ls_spl_obs) put2(o->ls_spl_obs + 2 * i, L.spl_obs);
        if (o->ls_epl_obs) put2(o->ls_epl_obs + 2 * i, L.epl_obs);
        if (o->ls_sdisp) o->ls_sdisp[i] = L.sdisp;
        if (o->ls_edisp) o->ls_edisp[i] = L.edisp;
        if (o->ls_sdisp_obs) o->ls_sdisp_obs[i] = L.sdisp_obs;
        if (o->ls_edisp_obs) o->ls_edisp_obs[i] = L.edisp_obs;
        if (o->ls_angle) o->ls_angle[i] = L.angle;
        if (o->ls_sigma2) o->ls_sigma2[i] = L.sigma2;
        if (o->ls_sP) put3(o->ls_sP + 3 * i, L.sP);
        if (o->ls_eP) put3(o->ls_eP + 3 * i, L.eP);
        if (o->ls_le) put3(o->ls_le + 3 * i, L.le);
        if (o->ls_le_obs) put3(o->ls_le_obs + 3 * i, L.le_obs);
        if (o->ls_covS) std::memcpy(o->ls_covS + 9 * i, L.covS, sizeof L.covS);
        if (o->ls_covE) std::memcpy(o->ls_covE + 9 * i, L.covE, sizeof L.covE);
        if (o->ls_cut) put2(o->ls_cut + 2 * i, L.cut);
        if (o->ls_invcov) std::memcpy(o->ls_invcov + 36 * i, L.invCov, sizeof L.invCov);
        if (o->ls_idx) o->ls_idx[i] = L.idx;
        if (o->ls_level) o->ls_level[i] = L.level;
        if (o->ls_inlier) o->ls_inlier[i] = L.inlier ? 1 : 0;
        if (o->ldesc) std::memcpy(o->ldesc + 32 * i, f.ldesc[i].data(), 32);
    }
    std::memcpy(o->Tfw, f.Tfw, sizeof f.Tfw);
    std::memcpy(o->DT, f.DT, sizeof f.DT);
    std::memcpy(o->DT_cov, f.DT_cov, sizeof f.DT_cov);
    std::memcpy(o->Tfw_cov, f.Tfw_cov, sizeof f.Tfw_cov);
    std::memcpy(o->DT_cov_eig, f.DT_cov_eig, sizeof f.DT_cov_eig);
    o->err_norm = f.err_norm;
    o->time_stamp = f.time_stamp;
}

void host_to_frame(const gfpl_frame_host* o, Frame& f) {
    f.pt.assign(o->n_pt, PointF());
    f.pdesc.assign(o->n_pt, Desc());
    for (int i = 0; i < o->n_pt; ++i) {
        PointF& p = f.pt[i];
        put2(p.pl, o->pt_pl + 2 * i);
        put2(p.pl_obs, o->pt_pl_obs + 2 * i);
        p.disp = o->pt_disp[i];
        put3(p.P, o->pt_P + 3 * i);
        p.sigma2 = o->pt_sigma2[i];
        p.idx = o->pt_idx[i];
        p.level = o->pt_level[i];
        p.inlier = o->pt_inlier[i] != 0;
        std::memcpy(f.pdesc[i].data(), o->pdesc + 32 * i, 32);
    }
    f.ls.assign(o->n_ls, LineF());
    f.ldesc.assign(o->n_ls, Desc());
    for (int i = 0; i < o->n_ls; ++i) {
        LineF& L = f.ls[i];
        put2(L.spl, o->ls_spl + 2 * i);
        put2(L.epl, o->ls_epl + 2 * i);
        put2(L.spl_obs, o->ls_spl_obs + 2 * i);
        put2(L.epl_obs, o->ls_epl_obs + 2 * i);
        L.sdisp = o->ls_sdisp[i]; L.edisp = o->ls_edisp[i];
        L.sdisp_obs = o->ls_sdisp_obs[i]; L.edisp_obs = o->ls_edisp_obs[i];
        L.angle = o->ls_angle[i]; L.sigma2 = o->ls_sigma2[i];
        put3(L.sP, o->ls_sP + 3 * i);
        put3(L.eP, o->ls_eP + 3 * i);
        put3(L.le, o->ls_le + 3 * i);
        put3(L.le_obs, o->ls_le_obs + 3 * i);
        std::memcpy(L.covS, o->ls_covS + 9 * i, sizeof L.covS);
        std::memcpy(L.covE, o->ls_covE + 9 * i, sizeof L.covE);
        put2(L.cut, o->ls_cut + 2 * i);
        std::memcpy(L.invCov, o->ls_invcov + 36 * i, sizeof L.invCov);
        L.idx = o->ls_idx[i]; L.level = o->ls_level[i];
        L.inlier = o->ls_inlier[i] != 0;
        std::memcpy(f.ldesc[i].data(), o->ldesc + 32 * i, 32);
    }
    std::memcpy(f.Tfw, o->Tfw, sizeof f.Tfw);
    std::memcpy(f.DT, o->DT, sizeof f.DT);
    std::memcpy(f.DT_cov, o->DT_cov, sizeof f.DT_cov);
    std::memcpy(f.Tfw_cov, o->Tfw_cov, sizeof f.Tfw_cov);
    std::memcpy(f.DT_cov_eig, o->DT_cov_eig, sizeof f.DT_cov_eig);
    f.err_norm = o->err_norm;
    f.time_stamp = o->time_stamp;
}
}  // namespace

extern "C" {

gfplo_handler* gfplo_create(const gfpl_camera* cam, const gfpl_config* cfg) {
    if (!cam || !cfg) return nullptr;
    gfplo_handler* h = new gfplo_handler();
    h->cfg = *cfg;
    if (init_cam(h->cam, cam, cfg)) { delete h; return nullptr; }
    h->pyr_bytes = cam->pyr_bytes;
    return h;
}

void gfplo_destroy(gfplo_handler* h) {
    if (!h) return;
    delete h->prev;
    delete h->curr;
    delete h;
}

int gfplo_initialize(gfplo_handler* h, const gfpl_frames* in, int seq) {
    delete h->prev; delete h->curr;
    h->curr = nullptr;
    h->prev = new Frame();
    h->prev->in = in; h->prev->seq = seq;
    h->prev->time_stamp = in->time_stamp[seq];
    h->extractInitialStereoFeatures(*h->prev);
    for (int i = 0; i < 16; ++i) h->prev->Tfw[i] = h->prev->DT[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int i = 0; i < 36; ++i) h->prev->Tfw_cov[i] = (i % 7 == 0) ? 1.0 : 0.0;
    h->numFrameLoss = 0;
    // SLAM variables for KF decision (src/stereoFrameHandler.cpp:54-58); a fresh
    // handler also starts numFrameSinceKeyframe at 0 (include/stereoFrameHandler.h:147)
    for (int i = 0; i < 16; ++i) h->T_prevKF[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int i = 0; i < 36; ++i) h->cov_prevKF_currF[i] = 0.0;
    h->prev_f_iskf = true;
    h->numFrameSinceKeyframe = 0;
    h->entropy_first_prevKF = 0.0; h->entropy_ratio = 0.0; h->need_new_kf = 0;
    h->matched_pt.clear(); h->matched_ls.clear();
    h->prev->in = nullptr;
    return 0;
}

int gfplo_begin_frame(gfplo_handler* h, const gfpl_frames* in, int seq) {
    if (!h->prev) return GFPL_E_STATE;
    delete h->curr;
    h->curr = new Frame();
    h->curr->in_store = *in;
    h->curr->in = &h->curr->in_store; h->curr->seq = seq;
    h->curr->time_stamp = in->time_stamp[seq];
    return 0;
}
int gfplo_stereo_points(gfplo_handler* h) { if (!h->curr || !h->curr->in) return GFPL_E_STATE; h->stereoPoints(*h->curr); return 0; }
int gfplo_stereo_lines(gfplo_handler* h) { if (!h->curr || !h->curr->in) return GFPL_E_STATE; h->stereoLines(*h->curr); return 0; }
int gfplo_line_uncertainty(gfplo_handler* h) { if (!h->prev) return GFPL_E_STATE; h->estimateStereoUncertainty(*h->prev); return 0; }
int gfplo_cross_points(gfplo_handler* h) {
    if (!h->prev || !h->curr) return GFPL_E_STATE;
    h->predictFramePose();
    h->crossPoints();
    h->finishCounts();
    return 0;
}
int gfplo_cross_lines(gfplo_handler* h) {
    if (!h->prev || !h->curr) return GFPL_E_STATE;
    h->crossLines();
    h->finishCounts();
    return 0;
}
int gfplo_line_cut(gfplo_handler* h) { if (!h->prev || !h->curr) return GFPL_E_STATE; h->lineCut(); return 0; }

int gfplo_insert_stereo_pair(gfplo_handler* h, const gfpl_frames* in, int seq) {
    int e = gfplo_begin_frame(h, in, seq);
    if (e) return e;
    h->stereoPoints(*h->curr);
    h->stereoLines(*h->curr);
    h->curr->in = nullptr;
    h->predictFramePose();
    if (h->cfg.use_line_conf_cut) h->estimateStereoUncertainty(*h->prev);
    h->crossPoints();
    h->crossLines();
    h->finishCounts();
    if (h->cfg.use_line_conf_cut) h->lineCut();
    h->numFrameSinceKeyframe++;   // (:150)
    return 0;
}

int gfplo_need_new_kf(gfplo_handler* h, int* flag) {
    if (!h->prev || !h->curr) return GFPL_E_STATE;
    const bool f = h->needNewKF();
    if (flag) *flag = f ? 1 : 0;
    return 0;
}
int gfplo_curr_frame_is_kf(gfplo_handler* h) {
    if (!h->curr) return GFPL_E_STATE;
    h->currFrameIsKF();
    return 0;
}
int gfplo_read_kf_state(gfplo_handler* h, gfpl_kf_state* out) {
    if (!out) return GFPL_E_INVALID;
    std::memcpy(out->T_prevKF, h->T_prevKF, sizeof out->T_prevKF);
    std::memcpy(out->cov_prevKF_currF, h->cov_prevKF_currF, sizeof out->cov_prevKF_currF);
    out->entropy_first_prevKF = h->entropy_first_prevKF;
    out->entropy_ratio = h->entropy_ratio;
    out->prev_f_iskf = h->prev_f_iskf ? 1 : 0;
    out->num_frame_since_kf = h->numFrameSinceKeyframe;
    out->need_new_kf = h->need_new_kf;
    return 0;
}

int gfplo_optimize_pose(gfplo_handler* h) {
    if (!h->prev || !h->curr) return GFPL_E_STATE;
    double DT_ini[16];
    std::memcpy(DT_ini, h->prev->DT, sizeof DT_ini);   // Q2
    h->optimizePose(DT_ini);
    return 0;
}
/* optimizePose(Matrix4d DT_ini) with an explicit initial guess (row-major 4x4) */
int gfplo_optimize_pose_ini(gfplo_handler* h, const double* DT_ini) {
    if (!h->prev || !h->curr || !DT_ini) return GFPL_E_STATE;
    double D[16];
    std::memcpy(D, DT_ini, sizeof D);
    h->optimizePose(D);
    return 0;
}

int gfplo_update_frame(gfplo_handler* h) {
    if (!h->prev || !h->curr) return GFPL_E_STATE;
    delete h->prev;
    h->prev = h->curr;
    h->curr = nullptr;
    h->prev->in = nullptr;
    h->matched_pt.clear(); h->matched_ls.clear();
    return 0;
}

int gfplo_read_frame(gfplo_handler* h, int which, gfpl_frame_host* out) {
    Frame* f = which == GFPL_PREV ? h->prev : h->curr;
    if (!f || !out) return GFPL_E_STATE;
    frame_to_host(*f, out);
    return 0;
}
int gfplo_write_frame(gfplo_handler* h, int which, const gfpl_frame_host* in) {
    Frame*& f = which == GFPL_PREV ? h->prev : h->curr;
    if (!f) f = new Frame();
    f->in = nullptr;
    host_to_frame(in, *f);
    return 0;
}
int gfplo_read_track(gfplo_handler* h, gfpl_track_host* out) {
    out->n_matched_pt = (int)h->matched_pt.size();
    out->n_matched_ls = (int)h->matched_ls.size();
    for (size_t i = 0; i < h->matched_pt.size() && i < GFPL_MAX_MATCHED_PT; ++i) out->matched_pt[i] = h->matched_pt[i];
    for (size_t i = 0; i < h->matched_ls.size() && i < GFPL_MAX_MATCHED_LS; ++i) out->matched_ls[i] = h->matched_ls[i];
    out->n_inliers = h->n_inliers; out->n_inliers_pt = h->n_inliers_pt; out->n_inliers_ls = h->n_inliers_ls;
    out->num_frame_loss = h->numFrameLoss;
    return 0;
}
int gfplo_write_track(gfplo_handler* h, const gfpl_track_host* in) {
    h->matched_pt.assign(in->matched_pt, in->matched_pt + in->n_matched_pt);
    h->matched_ls.assign(in->matched_ls, in->matched_ls + in->n_matched_ls);
    h->n_inliers = in->n_inliers; h->n_inliers_pt = in->n_inliers_pt; h->n_inliers_ls = in->n_inliers_ls;
    h->numFrameLoss = in->num_frame_loss;
    return 0;
}

int gfplo_hamming(const uint8_t* a, const uint8_t* b, int cell) { return hamming(a, b, cell); }

// BFMatcher::radiusMatch rows (StereoFrame::matchPointFeatures_radius / matchLineFeatures_radius,
// src/stereoFrame.cpp:1243-1257): every train row with distance <= max_dist (ledger T1), sorted by
// distance; OpenCV's std::sort of DMatch leaves ties unspecified — pinned to train order (T2) by a
// stable sort.  row_off[nq + 1]; GFPL_E_CAPACITY (row_off filled) when the rows exceed cap.
int gfplo_radius_match(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, float max_dist, int32_t* row_off,
                       int cap, int32_t* out_idx, float* out_dist) {
    std::vector<std::vector<std::pair<int, float>>> rows(nq);
    row_off[0] = 0;
    for (int i = 0; i < nq; ++i) {
        for (int j = 0; j < nt; ++j) {
            const float d = (float)hamming(q + 32 * (size_t)i, t + 32 * (size_t)j, cell);
            if (d <= max_dist) rows[i].push_back(std::make_pair(j, d));
        }
        std::stable_sort(rows[i].begin(), rows[i].end(),
                         [](const std::pair<int, float>& a, const std::pair<int, float>& b) { return a.second < b.second; });
        row_off[i + 1] = row_off[i] + (int)rows[i].size();
    }
    if (row_off[nq] > cap) return GFPL_E_CAPACITY;
    for (int i = 0; i < nq; ++i)
        for (size_t k = 0; k < rows[i].size(); ++k) {
            out_idx[row_off[i] + k] = rows[i][k].first;
            out_dist[row_off[i] + k] = rows[i][k].second;
        }
    return 0;
}

// pointDescriptorMAD / lineDescriptorMAD + *DescriptorBudgetThres (src/stereoFrame.cpp:1259-1341) on a
// knn-2 list given as its best / second distances; the reference's std::sort calls restated with a
// total order (NaN above +inf, ledger U12; equal keys are interchangeable, so the element at a rank
// is the reference's), nn_dist_median pinned to 0.0 where the reference reads it uninitialised (U1).
namespace {
struct NanLast {
    bool operator()(float a, float b) const {
        if (a != a) return false;
        if (b != b) return true;
        return a < b;
    }
};
float kth(std::vector<float> v, size_t k) {
    std::sort(v.begin(), v.end(), NanLast());
    return v[k];
}
}  // namespace
int gfplo_match_stats(int kind, const float* d0, const float* d1, int n, int max_num, double* out) {
    if (n < 1 || max_num < 1 || (kind != 0 && kind != 1)) return GFPL_E_INVALID;
    const double nn_dist_median = 0.0;   // U1
    std::vector<float> v(n);
    for (int j = 0; j < n; ++j) v[j] = std::fabs((float)((double)d0[j] - nn_dist_median));
    out[0] = 1.4826 * (double)kth(v, n / 2);
    if (kind == 1) {   // lineDescriptorMAD :1287-1313
        for (int j = 0; j < n; ++j) v[j] = std::fabs((float)((double)(d1[j] - d0[j]) - nn_dist_median));
        out[1] = 1.4826 * (double)kth(v, n / 2);
    } else {           // pointDescriptorMAD :1259-1285: the ratio order is descending (NN12_ratio's >)
        for (int j = 0; j < n; ++j) v[j] = d0[j] / d1[j];
        const double med = (double)kth(v, (size_t)(n - 1 - n / 2));
        for (int j = 0; j < n; ++j) v[j] = std::fabs((float)((double)(d0[j] / d1[j]) - med));
        out[1] = 1.4826 * (double)kth(v, n / 2);
    }
    for (int j = 0; j < n; ++j) v[j] = d0[j];
    out[2] = (double)kth(v, (size_t)(std::min(max_num, n) - 1));   // :1315-1341
    return 0;
}

int gfplo_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, int32_t* out_idx, float* out_dist) {
    if (nt < 2) return GFPL_E_TOO_FEW_TRAIN;
    std::vector<Desc> Q(nq), T(nt);
    for (int i = 0; i < nq; ++i) std::memcpy(Q[i].data(), q + 32 * i, 32);
    for (int i = 0; i < nt; ++i) std::memcpy(T[i].data(), t + 32 * i, 32);
    std::vector<Knn2> m = knn2(Q, T, cell);
    for (int i = 0; i < nq; ++i) {
        out_idx[2 * i] = m[i][0].trainIdx; out_idx[2 * i + 1] = m[i][1].trainIdx;
        out_dist[2 * i] = m[i][0].distance; out_dist[2 * i + 1] = m[i][1].distance;
    }
    return 0;
}

double gfplo_log(double x) { return det_log(x); }
double gfplo_sin(double x) { return det_sin(x); }
double gfplo_cos(double x) { return det_cos(x); }
double gfplo_logdet6(const double* M) { return logdet6(M); }
int gfplo_ldlt_solve6(const double* H, const double* g, double* x) { ldlt_solve6(H, g, x); return 0; }
int gfplo_inverse6(const double* A, double* out) { inverse6(A, out); return 0; }
double gfplo_det6(const double* A) { return det6(A); }
int gfplo_inverse4(const double* A, double* out) { mat4_inv(A, out); return 0; }
int gfplo_eig_sym(const double* A, int n, double* w) { if (n < 1 || n > 6) return GFPL_E_INVALID; eig_sym(A, n, w); return 0; }
int gfplo_expmap_se3(const double* x, double* T) { expmap_se3(x, T); return 0; }
int gfplo_inverse_se3(const double* T, double* out) { inverse_se3(T, out); return 0; }

}  // extern "C"

/* line-cut work counters since the last call (analysis of the search shape):
 * lines, steps, valid evaluations, bit-distinct evaluations per line,
 * lines that never moved, setup logdets not implied by the previous line, (7) moves that
 * decrease a ratio */
extern "C" void gfplo_cut_stats(int64_t* out8) {
#ifdef GFPL_ORACLE_CUT_STATS
    for (int i = 0; i < 8; ++i) { out8[i] = g_cut_stats[i]; g_cut_stats[i] = 0; }
    for (int i = 0; i < 20; ++i) { fprintf(stderr, "%lld ", (long long)g_cut_gap_hist[i]); g_cut_gap_hist[i] = 0; }
    if (FILE* f = fopen("/tmp/gfplo_cut_paths.txt", "w")) { fputs(g_cut_paths.c_str(), f); fclose(f); }
    g_cut_paths.clear();
    fprintf(stderr, "\nmoves:");
    for (int i = 0; i < 11; ++i) { fprintf(stderr, " %lld", (long long)g_cut_moves[i]); g_cut_moves[i] = 0; }
    fprintf(stderr, "\n");
#else
    for (int i = 0; i < 8; ++i) out8[i] = -1;   // not compiled in
#endif
}

// ============================================== keyframe consumers ==
// MapHandler::lookForCommonMatches, keyframe-pair stage (src/mapHandler.cpp:199-470).
// has_refinement is false in the reference (:199), so the loop's only effect on
// tracking state is the list of accepted (kf0, kf1) pairs in pmatches_12 order
// (knnMatch output is already in query order; the sort by queryIdx at :241/:364
// is the identity).  Points :207-338, lines :340-470.
extern "C" int gfplo_kf_common_matches(const gfpl_camera* cam, const gfpl_config* cfg, const gfpl_kf_view* kf0,
                                       const gfpl_kf_view* kf1, int32_t* pt_pairs, int* n_pt_pairs,
                                       int32_t* ls_pairs, int* n_ls_pairs) {
    if (!cam || !cfg || !kf0 || !kf1 || !n_pt_pairs || !n_ls_pairs) return GFPL_E_INVALID;
    if (kf0->n_pt < 0 || kf1->n_pt < 0 || kf0->n_ls < 0 || kf1->n_ls < 0) return GFPL_E_INVALID;
    *n_pt_pairs = 0;
    *n_ls_pairs = 0;
    // DT = inverse_se3(kf1->T_kf_w) * kf0->T_kf_w (:196)
    double Ti[16], DT[16];
    inverse_se3(kf1->T_kf_w, Ti);
    mat4_mul(Ti, kf0->T_kf_w, DT);
    auto proj = [&](const double* P, double* uv) {   // PinholeStereoCamera::projection
        uv[0] = cam->cx + (cam->fx * P[0]) / P[2];
        uv[1] = cam->cy + (cam->fy * P[1]) / P[2];
    };
    auto descs = [](const uint8_t* d, int n) {
        std::vector<Desc> v(n);
        for (int i = 0; i < n; ++i) std::memcpy(v[i].data(), d + 32 * i, 32);
        return v;
    };
    const double chi = std::sqrt(7.815);
    // points (:207-338); U4: the second neighbour must exist on both sides
    if (kf0->n_pt >= 2 && kf1->n_pt >= 2) {
        if (!pt_pairs || !kf0->pdesc || !kf1->pdesc) return GFPL_E_INVALID;
        const std::vector<Desc> d0 = descs(kf0->pdesc, kf0->n_pt), d1 = descs(kf1->pdesc, kf1->n_pt);
        const std::vector<Knn2> m12 = knn2(d0, d1, 1), m21 = knn2(d1, d0, 1);
        int n = 0;
        for (size_t i = 0; i < m12.size(); ++i) {
            const int q = m12[i][0].queryIdx, t = m12[i][0].trainIdx;
            const int rl = m21[t][0].trainIdx;
            const double dist_12 = (double)(m12[i][0].distance / m12[i][1].distance);   // float / float
            if (q == rl && dist_12 <= cfg->max_ratio_12_p) {
                double Pc[3], uv[2];
                se3_apply(DT, kf0->P + 3 * q, Pc);
                proj(Pc, uv);
                const double ex = uv[0] - kf1->pl[2 * t], ey = uv[1] - kf1->pl[2 * t + 1];
                const double err = std::sqrt(ex * ex + ey * ey) * std::sqrt(kf0->pt_sigma2[q]);
                if (err < chi) { pt_pairs[2 * n] = q; pt_pairs[2 * n + 1] = t; ++n; }
            }
        }
        *n_pt_pairs = n;
    }
    // lines (:340-470)
    if (kf0->n_ls >= 2 && kf1->n_ls >= 2) {
        if (!ls_pairs || !kf0->ldesc || !kf1->ldesc) return GFPL_E_INVALID;
        const std::vector<Desc> d0 = descs(kf0->ldesc, kf0->n_ls), d1 = descs(kf1->ldesc, kf1->n_ls);
        const std::vector<Knn2> m12 = knn2(d0, d1, 1), m21 = knn2(d1, d0, 1);
        const double nn12_dist_th = lineDescriptorMAD_nn12(m12) * cfg->desc_th_l;
        int n = 0;
        for (size_t i = 0; i < m12.size(); ++i) {
            const int q = m12[i][0].queryIdx, t = m12[i][0].trainIdx;
            const int rl = m21[t][0].trainIdx;
            const double dist_12 = (double)(m12[i][1].distance - m12[i][0].distance);
            if (q == rl && dist_12 > nn12_dist_th) {
                double sc[3], ec[3], su[2], eu[2];
                se3_apply(DT, kf0->sP + 3 * q, sc);
                proj(sc, su);
                se3_apply(DT, kf0->eP + 3 * q, ec);
                proj(ec, eu);
                const double* l = kf0->le + 3 * q;
                const double e0 = (l[0] * su[0] + l[1] * su[1]) + l[2];
                const double e1 = (l[0] * eu[0] + l[1] * eu[1]) + l[2];
                if (std::sqrt(e0 * e0 + e1 * e1) * std::sqrt(kf0->ls_sigma2[q]) < chi) {
                    ls_pairs[2 * n] = q; ls_pairs[2 * n + 1] = t; ++n;
                }
            }
        }
        *n_ls_pairs = n;
    }
    return 0;
}

// MapHandler::lookForCommonMatches, local-map stage (src/mapHandler.cpp:472-772).
// map_local_points / map_local_lines = the caller's rows that project inside the
// image in front of the camera, in map order; kf1 is already compacted to its
// unmatched rows.  Pair = (caller's map row, kf1 row).
extern "C" int gfplo_kf_local_map_matches(const gfpl_camera* cam, const gfpl_config* cfg, const gfpl_map_view* map,
                                          const gfpl_kf_view* kf1, double max_kf_epip_p, double max_kf_epip_l,
                                          int32_t* pt_pairs, int* n_pt_pairs, int32_t* ls_pairs, int* n_ls_pairs) {
    if (!cam || !cfg || !map || !kf1 || !n_pt_pairs || !n_ls_pairs) return GFPL_E_INVALID;
    if (map->n_pt < 0 || map->n_ls < 0 || kf1->n_pt < 0 || kf1->n_ls < 0) return GFPL_E_INVALID;
    *n_pt_pairs = 0;
    *n_ls_pairs = 0;
    double Twf[16];
    inverse_se3(kf1->T_kf_w, Twf);   // :202
    auto proj = [&](const double* P, double* uv) {
        uv[0] = cam->cx + (cam->fx * P[0]) / P[2];
        uv[1] = cam->cy + (cam->fy * P[1]) / P[2];
    };
    auto inside = [&](const double* Pf, const double* pf) {   // :482 / :622-625
        return pf[0] > 0 && pf[0] < cam->width && pf[1] > 0 && pf[1] < cam->height && Pf[2] > 0.0;
    };
    auto descs = [](const uint8_t* d, const std::vector<int>& rows) {
        std::vector<Desc> v(rows.size());
        for (size_t i = 0; i < rows.size(); ++i) std::memcpy(v[i].data(), d + 32 * (size_t)rows[i], 32);
        return v;
    };
    std::vector<int> all1;
    // points (:472-562)
    {
        std::vector<int> loc;
        for (int i = 0; i < map->n_pt; ++i) {
            double Pf[3], pf[2];
            se3_apply(Twf, map->P + 3 * i, Pf);
            proj(Pf, pf);
            if (inside(Pf, pf)) loc.push_back(i);
        }
        if (loc.size() >= 2 && kf1->n_pt >= 2) {
            if (!pt_pairs) return GFPL_E_INVALID;
            std::vector<int> r1(kf1->n_pt);
            for (int i = 0; i < kf1->n_pt; ++i) r1[i] = i;
            const std::vector<Desc> d0 = descs(map->pdesc, loc), d1 = descs(kf1->pdesc, r1);
            const std::vector<Knn2> m12 = knn2(d0, d1, 1), m21 = knn2(d1, d0, 1);
            int n = 0;
            for (size_t i = 0; i < m12.size(); ++i) {
                const int q = m12[i][0].queryIdx, t = m12[i][0].trainIdx;
                const int rl = m21[t][0].trainIdx;
                const double dist_12 = (double)(m12[i][0].distance / m12[i][1].distance);
                if (q == rl && dist_12 <= cfg->max_ratio_12_p) {
                    double Pf[3], pf[2];
                    se3_apply(Twf, map->P + 3 * loc[q], Pf);
                    if (Pf[2] > 0.0) {
                        proj(Pf, pf);
                        const double ex = pf[0] - kf1->pl[2 * t], ey = pf[1] - kf1->pl[2 * t + 1];
                        if (std::sqrt(ex * ex + ey * ey) < max_kf_epip_p) {
                            pt_pairs[2 * n] = loc[q]; pt_pairs[2 * n + 1] = t; ++n;
                        }
                    }
                }
            }
            *n_pt_pairs = n;
        }
    }
    // lines (:611-772)
    {
        std::vector<int> loc;
        for (int i = 0; i < map->n_ls; ++i) {
            double sPf[3], ePf[3], spf[2], epf[2];
            se3_apply(Twf, map->L + 6 * i, sPf);
            proj(sPf, spf);
            se3_apply(Twf, map->L + 6 * i + 3, ePf);
            proj(ePf, epf);
            if (inside(sPf, spf) && inside(ePf, epf)) loc.push_back(i);
        }
        if (loc.size() >= 2 && kf1->n_ls >= 2) {
            if (!ls_pairs) return GFPL_E_INVALID;
            std::vector<int> r1(kf1->n_ls);
            for (int i = 0; i < kf1->n_ls; ++i) r1[i] = i;
            const std::vector<Desc> d0 = descs(map->ldesc, loc), d1 = descs(kf1->ldesc, r1);
            const std::vector<Knn2> m12 = knn2(d0, d1, 1), m21 = knn2(d1, d0, 1);
            const double nn12_dist_th = lineDescriptorMAD_nn12(m12) * cfg->desc_th_l;
            int n = 0;
            for (size_t i = 0; i < m12.size(); ++i) {
                const int q = m12[i][0].queryIdx, t = m12[i][0].trainIdx;
                const int rl = m21[t][0].trainIdx;
                const double dist_12 = (double)(m12[i][1].distance - m12[i][0].distance);
                if (q == rl && dist_12 > nn12_dist_th) {
                    double sc[3], ec[3], su[2], eu[2];
                    se3_apply(Twf, map->L + 6 * loc[q], sc);
                    proj(sc, su);
                    se3_apply(Twf, map->L + 6 * loc[q] + 3, ec);
                    proj(ec, eu);
                    if (sc[2] > 0.0 && ec[2] > 0.0) {
                        const double* l = kf1->le + 3 * t;
                        const double e0 = (l[0] * su[0] + l[1] * su[1]) + l[2];
                        const double e1 = (l[0] * eu[0] + l[1] * eu[1]) + l[2];
                        if (e0 < max_kf_epip_l && e1 < max_kf_epip_l) {
                            ls_pairs[2 * n] = loc[q]; ls_pairs[2 * n + 1] = t; ++n;
                        }
                    }
                }
            }
            *n_ls_pairs = n;
        }
    }
    return 0;
}
