// k_cut.hip — good-line-cut: estimateProjUncertainty_submodular(0.05, {0,1})
// (src/stereoFrameHandler.cpp:1618-1764) with getPoseInfoOnLine (:1342-1411),
// getPoseInfoPoint (:1414-1447), updateEndPointByRatio (:1451-1470) and logdet
// (include/linespec.h:43-56).
//
// The search is a serial chain over matched lines: each line's greedy search
// reads invCov_sum after all earlier lines were cut.  Three kernels:
//  k_cut_prep   (one wave / sequence) r = (0,0) infos of lines and points and
//               invCov_sum, each entry summed in list order (lines, then points)
//               by one lane over 64-entry chunks staged in LDS;
//  k_cut_search (8 sequences per wave, 8 lanes each) the greedy search, one step
//               of every chain per wave iteration (see the comment at the kernel);
//  k_cut_finish (parallel) full 6x6 info of the chosen ratio (invCovPose) and
//               the cut endpoints of every matched line.
// Only the lower triangle is carried through the search: LLT reads nothing
// else (ledger Q11).
#include "gfpl_kernels.hpp"

namespace gfpl {

struct LineCutData {
    double sP[3], eP[3], covS[9], covE[9], Jl[2];
};

// projected residual variance of one cut endpoint (src/stereoFrameHandler.cpp:1356-1369)
__device__ __forceinline__ double endpointVar(const DevCam& cam, const double* DT_inv, const double* Jl,
                                              const double* Pt, const double* cov) {
    double Jdt[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) Jdt[i * 3 + j] = DT_inv[i * 4 + j];
    double cur[3];
    se3_apply(DT_inv, Pt, cur);
    // getJacob3D_2D (src/stereoFrame.cpp:1394-1412)
    const double f = cam.fx, pz = cur[2], pz_2 = pz * pz;
    double Jp[9];
    Jp[0] = f / pz; Jp[3] = 0.0; Jp[6] = 0.0;
    Jp[1] = 0.0; Jp[4] = f / pz; Jp[7] = 0.0;
    Jp[2] = ((-f) * cur[0]) / pz_2;
    Jp[5] = ((-f) * cur[1]) / pz_2;
    Jp[8] = ((-f) * cam.b) / pz_2;
    double T1[6], T2[6], T3[6], M[4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T1[i * 3 + j] = (Jp[i * 3 + 0] * Jdt[0 * 3 + j] + Jp[i * 3 + 1] * Jdt[1 * 3 + j]) + Jp[i * 3 + 2] * Jdt[2 * 3 + j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T2[i * 3 + j] = (T1[i * 3 + 0] * cov[0 * 3 + j] + T1[i * 3 + 1] * cov[1 * 3 + j]) + T1[i * 3 + 2] * cov[2 * 3 + j];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T3[i * 3 + j] = (T2[i * 3 + 0] * Jdt[j * 3 + 0] + T2[i * 3 + 1] * Jdt[j * 3 + 1]) + T2[i * 3 + 2] * Jdt[j * 3 + 2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            M[i * 2 + j] = (T3[i * 3 + 0] * Jp[j * 3 + 0] + T3[i * 3 + 1] * Jp[j * 3 + 1]) + T3[i * 3 + 2] * Jp[j * 3 + 2];
    const double r0 = Jl[0] * M[0] + Jl[1] * M[2];
    const double r1 = Jl[0] * M[1] + Jl[1] * M[3];
    return r0 * Jl[0] + r1 * Jl[1];
}

// One cut endpoint of getPoseInfoOnLine (src/stereoFrameHandler.cpp:1350-1388):
// P = (1-c)*P0 + c*P1 with its covariance blend (1-c)^2*C0 + c^2*C1, the
// projected residual variance v and the pose Jacobian J of that endpoint.
// Start endpoint: (sP, eP, covS, covE, c0); end endpoint: (eP, sP, covE, covS, c1).
// The start terms depend on c0 only and the end terms on c1 only, which the
// search exploits.
__device__ __forceinline__ void cut_endpoint(const DevCam& cam, double homog, const double* DT_inv, const double* Jl,
                                             const double* P0, const double* P1, const double* C0, const double* C1,
                                             double c, double* out7) {
    double Pt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) Pt[k] = (1 - c) * P0[k] + c * P1[k];
    const double a = (1 - c) * (1 - c), q = c * c;
    double cov[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) cov[i] = a * C0[i] + q * C1[i];
    out7[0] = endpointVar(cam, DT_inv, Jl, Pt, cov);
    double cur[3];
    se3_apply(DT_inv, Pt, cur);
    poseJac(cam, homog, cur, Jl[0], Jl[1], out7 + 1);
}

// info = [Js Je] inv(diag(vs, ve)) [Js Je]^T, Eigen 2x2 inverse via invdet (ledger Q10)
// FULL -> 36 entries row-major, else lower triangle (21)
template <bool FULL>
__device__ __forceinline__ void cut_assemble(const double* S7, const double* E7, double* info) {
    const double vs = S7[0], ve = E7[0];
    const double* Js = S7 + 1;
    const double* Je = E7 + 1;
    const double det = vs * ve - 0.0 * 0.0;
    const double invdet = 1.0 / det;
    const double i00 = ve * invdet, i10 = -0.0 * invdet, i01 = -0.0 * invdet, i11 = vs * invdet;
    double T0[6], T1[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        T0[i] = Js[i] * i00 + Je[i] * i10;
        T1[i] = Js[i] * i01 + Je[i] * i11;
    }
    if (FULL) {
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) info[i * 6 + j] = T0[i] * Js[j] + T1[i] * Je[j];
    } else {
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) info[tri(i, j)] = T0[i] * Js[j] + T1[i] * Je[j];
    }
}

// getPoseInfoOnLine (src/stereoFrameHandler.cpp:1342-1411)
template <bool FULL>
__device__ __forceinline__ void poseInfoOnLine(const DevCam& cam, double homog, const double* DT_inv,
                                               const LineCutData& L, double c0, double c1, double* info) {
    double S7[7], E7[7];
    cut_endpoint(cam, homog, DT_inv, L.Jl, L.sP, L.eP, L.covS, L.covE, c0, S7);
    cut_endpoint(cam, homog, DT_inv, L.Jl, L.eP, L.sP, L.covE, L.covS, c1, E7);
    cut_assemble<FULL>(S7, E7, info);
}

__device__ __forceinline__ void load_line(const DevLines& L, size_t q, LineCutData& d) {
#pragma unroll
    for (int k = 0; k < 3; ++k) { d.sP[k] = L.sP[3 * q + k]; d.eP[k] = L.eP[3 * q + k]; }
#pragma unroll
    for (int k = 0; k < 9; ++k) { d.covS[k] = L.covS[9 * q + k]; d.covE[k] = L.covE[9 * q + k]; }
    d.Jl[0] = L.le_obs[3 * q];
    d.Jl[1] = L.le_obs[3 * q + 1];
}

// ------------------------------------------------------ fast cut endpoints --
// The certified comparisons (k_cut_search) need each endpoint's variance v and
// pose Jacobian J only to ~1e-14, so the search evaluates them in a shorter,
// non-reference order from per-line data:  DT is affine, so the transformed cut
// point is (1-c) DT P0 + c DT P1, and getPoseInfoOnLine's variance
// Jl^T Jp R cov R^T Jp^T Jl is u^T [(1-c)^2 R C0 R^T + c^2 R C1 R^T] u with
// u = Jp^T Jl = (Jl0 f/z, Jl1 f/z, -f (Jl0 x + Jl1 y)/z^2).  Per line (CUT_FAST):
// DT sP [3], DT eP [3], R covS R^T and R covE R^T (xx xy xz yy yz zz) [6+6], Jl [2],
// and (k_cut_prep) the list index of the line after it [1].
__device__ __forceinline__ void cut_fast_data(const double* Dl, const LineCutData& d, double* fd) {
    se3_apply(Dl, d.sP, fd);
    se3_apply(Dl, d.eP, fd + 3);
    const double* Cs[2] = {d.covS, d.covE};
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        double T[9];   // R C
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                T[i * 3 + k] = (Dl[i * 4 + 0] * Cs[w][0 * 3 + k] + Dl[i * 4 + 1] * Cs[w][1 * 3 + k]) + Dl[i * 4 + 2] * Cs[w][2 * 3 + k];
        const int ii[6] = {0, 0, 0, 1, 1, 2}, jj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
        for (int e = 0; e < 6; ++e)
            fd[6 + 6 * w + e] = (T[ii[e] * 3 + 0] * Dl[jj[e] * 4 + 0] + T[ii[e] * 3 + 1] * Dl[jj[e] * 4 + 1]) +
                                T[ii[e] * 3 + 2] * Dl[jj[e] * 4 + 2];
    }
    fd[18] = d.Jl[0];
    fd[19] = d.Jl[1];
}

// one endpoint from the fast data: g0/g1 the transformed points it blends, A0/A1
// the rotated covariances, t the cut ratio -> v, J[6]
__device__ __forceinline__ void cut_endpoint_fast(const DevCam& cam, double homog, const double* g0, const double* g1,
                                                  const double* A0, const double* A1, double jl0, double jl1, double t,
                                                  double* out7) {
    const double om = 1.0 - t;
    double g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) g[k] = __builtin_fma(om, g0[k], t * g1[k]);
    const double iz = 1.0 / g[2];
    const double fz = cam.fx * iz;
    const double u0 = jl0 * fz, u1 = jl1 * fz, u2 = -__builtin_fma(jl0, g[0], jl1 * g[1]) * fz * iz;
    auto quad = [&](const double* A) {
        const double diag = __builtin_fma(A[0] * u0, u0, __builtin_fma(A[3] * u1, u1, A[5] * u2 * u2));
        const double off = __builtin_fma(A[1] * u0, u1, __builtin_fma(A[2] * u0, u2, A[4] * u1 * u2));
        return __builtin_fma(2.0, off, diag);
    };
    out7[0] = __builtin_fma(om * om, quad(A0), t * t * quad(A1));
    poseJac(cam, homog, g, jl0, jl1, out7 + 1);
}

// ------------------------------------------------------------------ prep --
#ifndef GFPL_PREP_WAVES
#define GFPL_PREP_WAVES 1
#endif
__global__ void __launch_bounds__(64, GFPL_PREP_WAVES) k_cut_prep(KParams p) {
    __shared__ double chunk[21][65];   // lower-triangle infos of 64 list entries (padded row: lanes read 21 rows)
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int nls = p.tr.n_matched_ls[b];
    const int npt = p.tr.n_matched_pt[b];
    if (nls == 0) return;
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    DevLines& L = p.prev.ls;
    const DevPoints& P = p.prev.pt;
    const size_t lb = (size_t)b * p.kl_cap, pbase = (size_t)b * p.kp_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    const int32_t* mpt = p.tr.matched_pt + (size_t)b * p.mpt_cap;
    double* scr_l = p.scr.cut_ls + (size_t)b * p.mls_cap * 21;
    double* fast_l = p.scr.cut_fast + (size_t)b * p.mls_cap * CUT_FAST;
    // DT_inv = curr.Tfw^-1 * prev.Tfw (src/stereoFrameHandler.cpp:1635), every lane
    double Dl[16];
    {
        double Tc[16], Tp[16], Ti[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) { Tc[i] = p.curr.pose.Tfw[16 * b + i]; Tp[i] = p.prev.pose.Tfw[16 * b + i]; }
        mat4_inv(Tc, Ti);
        mat4_mul(Ti, Tp, Dl);
    }
    if (lane < 16) p.scr.cut_dtinv[16 * b + lane] = Dl[lane];
    // invCov_sum: lines then points, each entry summed in list order by lane e < 21,
    // 64 list entries at a time staged through LDS (src/stereoFrameHandler.cpp:1640-1657)
    double s = 0.0;
    const int nl_ch = (nls + 63) >> 6, np_ch = (npt + 63) >> 6;
    for (int c = 0; c < nl_ch + np_ch; ++c) {
        const bool lines = c < nl_ch;
        const int m = ((lines ? c : c - nl_ch) << 6) + lane;
        const int cnt = min(64, (lines ? nls : npt) - (((lines ? c : c - nl_ch)) << 6));
        double info[21];
        if (lane < cnt) {
            if (lines) {
                LineCutData d;
                load_line(L, lb + mls[m], d);
                poseInfoOnLine<false>(cam, homog, Dl, d, 0.0, 0.0, info);
#pragma unroll
                for (int i = 0; i < 21; ++i) scr_l[(size_t)m * 21 + i] = info[i];   // k_cut_search subtracts it
                double fd[CUT_FAST];
                cut_fast_data(Dl, d, fd);
                fd[CUT_FAST - 1] = (double)mls[min(m + 1, nls - 1)];   // k_cut_search's next-next line
#pragma unroll
                for (int i = 0; i < CUT_FAST; ++i) fast_l[(size_t)m * CUT_FAST + i] = fd[i];
            } else {
                const size_t q = pbase + mpt[m];
                double Pp[3] = {P.P[3 * q], P.P[3 * q + 1], P.P[3 * q + 2]};
                double cur[3], uv[2];
                se3_apply(Dl, Pp, cur);
                projection(cam, cur, uv);
                const double dx = uv[0] - P.pl_obs[2 * q], dy = uv[1] - P.pl_obs[2 * q + 1];
                double J[6];
                poseJac(cam, homog, cur, dx, dy, J);   // getPoseInfoPoint (:1414-1447)
#pragma unroll
                for (int i = 0; i < 6; ++i)
#pragma unroll
                    for (int j = 0; j <= i; ++j) info[tri(i, j)] = J[i] * J[j];
            }
#pragma unroll
            for (int i = 0; i < 21; ++i) chunk[i][lane] = info[i];
        }
        __syncthreads();
        if (lane < 21)
            for (int k = 0; k < cnt; ++k) s = s + chunk[lane][k];
        __syncthreads();
    }
    if (lane < 21) p.scr.cut_sum[24 * b + lane] = s;
}

// ---------------------------------------------------------------- search --
// 8 sequences per wave, 8 lanes each; every wave iteration is one greedy step
// of each of its 8 chains.
//
// Certified comparisons.  Within line m the search compares
// logdet(S + info(t0, t1)) over neighbours, S = invCov_sum - info_m(0, 0) fixed
// for the line, and info = Js Js^T / vs + Je Je^T / ve (rank 2, ledger Q10).  By
// the matrix determinant lemma logdet(S + info) = logdet(S) + log d with
//   d = (1 + as)(1 + ae) - c^2 / (vs ve),  as = |ws|^2 / vs, ae = |we|^2 / ve,
//   c = ws . we,  ws = L^-1 Js, we = L^-1 Je,  S = L L^T,
// so the step's decision (the reference's first strict maximum over the valid
// neighbours, starting from the centre's metric) only needs the d values: ws and
// as depend on t0 only, we and ae on t1 only, and a neighbour costs one 6-term
// dot product instead of a 6x6 LLT and six logs.  The decision is accepted when
// every comparison it rests on is separated by more than cfg.cut_certify
// (relative, 1e-9) — four orders of magnitude above the measured disagreement
// between d and the reference's own LLT arithmetic (<= 1e-13).
// Otherwise (and whenever S or an endpoint is not healthy) the group evaluates
// that step exactly as the reference does: neighbour j's info assembled from its
// endpoints, + S, LLT, six fdlibm logs, against the exact centre metric.  Either
// way the chosen ratios are the reference's; the metric values themselves are
// never output.
//
// Phases (wave barriers between them):
//   E1  lanes 0-2 compute the start endpoint at t0 = r0 + {-s, 0, +s}, lanes 3-5
//       the end endpoint at t1 = r1 + {-s, 0, +s} (cut_endpoint); lane 6 factors
//       S when the line just opened;
//   E2  lanes 0-5: w = L^-1 J and a = |w|^2 / v of their endpoint;
//   C   lane j: d of neighbour j; every lane: d of the centre;
//   D   certified decision, or the exact evaluation of the step (X) when any
//       group of the wave needs it; no improvement finalises the line:
//       invCov_sum += info of the chosen ratio (re-assembled from the middle
//       endpoints, the same arithmetic as the chosen candidate's), the cut
//       ratio is stored and the next line opens at (0, 0).
#define CUT_G 8          // sequences per wave (8 lanes each)
#define CUT_SL 15        // endpoint slot: v, J[6], w[6], a, (pad)
#define CUT_EP 91        // per-group endpoint block: 6 slots + 1 (odd stride)
#define CUT_CH 29        // per-group factor of S: L (21), 1/L_kk (6), ok, (pad)

__device__ __forceinline__ double nb_step(int j, int side, double st) {
    // neighbour j of (r0, r1) (src/stereoFrameHandler.cpp:1624-1633)
    const int a = side == 0 ? ((j == 0 || j == 4 || j == 5) ? 1 : ((j == 1 || j == 6 || j == 7) ? -1 : 0))
                            : ((j == 2 || j == 4 || j == 6) ? 1 : ((j == 3 || j == 5 || j == 7) ? -1 : 0));
    return a > 0 ? st : (a < 0 ? -st : 0.0);
}
__device__ __forceinline__ int nb_slot(int j, int side) {   // endpoint slot: 0: -s, 1: 0, 2: +s
    if (side == 0) return (j == 0 || j == 4 || j == 5) ? 2 : ((j == 1 || j == 6 || j == 7) ? 0 : 1);
    return (j == 2 || j == 4 || j == 6) ? 2 : ((j == 3 || j == 5 || j == 7) ? 0 : 1);
}

// S = L L^T for the certified comparisons (out: L strictly lower 21, 1/L_kk 6, ok).  ok = 0
// unless every pivot keeps at least GFPL_CUT_MIN_PIVOT (1e-2) of its diagonal; the line
// is then searched with exact steps only.  The pivot ratios bound the condition of the
// diagonally scaled S, which sets both the lemma's and the reference LLT's rounding
// error; above 1e-2 the measured disagreement stays <= 1e-13 (the
// synthetic, KITTI and EuRoC workloads stay above 0.1), four orders below the margin.
#ifndef GFPL_CUT_MIN_PIVOT
#define GFPL_CUT_MIN_PIVOT 1e-2
#endif
__device__ __forceinline__ void chol_s(const double* a, double* out) {
    double L[21];
#pragma unroll
    for (int i = 0; i < 21; ++i) L[i] = a[i];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double akk = L[tri(k, k)];
        double x = akk;
#pragma unroll
        for (int j = 0; j < k; ++j) x = x - L[tri(k, j)] * L[tri(k, j)];
        if (!(x > GFPL_CUT_MIN_PIVOT * akk && akk < 1e300)) { ok = false; x = 1.0; }
        // 1 / L_kk (the only use of the pivot): hardware rsq + two Newton steps
        double r = __builtin_amdgcn_rsq(x);
        r = r * (1.5 - (0.5 * x) * (r * r));
        r = r * (1.5 - (0.5 * x) * (r * r));
        L[tri(k, k)] = 0.0;
        out[21 + k] = r;
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            double v = L[tri(i, k)];
#pragma unroll
            for (int j = 0; j < k; ++j) v = v - L[tri(i, j)] * L[tri(k, j)];
            L[tri(i, k)] = v * r;
        }
    }
#pragma unroll
    for (int i = 0; i < 21; ++i) out[i] = L[i];
    out[27] = ok ? 1.0 : 0.0;
}

// Reciprocal for the certified comparisons only (never for an output or an exact
// step): hardware v_rcp_f64 refined by two Newton steps, within an ulp or two of 1/x;
// 0, infinities and NaN come out NaN or infinite and fail the health tests.
__device__ __forceinline__ double rcp_fast(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
    return r;
}

// d of the neighbour whose endpoints sit in slots S, E (NaN when not usable)
__device__ __forceinline__ double cut_d(const double* S, const double* E) {
    double c = S[7] * E[7];
#pragma unroll
    for (int i = 1; i < 6; ++i) c = __builtin_fma(S[7 + i], E[7 + i], c);
    const double vs = S[0], ve = E[0];
    const double d = __builtin_fma(1.0 + S[13], 1.0 + E[13], -(c * c) * rcp_fast(vs * ve));
    return (vs > 0.0 && ve > 0.0 && d > 0.0 && d < 1e300) ? d : __longlong_as_double(0x7ff8000000000000ll);
}

// ---- polynomial form of the certified-comparison terms.
// Along a side the cut point is g(t) = g0 + t (g1 - g0) (camera frame), so
// J(t) = fgz2(t) P(t) with P quadratic in t and fgz2 = fx / gz^2 (lines whose
// segment keeps gz^2 above homog_th; others are searched with exact steps), and
// v(t) = fgz2(t)^2 v'(t) with v'(t) = p^T ((1-t)^2 A0 + t^2 A1) p,
// p = (jl0 gz, jl1 gz, -(jl0 gx + jl1 gy)).  The factors fgz2 cancel in the
// determinant lemma: a = |L^-1 P|^2 / v' and c^2 / (vs ve) = (Ws . We)^2 / (v's v'e)
// with W(t) = L^-1 P(t) = W0 + t W1 + t^2 W2, whose coefficients are solved once
// when the line opens (lane j < 6: side j / 3, power j % 3).  A step then costs no
// triangular solve and no division but one reciprocal.
__device__ __forceinline__ void cut_poly_coeff(const double* g0, const double* g1, double lx, double ly, int k,
                                               double* Pk) {
    const double dx = g1[0] - g0[0], dy = g1[1] - g0[1], dz = g1[2] - g0[2];
    // coefficient k of the product (a0 + t a1)(b0 + t b1)
    auto prod = [&](double a0, double a1, double b0, double b1) {
        return k == 0 ? a0 * b0 : (k == 1 ? a0 * b1 + a1 * b0 : a1 * b1);
    };
    auto lin = [&](double a0, double a1) { return k == 0 ? a0 : (k == 1 ? a1 : 0.0); };
    const double x0 = g0[0], y0 = g0[1], z0 = g0[2];
    Pk[0] = lx * lin(z0, dz);
    Pk[1] = ly * lin(z0, dz);
    Pk[2] = -(lx * lin(x0, dx) + ly * lin(y0, dy));
    Pk[3] = -((lx * prod(x0, dx, y0, dy) + ly * prod(y0, dy, y0, dy)) + ly * prod(z0, dz, z0, dz));
    Pk[4] = (lx * prod(x0, dx, x0, dx) + lx * prod(z0, dz, z0, dz)) + ly * prod(x0, dx, y0, dy);
    Pk[5] = ly * prod(x0, dx, z0, dz) - lx * prod(y0, dy, z0, dz);
}

// The reference's evaluation of one step (X): neighbour j's metric logdet(info_j + S)
// and the centre metric — logdet(invCov_sum) on a line's first step (:1671), else the
// previous step's chosen candidate re-evaluated (same operands, same bits).  Out of
// line: it is rare, and inlined its two 6x6 LLTs would set the register budget of
// the whole search loop.
__device__ __attribute__((noinline)) double cut_exact_step(const double* sj, const double* ej, const double* s1,
                                                           const double* e4, const double* S, const double* Sb,
                                                           int first, double* mc) {
    double tot[21], tmp[21];
    cut_assemble<false>(sj, ej, tmp);
#pragma unroll
    for (int i = 0; i < 21; ++i) tot[i] = tmp[i] + S[i];
    const double vj = logdet6_lower(tot);
    if (first) {
#pragma unroll
        for (int i = 0; i < 21; ++i) tot[i] = Sb[i];
    } else {
        cut_assemble<false>(s1, e4, tmp);
#pragma unroll
        for (int i = 0; i < 21; ++i) tot[i] = tmp[i] + S[i];
    }
    *mc = logdet6_lower(tot);
    return vj;
}

// Group-of-8 exchange on the DPP crossbar (no LDS): xor 1, xor 2 (quad_perm) and
// the half-row mirror (lane i <-> 7 - i) pair every lane of a group in 3 steps.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
#define DPP_XOR1 0xB1
#define DPP_XOR2 0x4E
#define DPP_HALF_MIRROR 0x141

// The reference's j-loop "if (m > metric_init)" over the group's 8 lanes: the
// largest value, ties to the lowest j, NaN / invalid never chosen; -1 unless it
// beats the centre metric mc.  (v, j) ends up identical in all 8 lanes.
template <int CTRL>
__device__ __forceinline__ void argmax_step(double& v, int& k) {
    const double ov = dpp_f64<CTRL>(v);
    const int ok = dpp_i32<CTRL>(k);
    if (ov > v || (ov == v && ok < k)) { v = ov; k = ok; }
}
__device__ __forceinline__ int group_first_max(double v, int valid, int j, double mc, double& top) {
    double x = (valid && v == v) ? v : -__builtin_inf();
    int k = valid && v == v ? j : 8;
    argmax_step<DPP_XOR1>(x, k);
    argmax_step<DPP_XOR2>(x, k);
    argmax_step<DPP_HALF_MIRROR>(x, k);
    top = x;
    return (k < 8 && x > mc) ? k : -1;
}

// The search block is one wave: LDS accesses of a wave execute in order, so a
// phase boundary only has to keep the compiler from moving LDS accesses across
// it and drain the wave's LDS queue — unlike __syncthreads it does not wait for
// the in-flight global prefetch loads.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Per iteration (one LDS sync between the halves, one at the end):
//   A  lanes 0-2: the start endpoint at t0 = r0 + {-s, 0, +s}, lanes 3-5: the end
//      endpoint at t1 = r1 + {-s, 0, +s} (cut_endpoint), then w = L^-1 J and
//      a = |w|^2 / v of that endpoint; prefetched line data lands in LDS;
//   B  lane j: d of neighbour j and of the centre, the group decision by DPP
//      reduction, its certification by ballot; the exact step (X) when any
//      group of the wave needs it; a move, or the line's finalisation.
__global__ void __launch_bounds__(64) k_cut_search(KParams p) {
    // per-group rows padded to odd strides so the 8 groups of a wave sit in
    // different LDS banks when their lanes read the same entry
    __shared__ double sumA[CUT_G][25];   // approximate S of the current line
    __shared__ double sumE[CUT_G][25];   // exact invCov_sum before line m_sync (lazy, for exact steps)
    __shared__ double wpl[CUT_G][37];    // W(t) coefficients of the current line: [side * 3 + power][6]
    __shared__ double epf[CUT_G][CUT_EP];
    __shared__ double fst[CUT_G][21];    // fast data of the current line
    __shared__ double nxt[CUT_G][43];    // prefetched next line: fast data (21) | r = 0 info (21)
    __shared__ double xs[CUT_G][25];     // exact step: exact S of the line / flush endpoints
    __shared__ double dtl[CUT_G][13];    // DT_inv rows 0-2
    const int lane = threadIdx.x;
    const int g = lane >> 3, j = lane & 7;
    const int b = blockIdx.x * CUT_G + g;
    const bool live = b < p.B;
    const int nls = live ? p.tr.n_matched_ls[b] : 0;
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    const double tau = p.cfg.cut_certify;
    DevLines& L = p.prev.ls;
    const size_t lb = (size_t)(live ? b : 0) * p.kl_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)(live ? b : 0) * p.mls_cap;
    const double* scr_l = p.scr.cut_ls + (size_t)(live ? b : 0) * p.mls_cap * 21;
    const double* fast_l = p.scr.cut_fast + (size_t)(live ? b : 0) * p.mls_cap * CUT_FAST;
    for (int i = j; i < 12; i += 8) dtl[g][i] = live && nls > 0 ? p.scr.cut_dtinv[16 * b + i] : 0.0;
    const double* Dl = dtl[g];
    const double st = p.cfg.cut_step;
    const double rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    // E role of this lane: lanes 0-2 start endpoint (blend sP -> eP), 3-5 end (eP -> sP)
    const int eside = j < 3 ? 0 : 1;
    const double eoff = (j % 3) == 0 ? -st : ((j % 3) == 2 ? st : 0.0);
    double* my_slot = &epf[g][CUT_SL * (j < 6 ? j : 0)];
    const double* G0 = &fst[g][eside ? 3 : 0];
    const double* G1 = &fst[g][eside ? 0 : 3];
    const double* A0 = &fst[g][eside ? 12 : 6];
    const double* A1 = &fst[g][eside ? 6 : 12];
    // C role: neighbour j
    const double nb0 = nb_step(j, 0, st), nb1 = nb_step(j, 1, st);
    const int cs = nb_slot(j, 0), ce = 3 + nb_slot(j, 1);
    const unsigned long long gmask = 0xFFull << (8 * g);
    // group state (identical in the 8 lanes of a group)
    int m = 0;
    int m_sync = 0;      // sumE holds the exact invCov_sum before line m_sync
    int first = 1;       // first step of the line: the exact centre metric is logdet(invCov_sum)
    double r0 = 0.0, r1 = 0.0;
    int line_ok = 0;     // certified comparisons allowed on the current line
    // A line opens: every lane factors S in registers (identical values), then lane
    // j < 6 solves the W(t) coefficient of side j / 3, power j % 3 from the line's
    // fast data fd.  Certification needs the factor healthy and gz^2 > homog_th along
    // the segment (fgz2 = fx / gz^2 on it); otherwise the line takes exact steps.
    auto open_line = [&](const double* s21, const double* fd) {
        double o[28];
        chol_s(s21, o);
        const double z0 = fd[2], z1 = fd[5];
        line_ok = (o[27] != 0.0) && ((z0 > 0.0 && z1 > 0.0) || (z0 < 0.0 && z1 < 0.0)) &&
                  z0 * z0 > 2.0 * homog && z1 * z1 > 2.0 * homog;
        if (j < 6) {
            double P[6], w[6];
            cut_poly_coeff(fd + (eside ? 3 : 0), fd + (eside ? 0 : 3), fd[18], fd[19], j % 3, P);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double u = P[i];
#pragma unroll
                for (int k = 0; k < i; ++k) u = __builtin_fma(-o[tri(i, k)], w[k], u);
                w[i] = u * o[21 + i];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) wpl[g][6 * j + i] = w[i];
        }
    };
    // Next-line prefetch: lane j loads elements j, j+8, ... of the 42-element vector
    // [fast data (its last entry: the list index of the line after it) | r = 0 info]
    // of the group's next line right after a line opens; the values land in LDS one
    // iteration later.  Every load is a plain f64 load whose value reaches its use
    // through LDS, so nothing waits for it before that store.
    size_t q_cur = 0, q_nx = 0;
    double pf[6];
    int pending = 0;
    auto pf_issue = [&](int mm) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int e = j + 8 * k;
            pf[k] = e < CUT_FAST ? fast_l[(size_t)mm * CUT_FAST + e]
                                 : scr_l[(size_t)mm * 21 + (size_t)(e < 42 ? e - CUT_FAST : 0)];
        }
        pending = 1;
    };
    if (m < nls) {
        q_cur = lb + mls[0];
        if (nls > 1) q_nx = lb + mls[1];
        double fd0[CUT_FAST];
#pragma unroll
        for (int e = 0; e < CUT_FAST; ++e) fd0[e] = fast_l[e];
        for (int e = j; e < CUT_FAST; e += 8) fst[g][e] = fd0[e];
        double s21[21];
#pragma unroll
        for (int e = 0; e < 21; ++e) {
            const double s0 = p.scr.cut_sum[24 * b + e];
            s21[e] = s0 - scr_l[e];
            sumE[g][e] = s0;
            sumA[g][e] = s21[e];
        }
        open_line(s21, fd0);
        if (nls > 1) pf_issue(1);
    } else {
        for (int e = j; e < CUT_FAST; e += 8) fst[g][e] = (e == 2 || e == 5) ? 1.0 : 0.0;
    }
    __syncthreads();
#ifdef GFPL_CUT_PROF
    unsigned long long cp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, cp_last = clock64(), cp_it = 0, cp_fin = 0;
#define CUT_PROF(k) { const unsigned long long _t = clock64(); cp_acc[k] += _t - cp_last; cp_last = _t; }
#else
#define CUT_PROF(k)
#endif
    while (__any(m < nls)) {   // wave-uniform loop; groups that are done idle
        const bool act = m < nls;
        // ---- A: this lane's endpoint terms for the certified comparisons (polynomial
        //      form, see cut_poly_coeff): v' (slot 0), W (slots 7-12), a = |W|^2 / v' (13)
        if (j < 6) {
            const double t = (eside == 0 ? r0 : r1) + eoff;
            const double om = 1.0 - t;
            double gv[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) gv[k] = __builtin_fma(om, G0[k], t * G1[k]);
            const double jl0 = fst[g][18], jl1 = fst[g][19];
            const double p0 = jl0 * gv[2], p1 = jl1 * gv[2], p2 = -__builtin_fma(jl0, gv[0], jl1 * gv[1]);
            auto quad = [&](const double* A) {
                const double diag = __builtin_fma(A[0] * p0, p0, __builtin_fma(A[3] * p1, p1, A[5] * p2 * p2));
                const double off = __builtin_fma(A[1] * p0, p1, __builtin_fma(A[2] * p0, p2, A[4] * p1 * p2));
                return __builtin_fma(2.0, off, diag);
            };
            const double v = __builtin_fma(om * om, quad(A0), t * t * quad(A1));
            const double* Wc = &wpl[g][18 * eside];
            double w[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) w[i] = __builtin_fma(t, __builtin_fma(t, Wc[12 + i], Wc[6 + i]), Wc[i]);
            double a = w[0] * w[0];
#pragma unroll
            for (int i = 1; i < 6; ++i) a = __builtin_fma(w[i], w[i], a);
            my_slot[0] = v;
#pragma unroll
            for (int i = 0; i < 6; ++i) my_slot[7 + i] = w[i];
            my_slot[13] = a * rcp_fast(v);
        }
        // the prefetched next line lands in LDS (its loads were issued >= 1 iteration ago)
        if (pending) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (j + 8 * k < 42) nxt[g][j + 8 * k] = pf[k];
            pending = 0;
        }
        wave_lds_sync();
        CUT_PROF(0);
        // ---- B: d of neighbour j and of the centre; certified group decision
        const double t0 = r0 + nb0, t1 = r1 + nb1;
        int valid = act ? 1 : 0;
        if (t0 + t1 > 1.0) valid = 0;
        if (t0 < rlo || t0 > rhi) valid = 0;
        if (t1 < rlo || t1 > rhi) valid = 0;
        const double dj = cut_d(&epf[g][CUT_SL * cs], &epf[g][CUT_SL * ce]);
        const double dc = cut_d(&epf[g][CUT_SL * 1], &epf[g][CUT_SL * 4]);
        double top;
        int best = group_first_max(dj, valid, j, dc, top);
        // every comparison the decision rests on must clear the margin; NaN
        // (unhealthy) values fail every test
        int ok = 1;
        if (best >= 0) {
            if (valid && j != best && !(top - dj > tau * top)) ok = 0;
            if (!(top - dc > tau * top)) ok = 0;
        } else {
            if (valid && !(dc - dj > tau * dc)) ok = 0;
        }
        if (!(tau > 0.0 && line_ok && dc == dc)) ok = 0;
        const bool exact = act && (__ballot(!ok) & gmask) != 0;
        CUT_PROF(1);
        if (__any(exact)) {
            // ---- X: the reference's evaluation of this step for the groups that need it.
            // 1. the exact invCov_sum is brought up to line m (lines m_sync .. m-1 at
            //    their final ratios, one line per round: lanes 0 / 1 its start / end
            //    endpoint, then every lane the reference's sum chain)
            while (__any(exact && m_sync < m)) {
                const bool fl = exact && m_sync < m;
                const size_t qf = fl ? lb + mls[m_sync] : lb;
                __threadfence_block();   // this lane's own L.cut stores are complete
                if (fl && j == 0) {   // ratios stored by this lane at the line's finalisation
                    xs[g][14] = L.cut[2 * qf];
                    xs[g][15] = L.cut[2 * qf + 1];
                }
                wave_lds_sync();
                if (fl && j < 2) {
                    LineCutData d;
                    load_line(L, qf, d);
                    double P0[3], P1[3], C0[9], C1[9], o7[7];
#pragma unroll
                    for (int k = 0; k < 3; ++k) { P0[k] = j ? d.eP[k] : d.sP[k]; P1[k] = j ? d.sP[k] : d.eP[k]; }
#pragma unroll
                    for (int k = 0; k < 9; ++k) { C0[k] = j ? d.covE[k] : d.covS[k]; C1[k] = j ? d.covS[k] : d.covE[k]; }
                    cut_endpoint(cam, homog, Dl, d.Jl, P0, P1, C0, C1, xs[g][14 + j], o7);
#pragma unroll
                    for (int i = 0; i < 7; ++i) xs[g][7 * j + i] = o7[i];
                }
                wave_lds_sync();
                if (fl) {
                    double info[21];
                    cut_assemble<false>(&xs[g][0], &xs[g][7], info);
#pragma unroll
                    for (int e = 0; e < 21; ++e) {
                        const double S = sumE[g][e] - scr_l[(size_t)m_sync * 21 + e];
                        sumE[g][e] = S + info[e];
                    }
                    ++m_sync;
                }
                wave_lds_sync();
            }
            // 2. exact endpoints of this step's six slots, exact S of line m
            if (exact) {
                LineCutData d;
                load_line(L, q_cur, d);
                if (j < 6) {
                    const double t = (eside == 0 ? r0 : r1) + eoff;
                    double P0[3], P1[3], C0[9], C1[9], o7[7];
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        P0[k] = eside ? d.eP[k] : d.sP[k];
                        P1[k] = eside ? d.sP[k] : d.eP[k];
                    }
#pragma unroll
                    for (int k = 0; k < 9; ++k) {
                        C0[k] = eside ? d.covE[k] : d.covS[k];
                        C1[k] = eside ? d.covS[k] : d.covE[k];
                    }
                    cut_endpoint(cam, homog, Dl, d.Jl, P0, P1, C0, C1, t, o7);
#pragma unroll
                    for (int i = 0; i < 7; ++i) my_slot[i] = o7[i];
                }
#pragma unroll
                for (int e = 0; e < 21; ++e) xs[g][e] = sumE[g][e] - scr_l[(size_t)m * 21 + e];
            }
            wave_lds_sync();
            // 3. the reference's metrics and decision
            if (exact) {
                double mc;
                const double vj = cut_exact_step(&epf[g][CUT_SL * cs], &epf[g][CUT_SL * ce], &epf[g][CUT_SL * 1],
                                                 &epf[g][CUT_SL * 4], xs[g], sumE[g], first, &mc);
                best = group_first_max(vj, valid, j, mc, top);
            }
        }
        CUT_PROF(2);
        int finalize = 0;
        if (act) {
            first = 0;
            if (best >= 0) {
                r0 = r0 + nb_step(best, 0, st);
                r1 = r1 + nb_step(best, 1, st);
                if (!(r0 + r1 <= 1.0)) finalize = 1;   // while-condition
            } else {
                finalize = 1;   // the middle endpoints of this step are (r0 + 0, r1 + 0) = (r0, r1)
            }
        }
        if (act && finalize) {
            // approximate invCov_sum += info of the chosen ratio (the exact one is
            // accumulated lazily, only when an exact step needs it)
            // (the slots hold the polynomial-form terms, not v and J)
            double S7[7], E7[7];
            cut_endpoint_fast(cam, homog, &fst[g][0], &fst[g][3], &fst[g][6], &fst[g][12], fst[g][18], fst[g][19],
                              r0, S7);
            cut_endpoint_fast(cam, homog, &fst[g][3], &fst[g][0], &fst[g][12], &fst[g][6], fst[g][18], fst[g][19],
                              r1, E7);
            double info[21];
            CUT_PROF(4);
            cut_assemble<false>(S7, E7, info);
            double s21[21];
#pragma unroll
            for (int e = 0; e < 21; ++e) s21[e] = sumA[g][e] + info[e];
            CUT_PROF(5);
            if (j == 0) {
                L.cut[2 * q_cur] = r0;
                L.cut[2 * q_cur + 1] = r1;
            }
            ++m;
            if (m < nls) {
                q_cur = q_nx;
                q_nx = lb + (size_t)(int)nxt[g][CUT_FAST - 1];
                first = 1;
                r0 = 0.0;
                r1 = 0.0;
                // line m from the prefetch buffer
                double nx[42];
#pragma unroll
                for (int e = 0; e < 42; ++e) nx[e] = nxt[g][e];
#pragma unroll
                for (int e = 0; e < 21; ++e) s21[e] = s21[e] - nx[CUT_FAST + e];
#pragma unroll
                for (int e = 0; e < CUT_FAST; ++e) fst[g][e] = nx[e];
#pragma unroll
                for (int e = 0; e < 21; ++e) sumA[g][e] = s21[e];
                CUT_PROF(6);
                open_line(s21, nx);
                CUT_PROF(7);
                if (m + 1 < nls) pf_issue(m + 1);
            }
        }
#ifdef GFPL_CUT_PROF
        if (__any(act && finalize)) ++cp_fin;
#endif
        CUT_PROF(8);
        wave_lds_sync();
        CUT_PROF(3);
#ifdef GFPL_CUT_PROF
        ++cp_it;
#endif
    }
#ifdef GFPL_CUT_PROF
    if (lane == 0 && (blockIdx.x % 256) == 0)
        printf("cutprof blk %d it %llu fin %llu A %llu B %llu X %llu pre %llu asm %llu nxt %llu chol %llu post %llu sync %llu\n",
               blockIdx.x, cp_it, cp_fin, cp_acc[0], cp_acc[1], cp_acc[2], cp_acc[4], cp_acc[5], cp_acc[6], cp_acc[7],
               cp_acc[8], cp_acc[3]);
#endif
}

// ---------------------------------------------------------------- finish --
// invCovPose of the chosen ratio + updateEndPointByRatio (ledger Q4)
#ifndef GFPL_FIN_WAVES
#define GFPL_FIN_WAVES 1
#endif
__global__ void __launch_bounds__(64, GFPL_FIN_WAVES) k_cut_finish(KParams p) {
    const int b = blockIdx.x;
    const int nls = p.tr.n_matched_ls[b];
    if (nls == 0) return;
    const DevCam& cam = p.cam;
    DevLines& L = p.prev.ls;
    const size_t lb = (size_t)b * p.kl_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    double Dl[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) Dl[i] = p.scr.cut_dtinv[16 * b + i];
    for (int m = threadIdx.x; m < nls; m += blockDim.x) {
        const size_t q = lb + mls[m];
        LineCutData d;
        load_line(L, q, d);
        const double r0 = L.cut[2 * q], r1 = L.cut[2 * q + 1];
        double info[36];
        poseInfoOnLine<true>(cam, p.cfg.homog_th, Dl, d, r0, r1, info);
        // 16-B stores: a line's 36 doubles are contiguous and 288-B aligned (carve: 256-B field base)
        double2* iv = reinterpret_cast<double2*>(L.invcov + 36 * q);
#pragma unroll
        for (int i = 0; i < 18; ++i) iv[i] = make_double2(info[2 * i], info[2 * i + 1]);
        if (!(fabs(r0) < 0.0001 && fabs(r1) < 0.0001)) {
            double sP[3] = {d.sP[0], d.sP[1], d.sP[2]}, eP[3] = {d.eP[0], d.eP[1], d.eP[2]};
            if (fabs(r0) > 0.0001) {
                double s[3];
                for (int k = 0; k < 3; ++k) s[k] = (1 - r0) * sP[k] + r0 * eP[k];
                for (int k = 0; k < 3; ++k) { sP[k] = s[k]; L.sP[3 * q + k] = s[k]; }
                double uv[2];
                projection(cam, sP, uv);
                L.spl[2 * q] = uv[0]; L.spl[2 * q + 1] = uv[1];
                L.sdisp[q] = (cam.fx * cam.b) / sP[2];
            }
            if (fabs(r1) > 0.0001) {
                double e[3];
                for (int k = 0; k < 3; ++k) e[k] = (1 - r1) * eP[k] + r1 * sP[k];
                for (int k = 0; k < 3; ++k) { eP[k] = e[k]; L.eP[3 * q + k] = e[k]; }
                double uv[2];
                projection(cam, eP, uv);
                L.epl[2 * q] = uv[0]; L.epl[2 * q + 1] = uv[1];
                L.edisp[q] = (cam.fx * cam.b) / eP[2];
            }
        }
    }
}

hipError_t launch_line_cut(const KParams& p, hipStream_t s, const hipEvent_t* marks) {
    hipLaunchKernelGGL(k_cut_prep, dim3(p.B), dim3(64), 0, s, p);
    if (marks) (void)hipEventRecord(marks[0], s);
    hipLaunchKernelGGL(k_cut_search, dim3((p.B + CUT_G - 1) / CUT_G), dim3(64), 0, s, p);
    if (marks) (void)hipEventRecord(marks[1], s);
    hipLaunchKernelGGL(k_cut_finish, dim3(p.B), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace gfpl
