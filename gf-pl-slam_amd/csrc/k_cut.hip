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
#include <cstdlib>

#include "gfpl_kernels.hpp"

namespace gfpl {

struct LineCutData {
    double sP[3], eP[3], covS[9], covE[9], Jl[2];
};

// projected residual variance of one cut endpoint (src/stereoFrameHandler.cpp:1356-1369).
// Templated: T = double is the kernel's arithmetic, T = RB its running error bounds (the
// point's depth then takes the lower bound zlo, see rb_floor).
// SD (T = double only): the three divisions by pz^2 share the denominator's reciprocal refinement
// (SharedDiv, gfpl_device.hpp: every quotient keeps the bits of '/'), for k_cut_vref's evaluations
template <typename T, bool SD = false>
__device__ __forceinline__ T endpointVar_t(const DevCam& cam, const double* DT_inv, const T* Jl, const T* Pt,
                                           const T* cov, double zlo) {
    T Jdt[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) Jdt[i * 3 + j] = T(DT_inv[i * 4 + j]);
    T cur[3];
    se3_apply_t<T, double>(DT_inv, Pt, cur);
    rb_floor(cur[2], zlo);
    // getJacob3D_2D (src/stereoFrame.cpp:1394-1412)
    const T f = T(cam.fx), pz = cur[2], pz_2 = pz * pz;
    T Jp[9];
    Jp[0] = f / pz; Jp[3] = T(0.0); Jp[6] = T(0.0);
    Jp[1] = T(0.0); Jp[4] = f / pz; Jp[7] = T(0.0);
    if constexpr (SD) {
        const double n0 = (-f) * cur[0], n1 = (-f) * cur[1], n2 = (-f) * T(cam.b);
        const SharedDiv dz = div_prep(pz_2, n0);
        Jp[2] = div_by(dz, n0);
        Jp[5] = div_by(dz, n1);
        Jp[8] = div_by(dz, n2);
    } else {
        Jp[2] = ((-f) * cur[0]) / pz_2;
        Jp[5] = ((-f) * cur[1]) / pz_2;
        Jp[8] = ((-f) * T(cam.b)) / pz_2;
    }
    T T1[6], T2[6], T3[6], M[4];
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
    const T r0 = Jl[0] * M[0] + Jl[1] * M[2];
    const T r1 = Jl[0] * M[1] + Jl[1] * M[3];
    return r0 * Jl[0] + r1 * Jl[1];
}

// One cut endpoint of getPoseInfoOnLine (src/stereoFrameHandler.cpp:1350-1388):
// P = (1-c)*P0 + c*P1 with its covariance blend (1-c)^2*C0 + c^2*C1, the
// projected residual variance v and the pose Jacobian J of that endpoint.
// Start endpoint: (sP, eP, covS, covE, c0); end endpoint: (eP, sP, covE, covS, c1).
// The start terms depend on c0 only and the end terms on c1 only, which the
// search exploits.
template <typename T, bool VAR = true>
__device__ __forceinline__ void cut_endpoint_t(const DevCam& cam, double homog, const double* DT_inv, const T* Jl,
                                               const T* P0, const T* P1, const T* C0, const T* C1, T c, T* out7,
                                               double zlo) {
    T Pt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) Pt[k] = (T(1.0) - c) * P0[k] + c * P1[k];
    if (VAR) {   // (VAR = false: C0 / C1 are not read)
        const T a = (T(1.0) - c) * (T(1.0) - c), q = c * c;
        T cov[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) cov[i] = a * C0[i] + q * C1[i];
        out7[0] = endpointVar_t<T>(cam, DT_inv, Jl, Pt, cov, zlo);
    }
    T cur[3];
    se3_apply_t<T, double>(DT_inv, Pt, cur);
    rb_floor(cur[2], zlo);
    poseJac_t<T>(cam, homog, cur, Jl[0], Jl[1], out7 + 1);
}
__device__ __forceinline__ void cut_endpoint(const DevCam& cam, double homog, const double* DT_inv, const double* Jl,
                                             const double* P0, const double* P1, const double* C0, const double* C1,
                                             double c, double* out7) {
    cut_endpoint_t<double>(cam, homog, DT_inv, Jl, P0, P1, C0, C1, c, out7, 0.0);
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

// ------------------------------------------------- comparison polynomials --
// The greedy search compares logdet(S + info(t0, t1)) over neighbours.
// Along a side the transformed cut point is g(t) = (1-t) g0 + t g1 (DT is affine), and
// getPoseInfoOnLine's Jacobian and projected variance of that endpoint are
//   J(t) = fgz2(t) P(t),  v(t) = fgz2(t)^2 v'(t),  fgz2 = fx / gz^2,
// with P quadratic in t (its first three entries p(t) linear) and
//   v'(t) = p(t)^T ((1-t)^2 A0 + t^2 A1) p(t),  A = R cov R^T,
// a quartic — for lines whose segment keeps gz^2 above homog_th (PD_OK; other lines
// are searched with the reference's exact steps).  The fgz2 factors cancel in the
// determinant lemma, so a neighbour's comparison value needs only P and v'.
// Per matched line, k_cut_prep stores (CUT_FAST doubles):
#define PD_PS 0      // start side (sP -> eP, t = r0): P coefficients of t^0, t^1, t^2 [3 x 6]
#define PD_PE 18     // end side (eP -> sP, t = r1) [3 x 6]
#define PD_VS 36     // v'_s(t) coefficients of t^0 .. t^4 [5]
#define PD_VE 41     // v'_e(t) [5]
#define PD_OK 46     // 1.0: gz^2 > 2 homog_th at both ends, one sign (fgz2 = fx / gz^2 on the segment)
#define PD_NEXT 47   // list index of the line after this one (k_cut_search's prefetch)
#define PD_ERR 48    // k_cut_bounds: 14 floats (rounded up) packed in 7 doubles, per side (start, end):
                     // eP[6] (|P(t) - P*(t)|, ours + the reference's endpoint Jacobian in P units) | ev
                     // (|v'(t) - v'*(t)|), valid for every t of the range; +inf: no margined steps
static_assert(CUT_FAST == 56, "per-line comparison data layout");

// x^T A y, A symmetric packed (xx xy xz yy yz zz)
template <typename T>
__device__ __forceinline__ T sym3_t(const T* A, const T* x, const T* y) {
    const T ax = (A[0] * y[0] + A[1] * y[1]) + A[2] * y[2];
    const T ay = (A[1] * y[0] + A[3] * y[1]) + A[4] * y[2];
    const T az = (A[2] * y[0] + A[4] * y[1]) + A[5] * y[2];
    return (x[0] * ax + x[1] * ay) + x[2] * az;
}

// coefficient k of P(t) for the blend g0 -> g1 (poseJac's six terms without fgz2)
template <typename T>
__device__ __forceinline__ void cut_poly_coeff_t(const T* g0, const T* g1, T lx, T ly, int k, T* Pk) {
    const T dx = g1[0] - g0[0], dy = g1[1] - g0[1], dz = g1[2] - g0[2];
    // coefficient k of the product (a0 + t a1)(b0 + t b1)
    auto prod = [&](T a0, T a1, T b0, T b1) -> T {
        return k == 0 ? a0 * b0 : (k == 1 ? a0 * b1 + a1 * b0 : a1 * b1);
    };
    auto lin = [&](T a0, T a1) -> T { return k == 0 ? a0 : (k == 1 ? a1 : T(0.0)); };
    const T x0 = g0[0], y0 = g0[1], z0 = g0[2];
    Pk[0] = lx * lin(z0, dz);
    Pk[1] = ly * lin(z0, dz);
    Pk[2] = -(lx * lin(x0, dx) + ly * lin(y0, dy));
    Pk[3] = -((lx * prod(x0, dx, y0, dy) + ly * prod(y0, dy, y0, dy)) + ly * prod(z0, dz, z0, dz));
    Pk[4] = (lx * prod(x0, dx, x0, dx) + lx * prod(z0, dz, z0, dz)) + ly * prod(x0, dx, y0, dy);
    Pk[5] = ly * prod(x0, dx, z0, dz) - lx * prod(y0, dy, z0, dz);
}

// The comparison polynomials' coefficients of one line: P [side][k][6] (side 0: sP -> eP),
// v' [side][5], and the transformed endpoints g [2][3]
template <typename T>
__device__ __forceinline__ void cut_poly_coef_t(const double* Dl, const T* sP, const T* eP, const T* covS,
                                                const T* covE, const T* Jl, T* P, T* V, T* g) {
    se3_apply_t<T, double>(Dl, sP, g);
    se3_apply_t<T, double>(Dl, eP, g + 3);
    T A[2][6];   // R covS R^T, R covE R^T
    const T* Cs[2] = {covS, covE};
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        T Tm[9];   // R C
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                Tm[i * 3 + k] = (T(Dl[i * 4 + 0]) * Cs[w][0 * 3 + k] + T(Dl[i * 4 + 1]) * Cs[w][1 * 3 + k]) +
                                T(Dl[i * 4 + 2]) * Cs[w][2 * 3 + k];
        const int ii[6] = {0, 0, 0, 1, 1, 2}, jj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
        for (int e = 0; e < 6; ++e)
            A[w][e] = (Tm[ii[e] * 3 + 0] * T(Dl[jj[e] * 4 + 0]) + Tm[ii[e] * 3 + 1] * T(Dl[jj[e] * 4 + 1])) +
                      Tm[ii[e] * 3 + 2] * T(Dl[jj[e] * 4 + 2]);
    }
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        T* Ps = P + 18 * side;
#pragma unroll
        for (int k = 0; k < 3; ++k) cut_poly_coeff_t<T>(g + 3 * side, g + 3 * (1 - side), Jl[0], Jl[1], k, Ps + 6 * k);
        // v'(t) = (1-t)^2 Qa(t) + t^2 Qb(t), Q(t) = q0 + 2 t q1 + t^2 q2 for p(t) = P[0..2] = p0 + t p1
        const T* p0 = Ps;
        const T* p1 = Ps + 6;
        const T a0 = sym3_t<T>(A[side], p0, p0), a1 = sym3_t<T>(A[side], p0, p1), a2 = sym3_t<T>(A[side], p1, p1);
        const T b0 = sym3_t<T>(A[1 - side], p0, p0), b1 = sym3_t<T>(A[1 - side], p0, p1), b2 = sym3_t<T>(A[1 - side], p1, p1);
        T* v = V + 5 * side;
        v[0] = a0;
        v[1] = T(2.0) * (a1 - a0);
        v[2] = ((a2 - T(4.0) * a1) + a0) + b0;
        v[3] = T(2.0) * ((a1 - a2) + b1);
        v[4] = a2 + b2;
    }
}

__device__ __forceinline__ void cut_poly_data(const double* Dl, const LineCutData& d, double homog, double* fd) {
    double P[36], V[10], g[6];
    cut_poly_coef_t<double>(Dl, d.sP, d.eP, d.covS, d.covE, d.Jl, P, V, g);
#pragma unroll
    for (int i = 0; i < 18; ++i) { fd[PD_PS + i] = P[i]; fd[PD_PE + i] = P[18 + i]; }
#pragma unroll
    for (int i = 0; i < 5; ++i) { fd[PD_VS + i] = V[i]; fd[PD_VE + i] = V[5 + i]; }
    const double z0 = g[2], z1 = g[5];
    fd[PD_OK] = (((z0 > 0.0 && z1 > 0.0) || (z0 < 0.0 && z1 < 0.0)) && z0 * z0 > 2.0 * homog && z1 * z1 > 2.0 * homog)
                    ? 1.0 : 0.0;
}

// a wave's LDS stores visible to its own later loads (one wave: no barrier needed)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------------ prep --
// W waves per sequence (W = 1 from CUT_PREP_W8_MAX_B up; small batches W = 8): the waves compute W
// 64-entry chunks at once, each in its own LDS buffer, then wave 0's lanes e < 21 add the W chunks'
// infos in list order (the serial sum is the part that stays one wave's)
template <int W>
__global__ void __launch_bounds__(64 * W) k_cut_prep(KParams p) {
    extern __shared__ double prep_lds[];   // W x [21][65] lower-triangle infos of 64 list entries (padded row)
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = W > 1 ? (int)(threadIdx.x >> 6) : 0;
    const int nls = p.tr.n_matched_ls[b];
    const int npt = p.tr.n_matched_pt[b];
    if (nls == 0) return;
    double (*chunk)[65] = reinterpret_cast<double (*)[65]>(prep_lds + (size_t)wv * 21 * 65);
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    DevLines& L = p.prev.ls;
    const DevPoints& P = p.prev.pt;
    const size_t lb = (size_t)b * p.kl_cap, pbase = (size_t)b * p.kp_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    const int32_t* mpt = p.tr.matched_pt + (size_t)b * p.mpt_cap;
    double* rec_l = p.scr.cut_rec + (size_t)b * p.mls_cap * CUT_REC;
    // DT_inv = curr.Tfw^-1 * prev.Tfw (src/stereoFrameHandler.cpp:1635), every lane
    double Dl[16];
    {
        double Tc[16], Tp[16], Ti[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) { Tc[i] = p.curr.pose.Tfw[16 * b + i]; Tp[i] = p.prev.pose.Tfw[16 * b + i]; }
        mat4_inv(Tc, Ti);
        mat4_mul(Ti, Tp, Dl);
    }
    if (wv == 0 && lane < 16) p.scr.cut_dtinv[16 * b + lane] = Dl[lane];
    // invCov_sum: lines then points, each entry summed in list order by lane e < 21 of wave 0,
    // 64 list entries per wave at a time staged through LDS (src/stereoFrameHandler.cpp:1640-1657)
    double s = 0.0;
    const int nl_ch = (nls + 63) >> 6, np_ch = (npt + 63) >> 6;
    auto chunk_cnt = [&](int c) {
        const bool lines = c < nl_ch;
        return min(64, (lines ? nls : npt) - (((lines ? c : c - nl_ch)) << 6));
    };
    for (int c0 = 0; c0 < nl_ch + np_ch; c0 += W) {
        const int c = c0 + wv;
        if (c < nl_ch + np_ch) {   // (wave-uniform)
            const bool lines = c < nl_ch;
            const int m = ((lines ? c : c - nl_ch) << 6) + lane;
            const int cnt = chunk_cnt(c);
            double info[21];
            double fd[CUT_FAST];   // (lines) the record's comparison data
            if (lane < cnt) {
                if (lines) {
                    LineCutData d;
                    load_line(L, lb + mls[m], d);
                    poseInfoOnLine<false>(cam, homog, Dl, d, 0.0, 0.0, info);
#pragma unroll
                    for (int i = PD_ERR; i < CUT_FAST; ++i) fd[i] = 0.0;   // k_cut_bounds fills PD_ERR
                    cut_poly_data(Dl, d, homog, fd);
                    fd[PD_NEXT] = (double)mls[min(m + 1, nls - 1)];   // k_cut_search's next-next line
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
            }
            if (lines) {   // (wave-uniform)
                // The chunk's records (comparison data | r = 0 info | pad) leave in five slices of 16
                // doubles staged through the wave's chunk buffer (idle until the sums): a store
                // instruction then writes 8 whole 128-B lines of 8 records instead of 16 B of each of 64
                // records — stored straight from the lanes, the records took a third of the kernel
                // (profiles/r04_s/bench_prepprobe.log)
                double* stg = &chunk[0][0];   // [64][17] (odd row stride: the lanes' rows spread over the banks)
                const int pl = lane >> 3, pp = lane & 7;
                double* rc = rec_l + (size_t)(c << 6) * CUT_REC;
#pragma unroll
                for (int sl = 0; sl < CUT_REC / 16; ++sl) {
                    if (lane < cnt) {
#pragma unroll
                        for (int k = 0; k < 16; ++k) {
                            const int x = 16 * sl + k;
                            stg[lane * 17 + k] = x < CUT_FAST ? fd[x] : (x < CUT_FAST + 21 ? info[x - CUT_FAST] : 0.0);
                        }
                    }
                    wave_lds_sync();
                    // (reading four slices ahead of their stores measured the same: profiles/r04_aa)
#pragma unroll
                    for (int g8 = 0; g8 < 8; ++g8) {
                        const int ln = 8 * g8 + pl;
                        if (ln < cnt)
                            reinterpret_cast<double2*>(rc + (size_t)ln * CUT_REC + 16 * sl)[pp] =
                                make_double2(stg[ln * 17 + 2 * pp], stg[ln * 17 + 2 * pp + 1]);
                    }
                    wave_lds_sync();
                }
            }
            if (lane < cnt) {
#pragma unroll
                for (int i = 0; i < 21; ++i) chunk[i][lane] = info[i];
            }
        }
        __syncthreads();
        if (wv == 0 && lane < 21) {
            const double (*all)[21][65] = reinterpret_cast<const double (*)[21][65]>(prep_lds);
            for (int k = 0; k < W && c0 + k < nl_ch + np_ch; ++k) {
                const int cnt = chunk_cnt(c0 + k);
                for (int e = 0; e < cnt; ++e) s = s + all[k][lane][e];
            }
        }
        __syncthreads();
    }
    if (wv == 0 && lane < 21) p.scr.cut_sum[24 * b + lane] = s;
}
constexpr size_t cut_prep_lds(int w) { return (size_t)w * 21 * 65 * sizeof(double); }

// ---------------------------------------------------------------- bounds --
// Per matched line, the error bounds of the margined comparisons' operands,
// by running error analysis (RB) of the very expression trees the kernels evaluate, for every
// ratio of the range c in [0, C], C = max(rng[1], 0) (rng inside [0, 1]; otherwise the line
// gets +inf and is searched with exact steps):
//  ours  — cut_poly_coef_t: |P_k(computed) - P_k*| per coefficient, summed over t^k;
//  ref   — cut_endpoint_t: the reference's endpoint Jacobian J as getPoseInfoOnLine computes
//          it, |J^ - J*|, moved to P units by the exact fgz2*(t) = fx / gz*(t)^2 >= fx / zmax^2
//          (J = fgz2 P).  No variance bound: the proven search takes the reference's own
//          variances (its v'-table, k_cut_search<true>), where a bound over the range would be
//          ~1e-9 relative — the reference's v = l^T Jp (R C R^T) Jp^T l cancels the depth
//          variance along the viewing ray (~1e7 x the result in the synthetic workload).
// The depth gz* of the blended point lies between the transformed endpoints' (c in [0, 1]),
// which bounds the divisors from below (zlo) and fgz2* from below (zmax).
__device__ __forceinline__ float ceil_f32(double x) {
    if (!(x >= 0.0)) return __builtin_inff();   // NaN / negative: no bound
    float f = (float)x;
    if ((double)f < x) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}
// Proven mode: v'_ref(c) = v / fgz2^2 with v the reference's endpoint variance at ratio c (the
// expression tree of cut_endpoint_t<double>, hence its bits) and fgz2 = fx / max(homog, gz^2) of
// the blended point (poseJac's); P(t) of the comparison polynomials is J / fgz2, so the pair
// (P, v'_ref) carries the reference's info J J^T / v up to the scaling's rounding
__device__ __forceinline__ double ref_vprime(const DevCam& cam, double homog, const double* Dl, const DevLines& L,
                                             size_t q, int side, double c) {
    const double* P0 = side ? L.eP + 3 * q : L.sP + 3 * q;
    const double* P1 = side ? L.sP + 3 * q : L.eP + 3 * q;
    const double* C0 = side ? L.covE + 9 * q : L.covS + 9 * q;
    const double* C1 = side ? L.covS + 9 * q : L.covE + 9 * q;
    const double Jl[2] = {L.le_obs[3 * q], L.le_obs[3 * q + 1]};
    double Pt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) Pt[k] = (1.0 - c) * P0[k] + c * P1[k];
    const double a = (1.0 - c) * (1.0 - c), qq = c * c;
    double cov[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) cov[i] = a * C0[i] + qq * C1[i];
    const double v = endpointVar_t<double>(cam, Dl, Jl, Pt, cov, 0.0);
    double cur[3];
    se3_apply(Dl, Pt, cur);
    const double f = cam.fx / ref_max(homog, cur[2] * cur[2]);
    return v / (f * f);
}

// Proven line cut: per matched line, side and ratio key, the reference's endpoint variance scaled
// by its fgz2 (ref_vprime), into cut_vtab — one thread per (line, side, key), consecutive threads
// on one line (its inputs are one broadcast load)
__global__ void __launch_bounds__(256) k_cut_vtab(KParams p) {
    const int b = blockIdx.x;
    const int nls = p.tr.n_matched_ls[b];
    const int nk = p.cut_nkeys;
    if (nls == 0 || nk == 0 || (p.cfg.cut_proof != 2 && p.scr.cut_flag[b] == 0)) return;
    const DevLines& L = p.prev.ls;
    const double* Dl = p.scr.cut_dtinv + 16 * (size_t)b;
    const int per = 2 * nk;
    for (int idx = threadIdx.x; idx < nls * per; idx += 256) {
        const int m = idx / per, r = idx - m * per;
        const int side = r >= nk ? 1 : 0, slot = r - side * nk;
        const size_t q = (size_t)b * p.kl_cap + p.tr.matched_ls[(size_t)b * p.mls_cap + m];
        p.scr.cut_vtab[((size_t)b * p.mls_cap + m) * (2 * CUT_KS) + side * CUT_KS + slot] =
            ref_vprime(p.cam, p.cfg.homog_th, Dl, L, q, side, p.cut_keys[slot]);
    }
}

// the line's operand error bounds (above) for line q of sequence b: eb[0..5] / [7..12] the start /
// end side's |P - P*| in P units, eb[6] / [13] the blended depth's relative error bound; +inf: no
// usable bound (the line's steps are then exact)
__device__ __forceinline__ void cut_line_bounds(const KParams& p, size_t q, bool pd_ok, const double* Dl, float* eb) {
    const DevLines& L = p.prev.ls;
    const double rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    const double C = fmax(rhi, 0.0), T = fmax(fabs(rlo), fabs(rhi));
#pragma unroll
    for (int i = 0; i < 14; ++i) eb[i] = __builtin_inff();
    bool ok = rlo >= 0.0 && rhi <= 1.0 && pd_ok && p.cam.fx > 0.0;
    RB sP[3], eP[3], cS[9], cE[9], Jl[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) { sP[k] = RB(L.sP[3 * q + k]); eP[k] = RB(L.eP[3 * q + k]); }
#pragma unroll
    for (int k = 0; k < 9; ++k) { cS[k] = RB(L.covS[9 * q + k]); cE[k] = RB(L.covE[9 * q + k]); }
    Jl[0] = RB(L.le_obs[3 * q]);
    Jl[1] = RB(L.le_obs[3 * q + 1]);
    double eo[2][7];   // ours: eP[6], ev per side
    double zlo = 0.0, zmax = 0.0;
    if (ok) {
        RB P[36], V[10], g[6];
        cut_poly_coef_t<RB>(Dl, sP, eP, cS, cE, Jl, P, V, g);
        double gd[6];
        {
            const double s3[3] = {L.sP[3 * q], L.sP[3 * q + 1], L.sP[3 * q + 2]};
            const double e3[3] = {L.eP[3 * q], L.eP[3 * q + 1], L.eP[3 * q + 2]};
            se3_apply(Dl, s3, gd);
            se3_apply(Dl, e3, gd + 3);
        }
        zlo = fmin(fabs(gd[2]) - g[2].e, fabs(gd[5]) - g[5].e);
        zmax = fmax(fabs(gd[2]) + g[2].e, fabs(gd[5]) + g[5].e);
        ok = zlo > 0.0;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
#pragma unroll
            for (int i = 0; i < 6; ++i)
                eo[side][i] = (P[18 * side + i].e + T * (P[18 * side + 6 + i].e + T * P[18 * side + 12 + i].e));
            const RB* v = V + 5 * side;
            eo[side][6] = v[0].e + T * (v[1].e + T * (v[2].e + T * (v[3].e + T * v[4].e)));
        }
    }
    if (ok) {
        const double cam_fx = p.cam.fx;
        const double s1 = zmax * zmax / cam_fx;   // 1 / fgz2*_min
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            RB o7[7];
            cut_endpoint_t<RB, false>(p.cam, p.cfg.homog_th, Dl, Jl, side ? eP : sP, side ? sP : eP, side ? cE : cS,
                                      side ? cS : cE, RB(C, 0.0, 0.0), o7, zlo);
            // 1% slop: the bound arithmetic's own rounding
#pragma unroll
            for (int i = 0; i < 6; ++i) eb[7 * side + i] = ceil_f32(1.01 * (eo[side][i] + o7[1 + i].e * s1));
            // v': the proven search evaluates with the reference's own endpoint variances scaled by
            // fgz2 = fx / gz^2 of the blended point (its v'-table): slot 6 is gz's relative error
            // bound over the range (the blend and DT_inv's rounding), which the scaling carries x 4
            {
                const RB c(C, 0.0, 0.0);
                const RB* Q0 = side ? eP : sP;
                const RB* Q1 = side ? sP : eP;
                RB Pt[3], cur[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) Pt[k] = (RB(1.0) - c) * Q0[k] + c * Q1[k];
                se3_apply_t<RB, double>(Dl, Pt, cur);
                rb_floor(cur[2], zlo);
                eb[7 * side + 6] = cur[2].lo > 0.0 ? ceil_f32(1.01 * cur[2].e / cur[2].lo) : __builtin_inff();
            }
        }
    }
}

// k_cut_verify's variant: the same P bounds (our coefficients' RB error + the reference's Jacobian's)
// and the blended depth's relative error, without the v' coefficients' bound (the verification
// measures v' against the reference's own values instead) — so without R C R^T in RB
__device__ __forceinline__ void cut_line_bounds_p(const KParams& p, size_t q, bool pd_ok, const double* Dl, float* eb) {
    const DevLines& L = p.prev.ls;
    const double rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    const double C = fmax(rhi, 0.0), T = fmax(fabs(rlo), fabs(rhi));
#pragma unroll
    for (int i = 0; i < 14; ++i) eb[i] = __builtin_inff();
    if (!(rlo >= 0.0 && rhi <= 1.0 && pd_ok && p.cam.fx > 0.0)) return;
    RB sP[3], eP[3], Jl[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) { sP[k] = RB(L.sP[3 * q + k]); eP[k] = RB(L.eP[3 * q + k]); }
    Jl[0] = RB(L.le_obs[3 * q]);
    Jl[1] = RB(L.le_obs[3 * q + 1]);
    RB g[6];
    se3_apply_t<RB, double>(Dl, sP, g);
    se3_apply_t<RB, double>(Dl, eP, g + 3);
    double gd[6];
    {
        const double s3[3] = {L.sP[3 * q], L.sP[3 * q + 1], L.sP[3 * q + 2]};
        const double e3[3] = {L.eP[3 * q], L.eP[3 * q + 1], L.eP[3 * q + 2]};
        se3_apply(Dl, s3, gd);
        se3_apply(Dl, e3, gd + 3);
    }
    const double zlo = fmin(fabs(gd[2]) - g[2].e, fabs(gd[5]) - g[5].e);
    const double zmax = fmax(fabs(gd[2]) + g[2].e, fabs(gd[5]) + g[5].e);
    if (!(zlo > 0.0)) return;
    const double s1 = zmax * zmax / p.cam.fx;   // 1 / fgz2*_min
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        double eo[6] = {0, 0, 0, 0, 0, 0};
        double tk = 1.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {   // (cut_poly_coef_t's P part: coefficient k of the side's P(t))
            RB Pk[6];
            cut_poly_coeff_t<RB>(g + 3 * side, g + 3 * (1 - side), Jl[0], Jl[1], k, Pk);
#pragma unroll
            for (int i = 0; i < 6; ++i) eo[i] = eo[i] + tk * Pk[i].e;
            tk = tk * T;
        }
        RB o7[7];
        cut_endpoint_t<RB, false>(p.cam, p.cfg.homog_th, Dl, Jl, side ? eP : sP, side ? sP : eP, nullptr, nullptr,
                                  RB(C, 0.0, 0.0), o7, zlo);
#pragma unroll
        for (int i = 0; i < 6; ++i) eb[7 * side + i] = ceil_f32(1.01 * (eo[i] + o7[1 + i].e * s1));
        const RB c(C, 0.0, 0.0);
        const RB* Q0 = side ? eP : sP;
        const RB* Q1 = side ? sP : eP;
        RB Pt[3], cur[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) Pt[k] = (RB(1.0) - c) * Q0[k] + c * Q1[k];
        se3_apply_t<RB, double>(Dl, Pt, cur);
        rb_floor(cur[2], zlo);
        eb[7 * side + 6] = cur[2].lo > 0.0 ? ceil_f32(1.01 * cur[2].e / cur[2].lo) : __builtin_inff();
    }
}

// eager-proven mode (cut_proof 2, or the sequences cut_proof 1 could not verify): the bounds into
// the records, one thread per line
__global__ void __launch_bounds__(64) k_cut_bounds(KParams p) {
    const int b = blockIdx.y;
    const int m = blockIdx.x * 64 + threadIdx.x;
    const int nls = p.tr.n_matched_ls[b];
    if (m >= nls || (p.cfg.cut_proof != 2 && p.scr.cut_flag[b] == 0)) return;
    const size_t q = (size_t)b * p.kl_cap + p.tr.matched_ls[(size_t)b * p.mls_cap + m];
    double* rec = p.scr.cut_rec + ((size_t)b * p.mls_cap + m) * CUT_REC;
    double Dl[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) Dl[i] = p.scr.cut_dtinv[16 * b + i];
    float eb[14];
    cut_line_bounds(p, q, rec[PD_OK] != 0.0, Dl, eb);
    float* out = reinterpret_cast<float*>(rec + PD_ERR);
#pragma unroll
    for (int i = 0; i < 14; ++i) out[i] = eb[i];
}

// ---------------------------------------------------------------- search --
// 8 sequences per wave, 8 lanes each; every wave iteration is one greedy step
// of each of its 8 chains.
//
// Margined comparisons.  Within line m the search compares
// logdet(S + info(t0, t1)) over neighbours, S = invCov_sum - info_m(0, 0) fixed
// for the line, and info = Js Js^T / vs + Je Je^T / ve (rank 2, ledger Q10).  By
// the matrix determinant lemma logdet(S + info) = logdet(S) + log d with
//   d = (1 + as)(1 + ae) - c^2 / (vs ve),  as = |L^-1 Js|^2 / vs, ae = |L^-1 Je|^2 / ve,
//   c = (L^-1 Js) . (L^-1 Je),  S = L L^T,
// and with J = fgz2 P, v = fgz2^2 v' (see PD_*) the fgz2 factors cancel:
//   d = D / (v's v'e),  D = (v's + Ns)(v'e + Ne) - C^2,
//   Ns(t0) = |W(t0)|^2, Ne(t1) = |W(t1)|^2, C(t0, t1) = Ws(t0) . We(t1),  W = L^-1 P.
// W is quadratic in t, so with the Gram matrix G of the six coefficient vectors
// L^-1 P_{side,k} (solved once when the line opens) Ns and Ne are quartics in t and
// C is bi-quadratic in (t0, t1).  Lane j evaluates neighbour j's d from these
// polynomial coefficients in registers: no LDS, no triangular solve, one reciprocal.
//
// The reference's decision (first strict maximum over the valid neighbours,
// starting from the centre's metric) is taken from the d values when
//   (1) every comparison it rests on is separated by more than cfg.cut_certify
//       (relative, default 1e-9), and
//   (2) every d involved carries a computed forward rounding-error bound of at
//       most cut_certify / 4 (cut_dval: Horner and product error bounds from the
//       absolute values of the terms, so cancellation in Ns, C, D or v' shows up),
//       so in exact arithmetic the lemma's gaps exceed cut_certify / 2,
// and the line's S factored with every pivot above 1e-2 of its diagonal
// (chol_s).  The remaining disagreement — between the lemma in exact arithmetic and
// the reference's own rounded LLT + log evaluation — is bounded by measurement,
// not by proof.  Otherwise (and whenever S, an endpoint variance or
// d is not healthy) the group evaluates that step exactly as the reference does:
// neighbour j's info assembled from its endpoints, + S, LLT, six fdlibm logs, against
// the exact centre metric.  The metric values themselves are never output.
//
// Per iteration: lane j evaluates d of neighbour j, the group's first-strict-max by a
// 3-step DPP reduction, the margin tests by ballot; the exact step (X) when any group
// of the wave needs it; a move, or the line's finalisation: the approximate
// invCov_sum += info of the chosen ratio (from P and v', every lane), the next line's
// data from the prefetch registers through LDS, its S factored and the Gram matrix
// of its W coefficients formed across the group's lanes.
#define CUT_G 8          // sequences per wave (8 lanes each)
// A line transition waits until CUT_BATCH groups of the wave have finished their line
// or one of them has waited CUT_WAIT iterations (measured at B = 16384: 8 / 16, i.e.
// nearly lock-step lines, 6.7 ms; 3 / 3 8.5 ms; no batching 10.9 ms)
#ifndef CUT_BATCH
#define CUT_BATCH 8
#endif
#ifndef CUT_WAIT
#define CUT_WAIT 16
#endif
#define CUT_SL 7         // exact endpoint slot (X): v, J[6]
#define CUT_EP 43        // per-group exact endpoint block: 6 slots + 1 (odd stride)
#define CUT_NX (CUT_FAST + 21)   // used part of a line record: comparison data | r = 0 info
static_assert(CUT_REC * 8 == 640 && CUT_NX + 3 <= CUT_REC, "a record is 5 x 128 B: five 16-B loads per lane");
// record slots CUT_NX .. CUT_NX + 2: the line's agreement bound as k_cut_search formed it (6 floats,
// CutCmp::eb; diagnostics, gfpl_debug_cut_records)

// One reference-order cut endpoint (cut_endpoint) of line q: side 0 the start
// endpoint blended sP -> eP, side 1 the end endpoint eP -> sP, at ratio t.
__device__ __forceinline__ void exact_endpoint(const DevCam& cam, double homog, const double* Dl, const DevLines& L,
                                               size_t q, int side, double t, double* o7) {
    const double* sP = L.sP + 3 * q;
    const double* eP = L.eP + 3 * q;
    const double* cS = L.covS + 9 * q;
    const double* cE = L.covE + 9 * q;
    const double Jl[2] = {L.le_obs[3 * q], L.le_obs[3 * q + 1]};
    cut_endpoint(cam, homog, Dl, Jl, side ? eP : sP, side ? sP : eP, side ? cE : cS, side ? cS : cE, t, o7);
}

// neighbour j's offset on a side (src/stereoFrameHandler.cpp:1624-1633): bit masks of the moves that
// grow (0x31 / 0x54) and shrink (0xC2 / 0xA8) the start / end ratio, so a data-dependent j costs no branch
__device__ __forceinline__ int nb_off(int j, int side) {
    const unsigned pl = side == 0 ? 0x31u : 0x54u, mi = side == 0 ? 0xC2u : 0xA8u;
    return (int)((pl >> j) & 1u) - (int)((mi >> j) & 1u);
}
__device__ __forceinline__ double nb_step(int j, int side, double st) {
    return (double)nb_off(j, side) * st;   // (st, -st or +0.0: the bits of the ternary it replaces)
}
__device__ __forceinline__ int nb_slot(int j, int side) {   // endpoint slot: 0: -s, 1: 0, 2: +s
    return 1 + nb_off(j, side);
}

// S = L L^T for the margined comparisons (out: L strictly lower 21, 1/L_kk 6, ok).  ok = 0
// unless every pivot keeps at least CUT_MIN_PIVOT of its diagonal; the line is then
// searched with exact steps only.  The pivot ratios bound the condition of the
// diagonally scaled S, which sets both the lemma's and the reference LLT's rounding
// error (the synthetic, KITTI and EuRoC workloads stay above 0.1).
constexpr double CUT_MIN_PIVOT = 1e-2;
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
        if (!(x > CUT_MIN_PIVOT * akk && akk < 1e300)) { ok = false; x = 1.0; }
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

// Reciprocal for the margined comparisons only (never for an output or an exact
// step): hardware v_rcp_f64 refined by two Newton steps, within an ulp or two of 1/x;
// 0, infinities and NaN come out NaN or infinite and fail the health tests.
__device__ __forceinline__ double rcp_fast(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
    return r;
}

__device__ __forceinline__ double h4(const double* c, double t) {
    return __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, c[4], c[3]), c[2]), c[1]), c[0]);
}
// Horner with |coefficients| (the abs is a free source modifier of v_fma_f64)
__device__ __forceinline__ double h4abs(const double* c, double t) {
    return __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, fabs(c[4]), fabs(c[3])), fabs(c[2])),
                                          fabs(c[1])), fabs(c[0]));
}
__device__ __forceinline__ double h2(double c0, double c1, double c2, double t) {
    return __builtin_fma(t, __builtin_fma(t, c2, c1), c0);
}

// The measured search's own (approximate) info of a finished line at its final ratios, which it adds
// to its running invCov_sum: xs = [v'_s, P_s[6], v'_e, P_e[6]] from the line's comparison data (or the
// reference-order endpoints when PD_OK = 0), entry (ra, cb) = Ps Ps^T / v'_s + Pe Pe^T / v'_e.  Shared
// by k_cut_search and k_cut_verify, which replays the search's running sum bit for bit.
__device__ __forceinline__ double cut_ours_P(const double* fd, int side, int i, double t) {
    const int o = side ? PD_PE : PD_PS;
    return h2(fd[o + i], fd[o + 6 + i], fd[o + 12 + i], t);
}
__device__ __forceinline__ double cut_ours_V(const double* fd, int side, double t) {
    const int o = side ? PD_VE : PD_VS;
    return __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, fd[o + 4], fd[o + 3]), fd[o + 2]),
                                          fd[o + 1]), fd[o]);
}
__device__ __forceinline__ double cut_ours_info(const double* xs, double is, double ie, int ra, int cb) {
    return __builtin_fma(xs[1 + ra] * is, xs[1 + cb], (xs[8 + ra] * ie) * xs[8 + cb]);
}

// Comparison polynomials of the current line, one copy per lane (registers).  The fields a step
// reads (ns .. bnd, doubles 0-31) come first and the struct is 16-B aligned, 336 B (84 dwords)
// long: the per-step load is 16 ds_read_b128 (4 LDS cycles each, 256 B/clk) instead of
// ds_read2_b64 pairs (8 cycles each, 128 B/clk), and the 8 groups' rows start in 8 disjoint bank
// quads (84 g mod 64) of a b128 lane group.  Raw offsets (cl[]): ns 0, ne 5, vs 10, ve 15, cc 20,
// bnd 29, bs 32, be 35.
struct __attribute__((aligned(16))) CutCmp {
    double ns[5], ne[5];     // |W_s(t)|^2, |W_e(t)|^2
    double vs[5], ve[5];     // v'_s, v'_e
    double cc[9];            // C(t0, t1): cc[3 i + k] multiplies t0^i t1^k
    double bnd[3];           // the line's bound terms at |t| = T = max(|rlo|, |rhi|): P1, VsA, VeA
    double bs[3], be[3];     // |W_{side,k}| (error bounds: |Ns| terms <= (sum_k bs_k t^k)^2); line open only
    // the line's agreement bound: a step's neighbour value differs from the
    // reference's metric by at most E = 1/v's (A1 + A2/v's) + 1/v'e (B1 + B2/v'e) + K0 (+ a
    // per-step constant common to the step); the margins need E <= R0 = tau/8 - K0 and
    // EV (1/v's + 1/v'e) <= 1/4.  Floats: R0 rounded down, the others up.
    float eb[6];             // R0, A1, A2, B1, B2, EV
};
static_assert(sizeof(CutCmp) == 336, "CutCmp: 84 dwords (bank spread of the 8 groups' rows)");
// The step's operands (CutCmp without bs / be), read from LDS each step.
struct CutReg {
    double ns[5], ne[5], vs[5], ve[5], cc[9], bnd[3];
    float eb[6];
};
__device__ __forceinline__ void cut_reg_load(const CutCmp& c, CutReg& r) {
#pragma unroll
    for (int i = 0; i < 5; ++i) { r.ns[i] = c.ns[i]; r.ne[i] = c.ne[i]; r.vs[i] = c.vs[i]; r.ve[i] = c.ve[i]; }
#pragma unroll
    for (int i = 0; i < 9; ++i) r.cc[i] = c.cc[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) r.bnd[i] = c.bnd[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) r.eb[i] = c.eb[i];
}

// d at (t0, t1), NaN when not healthy; bound_ok: the forward rounding-error bound of
// d (relative, unit roundoff u, first order) is at most tau / 4 (tq = tau / 4 - 4u):
//   40u [(Bs^2 + VsA)(Be^2 + VeA) + Bs^2 Be^2] / D + 16u (VsA / v's + VeA / v'e) + 4u,
// where Bs^2 bounds the absolute terms of Ns and of the Gram entries behind it, Bs Be
// those of C, VsA those of v's (Horner with absolute coefficients at |t|).
// with P1 = (Bs^2 + VsA)(Be^2 + VeA) + Bs^2 Be^2 given
template <bool PROOF>
__device__ __forceinline__ double cut_dcore_p1(double Ns, double Vs, double Ne, double Ve, double C, double P1,
                                              double VsA, double VeA, const float* eb, double tq, int& bound_ok) {
    const double D = __builtin_fma(Vs + Ns, Ve + Ne, -(C * C));
    const double den = Vs * Ve;
    const double r = rcp_fast(den);
    const double d = D * r;
    const double P2 = __builtin_fma(VsA, Ve, VeA * Vs);
    constexpr double u = 0x1p-53;
    const double Dd = D * den;
    const bool healthy = (Vs > 0.0) & (Ve > 0.0) & (D > 0.0) & (d < 1e300) & (Dd < 1e300);
    // agreement with the reference's metric (CutCmp::eb), in f32 with a 1e-4 allowance
    const float iVs = (float)(Ve * r), iVe = (float)(Vs * r);
    const float E = __builtin_fmaf(iVs, __builtin_fmaf(eb[2], iVs, eb[1]), iVe * __builtin_fmaf(eb[4], iVe, eb[3]));
// PROOF: the margins also need the proven agreement bound (cut_proof = 1); measured mode
    // (cut_proof = 0) rests on the measured agreement
    bool agree = true;
    if (PROOF) agree = (E * 1.0001f <= eb[0]) & (eb[5] * (iVs + iVe) <= 0.25f);
    (void)E;
    // (bitwise: every test evaluated, no branch around the forward bound)
    const bool fwd = __builtin_fma((40.0 * u) * P1, den, ((16.0 * u) * P2) * D) <= tq * Dd;
    bound_ok = healthy & agree & fwd;
    return healthy ? d : __longlong_as_double(0x7ff8000000000000ll);
}
// Bs, Be, VsA, VeA are Horner sums of non-negative terms in |t|, increasing in |t|: their values at
// T = max(|rlo|, |rhi|) bound them for every valid neighbour (|t0|, |t1| <= T), so the line's P1,
// VsA, VeA (cmp.bnd, formed when it opens) replace the four per-neighbour evaluations
// (PROOF: v's, v'e are the reference's own endpoint variances at t0, t1, scaled — vs_t, ve_t —
// instead of the quartics)
template <bool PROOF>
__device__ __forceinline__ double cut_dval(const CutReg& c, double t0, double t1, double tq, int& bound_ok,
                                           double vs_t = 0.0, double ve_t = 0.0) {
    const double Ns = h4(c.ns, t0), Ne = h4(c.ne, t1);
    const double Vs = PROOF ? vs_t : h4(c.vs, t0), Ve = PROOF ? ve_t : h4(c.ve, t1);
    const double C = __builtin_fma(t1, __builtin_fma(t1, h2(c.cc[2], c.cc[5], c.cc[8], t0), h2(c.cc[1], c.cc[4], c.cc[7], t0)),
                                   h2(c.cc[0], c.cc[3], c.cc[6], t0));
    return cut_dcore_p1<PROOF>(Ns, Vs, Ne, Ve, C, c.bnd[0], c.bnd[1], c.bnd[2], c.eb, tq, bound_ok);
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
// The group's max by three DPP max steps (exact: max selects an operand), then the lowest lane
// holding it from the wave's ballot — 9 + 4 instructions against 3 x 14 for a (value, index)
// reduction with tie-breaks (the first strict max is the lowest j attaining the max)
template <int CTRL>
__device__ __forceinline__ double dpp_mov_f64(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int group_first_max(double v, int valid, int j, double mc, double& top) {
    const double x = (valid && v == v) ? v : -__builtin_inf();
    double mx = fmax(x, dpp_mov_f64<DPP_XOR1>(x));
    mx = fmax(mx, dpp_mov_f64<DPP_XOR2>(mx));
    mx = fmax(mx, dpp_mov_f64<DPP_HALF_MIRROR>(mx));
    top = mx;
    const unsigned long long at = __ballot((x == mx) & (mx > -__builtin_inf()));
    const unsigned gb = (unsigned)(at >> (threadIdx.x & ~7u)) & 0xFFu;
    const int k = gb ? __builtin_ctz(gb) : 8;
    (void)j;
    return (k < 8 && mx > mc) ? k : -1;
}

// The search block is one wave: LDS accesses of a wave execute in order, so a
// phase boundary only has to keep the compiler from moving LDS accesses across
// it and drain the wave's LDS queue — unlike __syncthreads it does not wait for
// the in-flight global prefetch loads.

// ---- exact step (X), out of line: rare, and its two 6x6 LLTs, reference-order endpoints
// and the exact-sum flush would otherwise set the register budget of the search loop.
struct CutX {
    int best;     // the reference's decision for groups that took the exact step (else unchanged)
    int m_sync;   // sumE now holds the exact invCov_sum before line m_sync (= m for those groups)
};
template <typename T>
__device__ __forceinline__ T* rl_ptr(T* p, int l) {   // lane l's pointer, wave-uniform
    const unsigned long long v = reinterpret_cast<unsigned long long>(p);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}
__device__ __attribute__((noinline)) CutX cut_exact_round(bool exact, int valid, int first, int m, int m_sync, double r0,
                                                          double r1, size_t q_cur, size_t lb, int best,
                                                          const int32_t* mls, const double* rec_l, double* sP, double* eP,
                                                          double* covS, double* covE, double* le_obs, double* cut,
                                                          double* sumE, double* tmp, double* tmpw, const double* Dl,
                                                          double fx, double cb, double homog, double st) {
    const int j = threadIdx.x & 7;
    const int lane = threadIdx.x & 63;
    DevCam cam{};
    cam.fx = fx;
    cam.b = cb;
    DevLines L{};
    L.sP = sP;
    L.eP = eP;
    L.covS = covS;
    L.covE = covE;
    L.le_obs = le_obs;
    L.cut = cut;
    // 1. the exact invCov_sum is brought up to line m (lines m_sync .. m-1 at their final
    //    ratios, stored by lane 0 of the group at each line's finalisation).  The whole wave
    //    serves one group at a time: lane l computes the reference-order info of line
    //    m_sync + l (64 lines per round; eight per round with the group's own lanes made an
    //    exact step cost ~130 us, profiles/r04_ad records), the infos and the lines' r = 0
    //    infos go through the wave's X scratch (idle outside exact rounds and line opens), and
    //    the group's lanes 0-3 add them into sumE in list order, four entries per pass (eight
    //    per pass with the r = 0 infos read from HBM in the chain measured slower, 5.68 vs 5.57 ms;
    //    profiles/r04_af).
    //    Writer and readers are one wave, so a workgroup-scope fence orders them (the
    //    device-scope __threadfence used before wrote back the XCD's L2 every round).
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    {
        unsigned long long need = __ballot(j == 0 && exact && m_sync < m);
        while (need) {   // (wave-uniform)
            const int gl = __ffsll((long long)need) - 1;   // lane 8 G of the group served
            need &= need - 1;
            const int ms = __builtin_amdgcn_readlane(m_sync, gl), me = __builtin_amdgcn_readlane(m, gl);
            const size_t lbG = (size_t)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)lb, gl) |
                               ((size_t)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(lb >> 32), gl) << 32);
            const int32_t* mlsG = rl_ptr(mls, gl);
            const double* recG = rl_ptr(rec_l, gl);
            const double* DlG = rl_ptr(Dl, gl);
            double* sumEG = rl_ptr(sumE, gl);
            const bool mine = (lane >> 3) == (gl >> 3);
            for (int s0 = ms; s0 < me; s0 += 64) {
                const int nl = min(64, me - s0);
                double info[21];
                if (lane < nl) {
                    const size_t qf = lbG + mlsG[s0 + lane];
                    const double c0 = __hip_atomic_load(&L.cut[2 * qf], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    const double c1 = __hip_atomic_load(&L.cut[2 * qf + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    double s7[7], e7[7];
                    exact_endpoint(cam, homog, DlG, L, qf, 0, c0, s7);
                    exact_endpoint(cam, homog, DlG, L, qf, 1, c1, e7);
                    cut_assemble<false>(s7, e7, info);
                }
#pragma unroll
                for (int c = 0; c < 6; ++c) {
                    if (lane < nl) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int e = 4 * c + i;
                            if (e < 21) {
                                tmpw[4 * lane + i] = info[e];
                                tmpw[256 + 4 * lane + i] = recG[(size_t)(s0 + lane) * CUT_REC + CUT_FAST + e];
                            }
                        }
                    }
                    wave_lds_sync();
                    if (mine && j < 4 && 4 * c + j < 21) {
                        const int e = 4 * c + j;
                        double Se = sumEG[e];
                        for (int l = 0; l < nl; ++l) Se = (Se - tmpw[256 + 4 * l + j]) + tmpw[4 * l + j];
                        sumEG[e] = Se;
                    }
                    wave_lds_sync();
                }
            }
            if (mine) m_sync = me;
        }
    }
    // 2. exact endpoints of this step's six slots (lanes 0-2: start endpoint at
    //    r0 + {-s, 0, +s}, lanes 3-5: end endpoint), exact S of line m
    double* const epf = tmp;
    double* const xs = tmp + CUT_EP;
    if (exact) {
        if (j < 6) {
            const int eside = j < 3 ? 0 : 1;
            const double eoff = (j % 3) == 0 ? -st : ((j % 3) == 2 ? st : 0.0);
            const double t = (eside == 0 ? r0 : r1) + eoff;
            double o7[7];
            exact_endpoint(cam, homog, Dl, L, q_cur, eside, t, o7);
#pragma unroll
            for (int i = 0; i < 7; ++i) epf[CUT_SL * j + i] = o7[i];
        }
#pragma unroll
        for (int e = 0; e < 21; ++e) xs[e] = sumE[e] - rec_l[(size_t)m * CUT_REC + CUT_FAST + e];
    }
    wave_lds_sync();
    // 3. the reference's metrics and decision
    if (exact) {
        const int cs = nb_slot(j, 0), ce = 3 + nb_slot(j, 1);
        double mc, top;
        const double vj = cut_exact_step(&epf[CUT_SL * cs], &epf[CUT_SL * ce], &epf[CUT_SL * 1], &epf[CUT_SL * 4], xs,
                                         sumE, first, &mc);
        best = group_first_max(vj, valid, j, mc, top);
    }
    wave_lds_sync();
    return CutX{best, m_sync};
}

// lower-triangle index e (0..20) -> row / column, packed 3 bits per entry
constexpr unsigned long long tri_pack(int want_row) {
    unsigned long long v = 0;
    int e = 0;
    for (int i = 0; i < 6; ++i)
        for (int k = 0; k <= i; ++k, ++e) v |= (unsigned long long)(want_row ? i : k) << (3 * e);
    return v;
}

// The line's agreement bound, out of line (once per line).  Row i = j < 6, with
// s_i = (S^-1)_ii (tg[57 + i]; x 1.002: the solves'
// rounding), S_ii, and the line's operand error bounds e (P units) / ev (v'), into wg[6 q + i]:
//   q = 0 S_ii s_i, 1 sqrt(S_ii s_i), 2 s_i (|P_s,i|(T) + e_s,i)^2, 3 (end side), 4 e_s,i sqrt(s_i),
//   5 e_e,i sqrt(s_i), 6 |log S_ii|, 7 0 (S is the reference's own in proven mode)
__device__ __attribute__((noinline)) void cut_bound_row(int j, double T, const double* fs, const double* sA,
                                                        const double* tg, double* wg) {
    const float* ef = reinterpret_cast<const float*>(fs + PD_ERR);
    const double sg = 1.002 * tg[57 + j];
    const double Sii = sA[tri(j, j)];
    const double es = ef[j], ee = ef[7 + j];
    const double ps = fabs(fs[PD_PS + j]) + T * (fabs(fs[PD_PS + 6 + j]) + T * fabs(fs[PD_PS + 12 + j])) + es;
    const double pe = fabs(fs[PD_PE + j]) + T * (fabs(fs[PD_PE + 6 + j]) + T * fabs(fs[PD_PE + 12 + j])) + ee;
    const double rs = sqrt(sg);
    double row = 0.0;
    // (S is the reference's own, bit for bit, in proven mode: the entrywise difference term is 0)
    const double kc = Sii * sg;
    const int ex = __builtin_amdgcn_frexp_exp(Sii);
    wg[j] = kc;
    wg[6 + j] = sqrt(kc);
    wg[12 + j] = sg * ps * ps;
    wg[18 + j] = sg * pe * pe;
    wg[24 + j] = es * rs;
    wg[30 + j] = ee * rs;
    wg[36 + j] = (Sii > 0.0 && Sii < 1e300) ? 0.6931471805599453 * (double)(abs(ex) + 1) : __builtin_inf();
    wg[42 + j] = row * rs;
}
// ... combined (one lane): eb = R0, A1, A2, B1, B2, EV of CutCmp
__device__ __attribute__((noinline)) void cut_bound_line(double T, double tau, const double* cl, const double* fs,
                                                         const double* wg, float* eb) {
    const float* ef = reinterpret_cast<const float*>(fs + PD_ERR);
    const double Bs = h2(cl[32], cl[33], cl[34], T), Be = h2(cl[35], cl[36], cl[37], T);
    double sum[8];
    for (int q = 0; q < 8; ++q) {
        double a = wg[6 * q];
        for (int i = 1; i < 6; ++i) a = a + wg[6 * q + i];
        sum[q] = a;
    }
    constexpr double u = 0x1p-53;
    const double Kc = sum[0], xi = sum[1], Qs = sum[2], Qe = sum[3], Lam = sum[6];
    const double epsS = sum[7] + (7.01 * u) * xi * xi;                                       // S difference + our factor
    const double hs = sum[4] + (6.01 * u) * Bs * xi, he = sum[5] + (6.01 * u) * Be * xi;   // + the solves' rounding
    // v': the reference's own variance scaled by our fgz2 (the line's v'-table), relative error
    // <= 4 x the blended depth's (ef[6] / ef[13], k_cut_bounds) + the scaling's roundings
    const double rvs = 4.1 * (double)ef[6] + 12.0 * u, rve = 4.1 * (double)ef[13] + 12.0 * u;
    const double ck = 110.0 * u;   // the reference's assembly, LLT and logs, per unit of tr(A~^-1)
    const double K0 = 1.002 * epsS + ck * Kc + (7.1 * u) * Lam;
    const double bs = Bs + hs, be = Be + he;
    // |Delta(1/v')| (B + eta)^2 <= rv (B + eta)^2 / v' (v' within rv <= 1/4 of its value): the
    // rank-one term's v part joins A1 / B1
    const double A1 = 1.03 * (2.0 * ck * Qs + 4.0 * hs * bs + 4.0 * rvs * bs * bs), A2 = 0.0;
    const double B1 = 1.03 * (2.0 * ck * Qe + 4.0 * he * be + 4.0 * rve * be * be), B2 = 0.0;
    double R0 = fmin(0.125 * tau, 1e-3) - 1.01 * K0;
    if (!(epsS <= 1e-3 && Kc <= 1e8 && R0 > 0.0)) R0 = -1.0;
    float r0f = (float)R0;
    if ((double)r0f > R0) r0f = R0 > 0.0 ? __uint_as_float(__float_as_uint(r0f) - 1u) : -1.0f;
    eb[0] = r0f;
    eb[1] = ceil_f32(A1);
    eb[2] = ceil_f32(A2);
    eb[3] = ceil_f32(B1);
    eb[4] = ceil_f32(B2);
    eb[5] = (rvs <= 0.25 && rve <= 0.25) ? 0.0f : __builtin_inff();   // the per-step |ev| <= v'/4 test
}

// Issue priority by progress.  A SIMD holds two search waves with the same work (B = 16384: 300
// lines per sequence, the greedy steps per wave within 2%), yet measured per wave
// (-DGFPL_CUT_CLOCK, profiles/r04_o, r04_r) the one in wave slot 0 finished in 5.2 ms and the one in
// slot 1 in 5.6 ms (up to 6.3), which then ran its end alone.  The two waves of a SIMD publish their
// progress (lines done) in HBM at every line transition and the one ahead of its partner yields
// (priority 0 vs 2); a per-quarter priority ladder measured 6.21 -> 6.15 ms against 6.14 -> 5.84
// (profiles/r04_q, r04_r) and was removed.  The partner is the wave slot ^ 1, checked on the GPU by
// test_cut_progress_partner_slots.
__device__ __forceinline__ int wave_sum8(int v) {   // sum over the wave's 8 groups of lane 8g's value
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return __builtin_amdgcn_readfirstlane(v);
}
// the wave's progress slot and its SIMD partner's (slot ^ 1) in scr.cut_prog: one entry per
// (XCC, SE, SH, CU, SIMD, wave slot) from the HW_ID / XCC_ID registers
struct CutProg { int* own; int* partner; };
__device__ __forceinline__ CutProg cut_prog_slots(int* base) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
    const unsigned simd = ((((xcc & 7u) * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u + ((hw >> 8) & 15u)) * 4u +
                          ((hw >> 4) & 3u);
    const unsigned slot = hw & 15u;
    return CutProg{base + simd * 16u + slot, base + simd * 16u + (slot ^ 1u)};
}
// REC (PROOF false): record every step's decision for k_cut_verify (proven mode's first pass); a
// template parameter so that the measured mode's kernel carries none of its registers
#ifndef GFPL_CUT_WPE
#define GFPL_CUT_WPE 2   // waves per SIMD (2: 256 VGPRs; LDS allows no more: 19 KB per wave)
#endif
// GFPL_CUT_NOPF (experiment): no next-line record prefetch (measured mode reads the record from HBM when
// the line opens, as proven mode does) and 21-double sum rows: 13.5 KB of LDS per wave, so that three
// waves fit a SIMD (with GFPL_CUT_WPE 3)
#ifndef GFPL_CUT_NOPF
#define GFPL_CUT_NOPF 0
#endif
#define CUT_SSTR (GFPL_CUT_NOPF ? 21 : 25)   // sum row stride (doubles; odd multiples of 2 banks apart)
template <bool PROOF, bool REC = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GFPL_CUT_WPE, GFPL_CUT_WPE))) k_cut_search(KParams p) {
    // per-group rows padded to odd strides so the 8 groups of a wave sit in
    // different LDS banks when their lanes read the same entry
    __shared__ double sumA[CUT_G][CUT_SSTR];    // approximate S of the current line (invCov_sum - its r = 0 info)
    __shared__ double sumE[CUT_G][CUT_SSTR];    // exact invCov_sum before line m_sync (lazy, for exact steps)
    __shared__ double fst[CUT_G][CUT_FAST + 1]; // comparison data of the current line
    // next-line records, written by LDS-DMA: 16-B piece k of group g's record lands at
    // nxl[k][16 g + ...] (the DMA writes base + 16 * lane)
    // (proven mode: no prefetch buffer — its v'-tables take the LDS, and 5 KB more would cost the
    // eighth wave of a CU; the record is read from HBM when the line opens)
    constexpr bool PF = !PROOF && !GFPL_CUT_NOPF;   // the next-line record prefetch (measured mode)
    __shared__ __attribute__((aligned(16))) double nxl[PF ? 5 : 1][PF ? 128 : 2];
    // per-group scratch, used either by an exact step (X) or by a line open, never both at once:
    //   X:    exact endpoints of the step's six slots [CUT_EP] | exact S / flush endpoints [25]
    //   open: W coefficient vectors [side * 3 + k][6] (36) | their Gram matrix, lower triangle (21)
    //   open: ... | diag(S^-1) [57..62]; the agreement bound's per-row partials over [0..48)
    //   transition: the finished line's error bounds (+ evaluation) [0..14)
    __shared__ double tmp[CUT_G][CUT_EP + 25 + 1];
    static_assert(CUT_G * (CUT_EP + 25 + 1) >= 512, "the exact-sum flush stages 64 x (4 + 4) doubles in tmp");
    __shared__ CutCmp cmpl[CUT_G];              // comparison polynomials of the current line
    // proven mode: the line's v'_ref at every ratio key (side * CUT_KS + slot; k_cut_vtab) and the
    // keys' +s / -s links (KParams::cut_keys; -1: no key — such a ratio is evaluated exactly)
    __shared__ double vtab[PROOF ? CUT_G : 1][PROOF ? 2 * CUT_KS : 1];
    __shared__ int cnxt[PROOF ? CUT_KS : 1], cprv[PROOF ? CUT_KS : 1];
    const int lane = threadIdx.x;
#ifdef GFPL_CUT_CLOCK
    const uint64_t t_beg = wall_clock64();   // (diagnostic build: the wave's duration in record slot 19)
#endif
    const int g = lane >> 3, j = lane & 7;
    const int b = blockIdx.x * CUT_G + g;
    if (!PROOF && p.cfg.cut_proof == 0 && j == 0 && b < p.B) {
        // the wave's HW_ID / XCC_ID in the debug slots 6 / 7 of its sequences (measured mode; read by
        // tests/test_gpu_parity.py::test_cut_progress_partner_slots: the progress exchange's slot ^ 1)
        p.scr.dbg[8 * (size_t)b + 6] = (int64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        p.scr.dbg[8 * (size_t)b + 7] = (int64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
    // proven mode (cut_proof 1 / 3): the eager-proven search runs only for the sequences whose
    // recorded search k_cut_verify did not prove (cut_flag); cut_proof 2 runs it for all of them
    const bool live = b < p.B && (!PROOF || p.cfg.cut_proof == 2 || p.scr.cut_flag[b] != 0);
    const int nls = live ? p.tr.n_matched_ls[b] : 0;
    // proven mode, first pass (the measured search): every step's decision is recorded for
    // k_cut_verify — one byte per step and line, CUT_PATH per line
    constexpr bool rec = !PROOF && REC;
    uint8_t* const path = p.scr.cut_path + (size_t)(live ? b : 0) * p.mls_cap * CUT_PATH;
    int lstep = 0;       // steps taken on the current line
    // REC: the current line's recorded steps, per group (stored to HBM when the line finishes)
    __shared__ __attribute__((aligned(8))) uint8_t pth[REC ? CUT_G : 1][REC ? CUT_PATH : 8];
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    const double tau = p.cfg.cut_certify;
    const double tq = p.cut_tq;   // d's bound budget tau / 4 - 4u (cut_dcore_p1; a kernel argument: SGPRs)
    DevLines& L = p.prev.ls;
    const size_t lb = (size_t)(live ? b : 0) * p.kl_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)(live ? b : 0) * p.mls_cap;
    const double* rec_l = p.scr.cut_rec + (size_t)(live ? b : 0) * p.mls_cap * CUT_REC;
    const double* Dl = p.scr.cut_dtinv + 16 * (size_t)(live ? b : 0);   // DT_inv (exact steps only)
    const double st = p.cfg.cut_step;
    const double rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    double* const xs = &tmp[g][CUT_EP];
    double* const wg = &tmp[g][0];
    double* const gm = &tmp[g][36];
    // neighbour j of this lane
    const double nb0 = nb_step(j, 0, st), nb1 = nb_step(j, 1, st);
    constexpr unsigned long long TRI_ROW = tri_pack(1), TRI_COL = tri_pack(0);
    if (PROOF) {   // the ratio keys and their links (host-formed, KParams)
        if (lane < CUT_KS) {
            cnxt[lane] = p.cut_knxt[lane];
            cprv[lane] = p.cut_kprv[lane];
        }
        __syncthreads();
    }
    // group state (identical in the 8 lanes of a group)
    int m = 0;
    int m_sync = 0;      // sumE holds the exact invCov_sum before line m_sync
    int first = 1;       // first step of the line: the exact centre metric is logdet(invCov_sum)
    double r0 = 0.0, r1 = 0.0;
    int line_ok = 0;     // margined comparisons allowed on the current line
    int pend = 0;        // the line finished; the next one opens at the next transition
    int wait = 0;        // iterations spent waiting for that transition
    double dc = 0.0;     // d of the centre
    int c_ok = 0;        // its error bound is within tau / 4
    int n_unb = 0;       // lines opened without a usable agreement bound
    // proven mode: the key slots of r0 / r1 and of their +s / -s neighbours (-1: none)
    int i0 = 0, i1 = 0, n0s = -1, p0s = -1, n1s = -1, p1s = -1;
    size_t q_cur = 0, q_nx = 0;   // the current / next line (global index)
    // A line opens (its data in fst, S in registers): every lane factors S (identical
    // values), lane k < 6 solves W_k = L^-1 P_k (side k / 3, power k % 3), lane j forms
    // Gram entries j, j + 8, j + 16, and every lane reads the 21 back into its
    // comparison polynomials.  Margins need the factor healthy and PD_OK.
    auto open_line = [&]() {
        if (PROOF) {   // the line's v'_ref at every key, both sides (k_cut_vtab), and r = (0, 0)'s slots
            const double* vt = p.scr.cut_vtab + ((size_t)(live ? b : 0) * p.mls_cap + m) * (2 * CUT_KS);
            for (int idx = j; idx < 2 * CUT_KS; idx += 8) vtab[g][idx] = vt[idx];
            i0 = 0;
            i1 = 0;
            n0s = n1s = cnxt[0];
            p0s = p1s = cprv[0];
        }
        double o[28];
        {
            double S[21];
#pragma unroll
            for (int e = 0; e < 21; ++e) S[e] = sumA[g][e];
            chol_s(S, o);
        }
        line_ok = (o[27] != 0.0) && (fst[g][PD_OK] != 0.0);
        if (j < 6) {
            double w[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double u = fst[g][6 * j + i];
#pragma unroll
                for (int k = 0; k < i; ++k) u = __builtin_fma(-o[tri(i, k)], w[k], u);
                w[i] = u * o[21 + i];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) wg[6 * j + i] = w[i];
            // (S^-1)_jj = |L^-1 e_j|^2 for the agreement bound
            double x[6], sg = 0.0;
            if (PROOF) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double uu = i == j ? 1.0 : 0.0;
#pragma unroll
                for (int k = 0; k < i; ++k) uu = __builtin_fma(-o[tri(i, k)], x[k], uu);
                x[i] = uu * o[21 + i];
                sg = __builtin_fma(x[i], x[i], sg);
            }
            tmp[g][57 + j] = sg;
            }
        }
        wave_lds_sync();
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) {
            const int e = j + 8 * kk;
            if (e < 21) {
                const int ra = (int)((TRI_ROW >> (3 * e)) & 7), cb = (int)((TRI_COL >> (3 * e)) & 7);
                double s = wg[6 * ra] * wg[6 * cb];
#pragma unroll
                for (int i = 1; i < 6; ++i) s = __builtin_fma(wg[6 * ra + i], wg[6 * cb + i], s);
                gm[e] = s;
            }
        }
        wave_lds_sync();
        // the comparison polynomials, written straight into cmpl by the lanes:
        //   lanes 0 / 1: ns / ne (side j), lanes 2 / 3: v'_s / v'e copies,
        //   lanes 4-6: cc[3 i + k] (i = j - 4) and the bounds bs[i], be[i]
        double* cl = reinterpret_cast<double*>(&cmpl[g]);
        if (j < 2) {
            const int a = 3 * j, b2 = a + 1, c2 = a + 2;
            double* o = cl + 5 * j;   // ns | ne
            o[0] = gm[tri(a, a)];
            o[1] = 2.0 * gm[tri(b2, a)];
            o[2] = __builtin_fma(2.0, gm[tri(c2, a)], gm[tri(b2, b2)]);
            o[3] = 2.0 * gm[tri(c2, b2)];
            o[4] = gm[tri(c2, c2)];
        } else if (j < 4) {
#pragma unroll
            for (int i = 0; i < 5; ++i) cl[10 + 5 * (j - 2) + i] = fst[g][PD_VS + 5 * (j - 2) + i];
        } else if (j < 7) {
            const int i = j - 4;
#pragma unroll
            for (int k = 0; k < 3; ++k) cl[20 + 3 * i + k] = gm[tri(3 + k, i)];
            // |W| with a 1% allowance for the approximate square root (bounds only)
            const double gs = fmax(gm[tri(i, i)], 0.0), ge = fmax(gm[tri(3 + i, 3 + i)], 0.0);
            cl[32 + i] = gs > 0.0 ? 1.01 * gs * __builtin_amdgcn_rsq(gs) : 0.0;
            cl[35 + i] = ge > 0.0 ? 1.01 * ge * __builtin_amdgcn_rsq(ge) : 0.0;
        }
        wave_lds_sync();
        // the line's bound terms at T (lane 7; see cut_dval), and lanes 0-5 the per-row terms of
        // the agreement bound, row i = j: with s_i = (S^-1)_ii (x 1.002: the
        // solves' rounding), S_ii, and the line's
        // operand error bounds e (P units) / ev (v'):
        //   [0] S_ii s_i  [1] sqrt(S_ii s_i)  [2] s_i (|P_s,i|(T) + e_s,i)^2  [3] (end side)
        //   [4] e_s,i sqrt(s_i)  [5] e_e,i sqrt(s_i)  [6] |log S_ii|  [7] 0
        // the line's bound terms at T (lane 7; see cut_dval), and the line's agreement bound
        // (CutCmp::eb): per-row terms by lanes 0-5, combined by lane 7
        const double T = fmax(fabs(rlo), fabs(rhi));
        if (j == 7) {
            const double Bs = h2(cl[32], cl[33], cl[34], T), Be = h2(cl[35], cl[36], cl[37], T);
            const double VsA = h4abs(cl + 10, T), VeA = h4abs(cl + 15, T);
            const double Bs2 = Bs * Bs, Be2 = Be * Be;
            cl[29] = __builtin_fma(Bs2 + VsA, Be2 + VeA, Bs2 * Be2);
            cl[30] = VsA;
            cl[31] = VeA;
        } else if (PROOF && j < 6) {
            cut_bound_row(j, T, fst[g], sumA[g], tmp[g], wg);
        }
        wave_lds_sync();
        if (PROOF && j == 7) cut_bound_line(T, tau, cl, fst[g], wg, cmpl[g].eb);
        wave_lds_sync();
        if (PROOF) {   // the line's bound, kept in its record (slots CUT_NX.., diagnostics) and counted if unusable
            const float* e6 = cmpl[g].eb;
            bool usable = e6[0] > 0.0f;
#pragma unroll
            for (int i = 1; i < 6; ++i) usable = usable && e6[i] < __builtin_inff();
            n_unb += usable ? 0 : 1;
            if (j < 6 && live) reinterpret_cast<float*>(const_cast<double*>(rec_l) + (size_t)m * CUT_REC + CUT_NX)[j] = e6[j];
        }
        // the centre of the first step: d at (0, 0)
        const double vs0 = PROOF ? vtab[g][0] : cl[10], ve0 = PROOF ? vtab[g][CUT_KS] : cl[15];
        dc = cut_dcore_p1<PROOF>(cl[0], vs0, cl[5], ve0, cl[20], cl[29], cl[30], cl[31], cmpl[g].eb, tq, c_ok);
    };
    // Next-line prefetch: right after a line opens the group's lanes copy the next line's
    // record (640 B) from HBM straight into LDS (global_load_lds, no registers); it is
    // waited for (vmcnt) and moved into fst / nxi when that line opens, >= 1 iteration later.
    // The DMA is issued by inline asm: the compiler treats a pending __builtin_amdgcn_global_load_lds
    // as a write to any LDS and put an s_waitcnt vmcnt(0) before the next step's first LDS read, so the
    // record's HBM latency was exposed right after the line opened; the only reader of nxl waits for
    // it explicitly (the transition's vmcnt(0)).  An op the compiler does not count can only make its
    // own vmcnt waits stricter (loads complete in order).
    auto pf_issue = [&](int mm) {
        if (!PF) return;
        const char* src = reinterpret_cast<const char*>(rec_l + (size_t)mm * CUT_REC) + 16 * j;
#pragma unroll
        for (int k = 0; k < (PF ? 5 : 0); ++k) {
            const uint32_t dst = (uint32_t)(uintptr_t)&nxl[k][0];   // LDS byte address (M0; lane l lands at + 16 l)
            asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src + 128 * k), "s"(dst)
                         : "memory", "m0");
        }
    };
    if (m < nls) {
        q_cur = lb + mls[0];
        if (nls > 1) q_nx = lb + mls[1];
        for (int e = j; e < CUT_FAST; e += 8) fst[g][e] = rec_l[e];
#pragma unroll
        for (int e = j; e < 21; e += 8) {
            const double s0 = p.scr.cut_sum[24 * b + e];
            sumA[g][e] = s0 - rec_l[CUT_FAST + e];
            sumE[g][e] = s0;
        }
        wave_lds_sync();
        open_line();
        if (nls > 1) pf_issue(1);
    }
    __syncthreads();
    int n_steps = 0, n_exact = 0;   // this sequence's search steps, and those evaluated exactly
    const CutProg prog = cut_prog_slots(p.scr.cut_prog);
    if (lane == 0) __hip_atomic_store(prog.own, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int partner_done = 0;   // the partner's lines done as read at the previous transition
    // measured mode: the partner's progress word is fetched by an untracked LDS DMA (lane 0) at the
    // end of a transition and read at the next one, after its vmcnt(0): as a load into a register the
    // compiler waited for it at once (a copy into the loop-carried register, then a WAW hazard on
    // that register at the next step's first LDS read), exposing its HBM latency every transition
    __shared__ int pslot[1];
    if (!PROOF && lane == 0) pslot[0] = 0;
    __builtin_amdgcn_s_setprio(2);
#ifdef GFPL_CUT_PCLOCK   // (diagnostic build: shader-clock cycles per phase of the wave in scr.dbg 0-3:
                         //  step evaluation + decision, exact rounds, bookkeeping, transitions)
    uint64_t pk[4] = {0, 0, 0, 0};
    uint64_t pk0 = clock64();
    int n_it = 0, n_tr = 0;   // loop iterations, transitions (scr.dbg 7: n_it << 32 | n_tr)
    uint64_t tk[3] = {0, 0, 0}, tk0 = 0;   // transition phases (scr.dbg 4-6): finished line's info + next
                                           // line's record and S, open_line + prefetch, progress exchange
#define PCK(i) do { const uint64_t t_ = clock64(); pk[i] += t_ - pk0; pk0 = t_; } while (0)
#define TCK0() do { tk0 = clock64(); } while (0)
#define TCK(i) do { const uint64_t t_ = clock64(); tk[i] += t_ - tk0; tk0 = t_; } while (0)
#else
#define PCK(i) do { } while (0)
#define TCK0() do { } while (0)
#define TCK(i) do { } while (0)
#endif
    while (__any(m < nls)) {   // wave-uniform loop; groups that are done idle
        const bool act = m < nls && !pend;
        // ---- lane j: d of neighbour j; the group decision and its margins
        const double t0 = r0 + nb0, t1 = r1 + nb1;
        int valid = act ? 1 : 0;
        if (t0 + t1 > 1.0) valid = 0;
        if (t0 < rlo || t0 > rhi) valid = 0;
        if (t1 < rlo || t1 > rhi) valid = 0;
        int bok;
        double dj;
        CutReg cr;
        cut_reg_load(cmpl[g], cr);   // the line's operands from LDS, every step (a register-resident
                                     // copy reloaded only after transitions / exact rounds measured
                                     // 7.00 vs 6.70 ms: its spills around those blocks cost more)
        double vst = 0.0, vet = 0.0;
        if (PROOF) {   // the reference's v' at t0 / t1 from the line's key table (no key: NaN, exact)
            const int s0 = nb0 > 0.0 ? n0s : (nb0 < 0.0 ? p0s : i0);
            const int s1 = nb1 > 0.0 ? n1s : (nb1 < 0.0 ? p1s : i1);
            vst = s0 >= 0 ? vtab[g][s0] : __longlong_as_double(0x7ff8000000000000ll);
            vet = s1 >= 0 ? vtab[g][CUT_KS + s1] : __longlong_as_double(0x7ff8000000000000ll);
        }
        dj = cut_dval<PROOF>(cr, t0, t1, tq, bok, vst, vet);
        double top;
        int best = group_first_max(dj, valid, j, dc, top);
        // every comparison the decision rests on must clear the margin, every d its
        // error bound; NaN (unhealthy) values fail every test
        // (bitwise, every comparison evaluated: no branches in the step)
        const bool has = best >= 0, vl = valid != 0;
        const bool f1 = vl & !bok;
        const bool f2 = has & vl & (j != best) & !(top - dj > tau * top);
        const bool f3 = has & !(top - dc > tau * top);
        const bool f4 = !has & vl & !(dc - dj > tau * dc);
        const bool f5 = !((tau > 0.0) & (line_ok != 0) & (c_ok != 0) & (dc == dc));
        const int ok = (f1 | f2 | f3 | f4 | f5) ? 0 : 1;
        const bool exact = act && ((__ballot(!ok) >> (8 * g)) & 0xFFull) != 0;   // (the group's 8 bits)
        n_steps += act ? 1 : 0;
        n_exact += exact ? 1 : 0;
        double dnext = top;   // d of the next centre (the chosen neighbour, same bits)
        int cnext = 1;
        PCK(0);
        if (__any(exact)) {
            // ---- X: the reference's evaluation of this step for the groups that need it
            const CutX xr = cut_exact_round(exact, valid, first, m, m_sync, r0, r1, q_cur, lb, best, mls, rec_l, L.sP, L.eP,
                                            L.covS, L.covE, L.le_obs, L.cut, sumE[g], tmp[g], &tmp[0][0], Dl, cam.fx, cam.b,
                                            homog, st);
            best = xr.best;
            m_sync = xr.m_sync;
            // the next centre's d and bound come from the lane that evaluated it
            const int src = (lane & ~7) + (best >= 0 ? best : 0);
            const double sd = __shfl(dj, src);
            const int sb = __shfl(bok, src);
            if (exact) { dnext = sd; cnext = sb; }
        }
        PCK(1);
        int finalize = 0;
        if (rec && act) {   // move j | CUT_P_STAY (no better neighbour) | CUT_P_EXACT, into the group's LDS row
            if (j == 0 && lstep < CUT_PATH)
                pth[g][lstep] = (uint8_t)((best >= 0 ? best : CUT_P_STAY) | (exact ? CUT_P_EXACT : 0));
            ++lstep;   // (every lane of the group: they store the row's 8-byte blocks)
        }
        if (act) {
            first = 0;
            if (best >= 0) {
                if (PROOF) {   // the new ratios' key slots (r + s, r - s, r: the table's links)
                    const double a0 = nb_step(best, 0, st), a1 = nb_step(best, 1, st);
                    i0 = i0 < 0 ? -1 : (a0 > 0.0 ? n0s : (a0 < 0.0 ? p0s : i0));
                    i1 = i1 < 0 ? -1 : (a1 > 0.0 ? n1s : (a1 < 0.0 ? p1s : i1));
                    n0s = i0 >= 0 ? cnxt[i0] : -1;
                    p0s = i0 >= 0 ? cprv[i0] : -1;
                    n1s = i1 >= 0 ? cnxt[i1] : -1;
                    p1s = i1 >= 0 ? cprv[i1] : -1;
                }
                r0 = r0 + nb_step(best, 0, st);
                r1 = r1 + nb_step(best, 1, st);
                dc = dnext;
                c_ok = cnext;
                if (!(r0 + r1 <= 1.0)) finalize = 1;   // while-condition
            } else {
                finalize = 1;
            }
        }
        if (rec && act && finalize && m + 1 >= nls) {   // the last line's recorded steps to HBM: 8 bytes per
            __builtin_amdgcn_wave_barrier();                // group lane (the others' at their transition)
            if (8 * j < lstep)
                *reinterpret_cast<unsigned long long*>(path + (size_t)m * CUT_PATH + 8 * j) =
                    *reinterpret_cast<const unsigned long long*>(&pth[g][8 * j]);
        }
        if (act && finalize) {
            // (measured mode: the cut of a line with a successor is stored at the transition, after its
            // vmcnt wait, so that wait does not include these stores' write acknowledgements; nothing
            // reads it before: an exact round's flush serves lines below its own group's open line)
            if (j == 0 && (PROOF || m + 1 >= nls)) {
                L.cut[2 * q_cur] = r0;
                L.cut[2 * q_cur + 1] = r1;
            }
            ++m;
            pend = m < nls;   // the next line opens at the next transition
            wait = 0;
        }
        // Transitions are batched: a group whose line finished waits (no steps) until
        // CUT_BATCH groups of the wave wait, one has waited CUT_WAIT iterations, or no
        // group has steps left; one transition then serves all of them, so the wave
        // pays its serial chain (factor, solves, LDS exchanges) fewer times.
        PCK(2);
        const int npend = __popcll(__ballot(pend)) >> 3;
#ifdef GFPL_CUT_PCLOCK
        ++n_it;
#endif
        if (npend > 0 && (npend >= CUT_BATCH || __any(pend && wait >= CUT_WAIT) || __ballot(m < nls && !pend) == 0)) {
#ifdef GFPL_CUT_PCLOCK
            ++n_tr;
#endif
            TCK0();
            double info[3];
            if (pend) {
                // approximate invCov_sum += info of the chosen ratio (the exact one is
                // accumulated lazily, only when an exact step needs it):
                // info = Ps Ps^T / v's + Pe Pe^T / v'e (the fgz2 factors cancel)
                // lane i < 6: entry i of Ps and Pe at the final ratios, lane 6 / 7: v's / v'e;
                // with PD_OK = 0 (the segment leaves the polynomial form's domain, rare)
                // lanes 0 / 1 write the reference-order endpoints (v, J) instead, J Js^T / v
                // being the same matrix as P P^T / v'
                if (!PROOF && fst[g][PD_OK] != 0.0) {   // (proven mode: the reference's endpoints, below)
                    if (j < 6) {
                        xs[1 + j] = cut_ours_P(fst[g], 0, j, r0);
                        xs[8 + j] = cut_ours_P(fst[g], 1, j, r1);
                    } else {
                        xs[7 * (j - 6)] = cut_ours_V(fst[g], j - 6, j == 6 ? r0 : r1);
                    }
                } else if (j < 2) {
                    double o7[7];
                    exact_endpoint(cam, homog, Dl, L, q_cur, j, j ? r1 : r0, o7);
#pragma unroll
                    for (int i = 0; i < 7; ++i) xs[7 * j + i] = o7[i];
                }
            }
            wave_lds_sync();   // the finished line's data is read before it is replaced
            if (pend) {
                // lane j: entries j, j + 8, j + 16 of info = Ps Ps^T / v's + Pe Pe^T / v'e; proven
                // mode: the reference's own assembly of its endpoints (cut_assemble's expressions,
                // entry by entry), so sumA / sumE stay the reference's invCov_sum bit for bit
                const double is = rcp_fast(xs[0]), ie = rcp_fast(xs[7]);
                const double invdet = 1.0 / (xs[0] * xs[7] - 0.0 * 0.0);
                const double i00 = xs[7] * invdet, i10 = -0.0 * invdet, i01 = -0.0 * invdet, i11 = xs[0] * invdet;
#pragma unroll
                for (int kk = 0; kk < 3; ++kk) {
                    const int e = min(j + 8 * kk, 20);   // entries past 20 are computed and dropped
                    const int ra = (int)((TRI_ROW >> (3 * e)) & 7), cb = (int)((TRI_COL >> (3 * e)) & 7);
                    if (PROOF) {
                        const double T0 = xs[1 + ra] * i00 + xs[8 + ra] * i10, T1 = xs[1 + ra] * i01 + xs[8 + ra] * i11;
                        info[kk] = T0 * xs[1 + cb] + T1 * xs[8 + cb];
                    } else {
                        info[kk] = cut_ours_info(xs, is, ie, ra, cb);
                    }
                }
                // line m from its prefetched record (the DMA was issued >= 1 iteration ago)
                if (!PF) {
#pragma unroll
                    for (int k = 0; k < CUT_FAST / 8; ++k) fst[g][j + 8 * k] = rec_l[(size_t)m * CUT_REC + j + 8 * k];
                }
                if (!PROOF) {
                    if (PF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (j == 0) {   // the finished line's cut (deferred from its finalisation)
                        L.cut[2 * q_cur] = r0;
                        L.cut[2 * q_cur + 1] = r1;
                    }
                    if (rec && 8 * j < lstep)   // ... and its recorded steps (line m - 1: m moved on)
                        *reinterpret_cast<unsigned long long*>(path + (size_t)(m - 1) * CUT_PATH + 8 * j) =
                            *reinterpret_cast<const unsigned long long*>(&pth[g][8 * j]);
#pragma unroll
                    for (int k = 0; k < (PF ? CUT_FAST / 8 : 0); ++k) {
                        const int e = j + 8 * k;
                        fst[g][e] = nxl[e >> 4][16 * g + (e & 15)];
                    }
                }
            }
            wave_lds_sync();
            if (pend) {
                q_cur = q_nx;
                q_nx = lb + (size_t)(int)fst[g][PD_NEXT];
                if (PROOF) m_sync = m;   // sumE was brought up to line m above
                first = 1;
                lstep = 0;
                r0 = 0.0;
                r1 = 0.0;
#pragma unroll
                for (int kk = 0; kk < 3; ++kk) {
                    const int e = j + 8 * kk;
                    const int x = CUT_FAST + e;   // the new line's r = 0 info, straight from its record
                    if (e < 21) {
                        const double mid = sumA[g][e] + info[kk];
                        const double nw = mid - (PF ? nxl[x >> 4][16 * g + (x & 15)] : rec_l[(size_t)m * CUT_REC + x]);
                        sumA[g][e] = nw;
                        if (PROOF) sumE[g][e] = mid;   // the exact invCov_sum, kept current (m_sync = m)
                    }
                }
            }
            wave_lds_sync();
            TCK(0);
            if (pend) {   // group-uniform; open_line exchanges through LDS only
                open_line();
                if (m + 1 < nls) pf_issue(m + 1);
                pend = 0;
            }
            TCK(1);
            {
                // (measured mode: the word the previous transition's DMA landed, after this
                // transition's vmcnt(0))
                if (!PROOF) partner_done = pslot[0];
                const int done = wave_sum8(j == 0 ? m : 0);
                if (done > __builtin_amdgcn_readfirstlane(partner_done)) __builtin_amdgcn_s_setprio(0);
                else __builtin_amdgcn_s_setprio(2);
                if (lane == 0) __hip_atomic_store(prog.own, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (PROOF) {
                    partner_done = __hip_atomic_load(prog.partner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // used next time
                } else if (lane == 0) {
                    const uint32_t dst = (uint32_t)(uintptr_t)&pslot[0];
                    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off sc1" ::"v"(prog.partner), "s"(dst)
                                 : "memory", "m0");
                }
            }
            TCK(2);
        } else if (pend) {
            ++wait;
        }
        PCK(3);
    }
#ifdef GFPL_CUT_PCLOCK
    if (live && j == 0)
        for (int i = 0; i < 4; ++i) p.scr.dbg[8 * (size_t)b + i] = (int64_t)pk[i];
    if (live && j == 0) {
        for (int i = 0; i < 3; ++i) p.scr.dbg[8 * (size_t)b + 4 + i] = (int64_t)tk[i];
        p.scr.dbg[8 * (size_t)b + 7] = ((int64_t)n_it << 32) | n_tr;
    }
#endif
#undef PCK
#undef TCK0
#undef TCK
    if (live && j == 0) {
        p.scr.bytes[(size_t)STEP_REC * b + 16] = n_steps;
        p.scr.bytes[(size_t)STEP_REC * b + 17] = n_exact;
        p.scr.bytes[(size_t)STEP_REC * b + 19] = n_unb;
#ifdef GFPL_CUT_CLOCK
        const uint64_t t_end = wall_clock64();
        p.scr.bytes[(size_t)STEP_REC * b + 19] = (int64_t)(t_end - t_beg);
        p.scr.dbg[8 * (size_t)b + 0] = (int64_t)t_beg;
        p.scr.dbg[8 * (size_t)b + 1] = (int64_t)t_end;
        p.scr.dbg[8 * (size_t)b + 2] = (int64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
        p.scr.dbg[8 * (size_t)b + 3] = (int64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // XCC_ID
#endif
    }
}

// ------------------------------------------------------- small-batch search --
// One sequence per wave, for small batches (B <= CUT_WAVE_MAX_B: the latency of one sequence, e.g. the
// reference app's one stream per process, app/plslam_mod.cpp:387-411).  Same decisions, same bits as
// k_cut_search<false> (measured mode, with the proven mode's step record): a round evaluates d on the 8 x 8
// grid of ratios at offsets -1 .. 6 from the centre on both sides (lane a * 8 + c), takes every interior
// position's decision at once (the one-step search's first-strict-maximum rule and margin tests over its
// 8 neighbours' values), then follows the decisions from the centre as far as they stay inside the grid.
// The greedy paths are runs of moves growing both ratios followed by runs growing one (oracle move
// statistics on cfg2: 80% (+,+), 10% (+,0), 10% (0,+), moves back 0.03%): 2.3 rounds per line against
// 3.0 with a five-step cap, and no 64-cell shape of the grid does better (profiles/r05_cutw).  The grid's
// ratios are accumulated as the search's moves accumulate them (r + s + s ...); a position whose
// neighbours' ratio bits differ from the grid's or leave it (a ratio that moved back), or that a margin
// test sends to the exact path, ends the round.  Exact steps and the lazy exact invCov_sum are
// cut_exact_round's, run by the wave as group 0.  Line transitions run on the whole wave at once.
#ifndef CUT_WAVE_MAX_B
#define CUT_WAVE_MAX_B 2048
#endif
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int nb_da(int j, int side) {   // neighbour j's offset on a side (nb_step's sign)
    return nb_off(j, side);
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_cut_search_w(KParams p) {
    __shared__ double sumA[25];                 // approximate S of the current line
    __shared__ double sumE[25];                 // exact invCov_sum before line m_sync (lazy, exact steps)
    __shared__ double fst[CUT_FAST + 1];        // comparison data of the current line
    __shared__ double tmp[CUT_G][CUT_EP + 25 + 1];   // exact round: row 0 | the flush staging (all rows)
    __shared__ double wgs[64];                  // line open: W [6][6] | Gram (21) at 36
    __shared__ double xsl[16];                  // transition: the finished line's [v'_s, P_s, v'_e, P_e]
    __shared__ CutCmp cmpl;
    __shared__ double dgx[100];                 // decision pass: the grid's values (-inf: invalid / NaN), padded,
    __shared__ int dgf[100];                    // and flags (bok | valid << 1 | valid NaN << 2); alt values at 82
    const int lane = threadIdx.x;
    const int b = blockIdx.x;
    const int nls = p.tr.n_matched_ls[b];
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    const double tau = p.cfg.cut_certify;
    const double tq = p.cut_tq;
    DevLines& L = p.prev.ls;
    const size_t lb = (size_t)b * p.kl_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    const double* rec_l = p.scr.cut_rec + (size_t)b * p.mls_cap * CUT_REC;
    const double* Dl = p.scr.cut_dtinv + 16 * (size_t)b;
    const double st = p.cfg.cut_step;
    const double rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    const bool rec = p.cfg.cut_proof != 0;
    uint8_t* const path = p.scr.cut_path + (size_t)b * p.mls_cap * CUT_PATH;
    constexpr unsigned long long TRI_ROW = tri_pack(1), TRI_COL = tri_pack(0);
    int m = 0, m_sync = 0, first = 1, line_ok = 0, c_ok = 0, lstep = 0;
    double r0 = 0.0, r1 = 0.0, dc = 0.0;
    size_t q_cur = 0;
    int n_steps = 0, n_exact = 0;
    // A line opens (fst and sumA hold its data): the k_cut_search<false> open, one lane per role
#ifdef GFPL_CUTW_TCLOCK   // (diagnostic build: line-transition phases in scr.dbg 0-7)
    uint64_t tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tk0 = clock64();
#define TCK(i) do { const uint64_t t_ = clock64(); tk[i] += t_ - tk0; tk0 = t_; } while (0)
#else
#define TCK(i) do { } while (0)
#endif
    auto open_line = [&]() {
        double o[28];
        {
            double S[21];
#pragma unroll
            for (int e = 0; e < 21; ++e) S[e] = sumA[e];
            chol_s(S, o);
        }
        TCK(2);
        line_ok = (o[27] != 0.0) && (fst[PD_OK] != 0.0);
        if (lane < 6) {
            double w[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double u = fst[6 * lane + i];
#pragma unroll
                for (int k = 0; k < i; ++k) u = __builtin_fma(-o[tri(i, k)], w[k], u);
                w[i] = u * o[21 + i];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) wgs[6 * lane + i] = w[i];
        }
        wave_lds_sync();
        TCK(3);
        if (lane < 21) {
            const int ra = (int)((TRI_ROW >> (3 * lane)) & 7), cb = (int)((TRI_COL >> (3 * lane)) & 7);
            double s = wgs[6 * ra] * wgs[6 * cb];
#pragma unroll
            for (int i = 1; i < 6; ++i) s = __builtin_fma(wgs[6 * ra + i], wgs[6 * cb + i], s);
            wgs[36 + lane] = s;
        }
        wave_lds_sync();
        TCK(4);
        // the line's comparison data (cmpl), formed by every lane in registers (no per-role branches and
        // LDS round trips), stored by lane 0 for the rounds' cut_reg_load
        const double* gm = wgs + 36;
        double* cl = reinterpret_cast<double*>(&cmpl);
        double G[21], cv[38];
#pragma unroll
        for (int e = 0; e < 21; ++e) G[e] = gm[e];
#pragma unroll
        for (int i = 0; i < 10; ++i) cv[10 + i] = fst[PD_VS + i];
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
            const int a0 = 3 * sd, b2 = a0 + 1, c2 = a0 + 2;
            cv[5 * sd + 0] = G[tri(a0, a0)];
            cv[5 * sd + 1] = 2.0 * G[tri(b2, a0)];
            cv[5 * sd + 2] = __builtin_fma(2.0, G[tri(c2, a0)], G[tri(b2, b2)]);
            cv[5 * sd + 3] = 2.0 * G[tri(c2, b2)];
            cv[5 * sd + 4] = G[tri(c2, c2)];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int k = 0; k < 3; ++k) cv[20 + 3 * i + k] = G[tri(3 + k, i)];
            const double gs = fmax(G[tri(i, i)], 0.0), ge = fmax(G[tri(3 + i, 3 + i)], 0.0);
            cv[32 + i] = gs > 0.0 ? 1.01 * gs * __builtin_amdgcn_rsq(gs) : 0.0;
            cv[35 + i] = ge > 0.0 ? 1.01 * ge * __builtin_amdgcn_rsq(ge) : 0.0;
        }
        {
            const double T = fmax(fabs(rlo), fabs(rhi));
            const double Bs = h2(cv[32], cv[33], cv[34], T), Be = h2(cv[35], cv[36], cv[37], T);
            const double VsA = h4abs(cv + 10, T), VeA = h4abs(cv + 15, T);
            const double Bs2 = Bs * Bs, Be2 = Be * Be;
            cv[29] = __builtin_fma(Bs2 + VsA, Be2 + VeA, Bs2 * Be2);
            cv[30] = VsA;
            cv[31] = VeA;
        }
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 38; ++i) cl[i] = cv[i];
        }
        wave_lds_sync();
        TCK(5);
        dc = cut_dcore_p1<false>(cv[0], cv[10], cv[5], cv[15], cv[20], cv[29], cv[30], cv[31], cmpl.eb, tq, c_ok);
        TCK(6);
    };
    if (nls > 0) {
        q_cur = lb + mls[0];
        for (int e = lane; e < CUT_FAST; e += 64) fst[e] = rec_l[e];
        if (lane < 21) {
            const double s0 = p.scr.cut_sum[24 * b + lane];
            sumA[lane] = s0 - rec_l[CUT_FAST + lane];
            sumE[lane] = s0;
        }
        wave_lds_sync();
        open_line();
    }
    // the next line's record and list entry, fetched while this line is searched (vector loads: the
    // line transition then waits for no memory round trip)
    double pf_f0 = 0.0, pf_i0 = 0.0;
    int pf_q = 0;
    auto prefetch = [&](int mn) {
        if (mn < nls) {   // (wave-uniform)
            int iv = mn;
            asm volatile("" : "+v"(iv));   // (a per-lane index: vector loads, counted apart from LDS)
            const double* rn = rec_l + (size_t)iv * CUT_REC;
            pf_i0 = lane < 21 ? rn[CUT_FAST + lane] : 0.0;
            pf_f0 = rn[lane < CUT_FAST ? lane : 0];
            pf_q = mls[iv];
        }
    };
    prefetch(1);
#ifdef GFPL_CUTW_CLOCK   // (diagnostic build: shader-clock cycles per phase and counts in scr.dbg)
    uint64_t ck_eval = 0, ck_dec = 0, ck_walk = 0, ck_trans = 0, ck_exact = 0, n_rounds = 0, n_trans = 0;
    uint64_t ck0 = clock64();
#define CUTW_CK(acc) do { const uint64_t ck1 = clock64(); acc += ck1 - ck0; ck0 = ck1; } while (0)
#else
#define CUTW_CK(acc) do { } while (0)
#endif
    while (m < nls) {   // (wave-uniform)
        // ---- the 8 x 8 grid of ratios at offsets -1 .. 6 from the centre, as the moves accumulate
        //      them
        double g0[8], g1[8];
        g0[1] = r0;
        g1[1] = r1;
        g0[0] = r0 + (-st);
        g1[0] = r1 + (-st);
#pragma unroll
        for (int k = 2; k < 8; ++k) { g0[k] = g0[k - 1] + st; g1[k] = g1[k - 1] + st; }
        // an interior index k whose r - s is not the grid value below (k = 3 and 20 of 0, s, 2s, ... for
        // s = 0.05: 0.15 - 0.05 != 0.1): its positions' lower neighbours are evaluated apart (alt values);
        // the lowest such index per side is served, positions at any other one stop the walk
        int inc0 = 0, inc1 = 0;
#pragma unroll
        for (int k = 2; k <= 6; ++k) {
            inc0 |= (__double_as_longlong(g0[k] + (-st)) != __double_as_longlong(g0[k - 1])) ? (1 << k) : 0;
            inc1 |= (__double_as_longlong(g1[k] + (-st)) != __double_as_longlong(g1[k - 1])) ? (1 << k) : 0;
        }
        const int k0 = inc0 ? __builtin_ctz(inc0) : -1, k1 = inc1 ? __builtin_ctz(inc1) : -1;
        int dj_valid = 0, bok = 0;
        double dj = 0.0;
        double t0 = g0[0], t1 = g1[0];   // the lane's grid ratios
        CutReg cr;
        cut_reg_load(cmpl, cr);
        {
            const int a = lane >> 3, c = lane & 7;
#pragma unroll
            for (int k = 1; k < 8; ++k) { t0 = a == k ? g0[k] : t0; t1 = c == k ? g1[k] : t1; }
            int valid = 1;
            if (t0 + t1 > 1.0) valid = 0;
            if (t0 < rlo || t0 > rhi) valid = 0;
            if (t1 < rlo || t1 > rhi) valid = 0;
            dj_valid = valid;
            dj = cut_dval<false>(cr, t0, t1, tq, bok);
        }
        if (inc0 | inc1) {   // (wave-uniform) the alt values (h0, g1[c]) -> slot 82 + c, (g0[a], h1) -> 90 + a,
                             // (h0, h1) -> 98, each on a lane that already holds its grid ratio: row items on
                             // lanes 0-7 (a = 0: t1 = g1[c]), column items a >= 1 on lanes 8a + 7 (t0 = g0[a]),
                             // column item 0 on lane 8, the corner on lane 16
            const int a = lane >> 3, c = lane & 7;
            const int k0s = __builtin_amdgcn_readfirstlane(k0), k1s = __builtin_amdgcn_readfirstlane(k1);
            // h = g[k] - s at the served index (t0 of lane 8k is g0[k], t1 of lane k is g1[k])
            const double h0 = readlane_f64(t0, k0s > 0 ? 8 * k0s : 0) + (-st);
            const double h1 = readlane_f64(t1, k1s > 0 ? k1s : 0) + (-st);
            const bool row = lane < 8, col = lane == 8 || (c == 7 && a >= 1), cor = lane == 16;
            const double u0 = (row || cor) ? h0 : (lane == 8 ? g0[0] : t0);
            const double u1 = row ? t1 : h1;
            int valid = (row && k0s >= 0) || (col && k1s >= 0) || (cor && k0s >= 0 && k1s >= 0);
            if (u0 + u1 > 1.0) valid = 0;
            if (u0 < rlo || u0 > rhi) valid = 0;
            if (u1 < rlo || u1 > rhi) valid = 0;
            int abok = 0;
            const double da = cut_dval<false>(cr, u0, u1, tq, abok);
            if (row | col | cor) {
                const int slot = row ? 82 + lane : (cor ? 98 : 90 + (lane == 8 ? 0 : a));
                dgx[slot] = (valid && da == da) ? da : -__builtin_inf();
                dgf[slot] = abok | (valid << 1) | ((valid && !(da == da)) ? 4 : 0);
            }
        }
        CUTW_CK(ck_eval);
        // ---- every grid position's decision at once: lane (a, c), 1 <= a, c <= 6, gathers its 8
        //      neighbours' values (bpermute) and takes k_cut_search's group decision and margin tests
        //      (group_first_max, f1-f5) with its own value as the centre: a move j, CUT_P_STAY, or
        //      WAVE_EXACT / WAVE_STOP (a margin test failed / a neighbour's ratio bits are not the grid's)
        constexpr int WAVE_EXACT = 16, WAVE_STOP = 32;
        int dec = WAVE_STOP;
        {
            const int a = lane >> 3, c = lane & 7;
            // a position's neighbour ratios are the grid's (r + s is the value above by construction, r - s
            // the value below unless the index is inconsistent) or the alt values of the served index
            const int bad0 = inc0 & ~(k0 >= 0 ? 1 << k0 : 0), bad1 = inc1 & ~(k1 >= 0 ? 1 << k1 : 0);
            const bool cons = a >= 1 && a <= 6 && c >= 1 && c <= 6 && !((bad0 >> a) & 1) && !((bad1 >> c) & 1);
            const bool ia = a == k0, ic = c == k1;
            // the neighbours' values and flags through LDS (8 reads each; border lanes read padding)
            const double xo = (dj_valid && dj == dj) ? dj : -__builtin_inf();
            dgx[9 + lane] = xo;
            dgf[9 + lane] = bok | (dj_valid << 1) | ((dj_valid && !(dj == dj)) ? 4 : 0);
            wave_lds_sync();
            double vjn[8];
            int fl[8];
            if (inc0 | inc1) {   // (wave-uniform) some lower neighbours are alt values
#pragma unroll
                for (int jn = 0; jn < 8; ++jn) {
                    const int da = nb_da(jn, 0), dc = nb_da(jn, 1);
                    const bool xa = ia && da < 0, xc = ic && dc < 0;
                    const int l = (xa && xc) ? 82 + 16 : (xa ? 82 + c + dc : (xc ? 90 + a + da : 9 + lane + 8 * da + dc));
                    vjn[jn] = dgx[l];
                    fl[jn] = dgf[l];
                }
            } else {   // every neighbour on the grid: constant offsets from the lane's slot
#pragma unroll
                for (int jn = 0; jn < 8; ++jn) {
                    const int l = 9 + lane + 8 * nb_da(jn, 0) + nb_da(jn, 1);
                    vjn[jn] = dgx[l];
                    fl[jn] = dgf[l];
                }
            }
            const double dcl = dj;
            const int cok = bok;
            // the first strict maximum (group_first_max's rule): a tree maximum, then the lowest index at it
            const double m01 = fmax(vjn[0], vjn[1]), m23 = fmax(vjn[2], vjn[3]);
            const double m45 = fmax(vjn[4], vjn[5]), m67 = fmax(vjn[6], vjn[7]);
            const double mx = fmax(fmax(m01, m23), fmax(m45, m67));
            int atm = 0;
#pragma unroll
            for (int jn = 0; jn < 8; ++jn) atm |= (vjn[jn] == mx) ? (1 << jn) : 0;
            const int kf = (mx > -__builtin_inf()) ? __builtin_ctz(atm | 256) : 8;
            const int best = (kf < 8 && mx > dcl) ? kf : -1;
            const double top = mx;
            const bool has = best >= 0;
            const double ttop = tau * top, tdc = tau * dcl;
            // (bitwise, not short-circuit: every flag read is issued at once instead of one LDS round trip per
            // neighbour behind a branch)
            int fail = (int)(has & !(top - dcl > ttop)) | (int)!((tau > 0.0) & (line_ok != 0) & (cok != 0) & (dcl == dcl));
#pragma unroll
            for (int jn = 0; jn < 8; ++jn) {
                const double v = vjn[jn];
                const int f = fl[jn];
                const int vl = (f >> 1) & 1;
                const int f1 = vl & ~f & 1;
                const int f2 = (int)has & vl & (int)(jn != best) & (int)!(top - v > ttop);
                const int f4 = (int)!has & vl & (int)!(dcl - v > tdc);
                const int f3 = (f >> 2) & 1;   // (a valid NaN: the raw value fails f2 / f4 in the group search)
                fail |= f1 | f2 | f3 | f4;
            }
            const bool ok = fail == 0;
            // a move below a served index leaves the grid, and the exact round reads the grid's neighbours:
            // both stop the walk (the next round, centred there, has them on its grid)
            const bool off = has && ((ia && nb_da(best, 0) < 0) || (ic && nb_da(best, 1) < 0));
            dec = !cons ? WAVE_STOP : (!ok ? ((ia || ic) ? WAVE_STOP : WAVE_EXACT) : (off ? WAVE_STOP : (has ? best : CUT_P_STAY)));
            // the walk's word: the decision, whether the move ends the line (r0 + r1 > 1 after it: the moved
            // ratios are the neighbour's grid values, bit for bit, at a consistent position) and the lane moved to
            const int mv = has ? best : 0;
            const double n0 = t0 + nb_step(mv, 0, st), n1 = t1 + nb_step(mv, 1, st);
            const int fin = (has && !(n0 + n1 <= 1.0)) ? 64 : 0;
            dec |= fin | ((lane + 8 * nb_da(mv, 0) + nb_da(mv, 1)) & 63) << 8;
        }
        CUTW_CK(ck_dec);
        // ---- follow the decisions from the centre while they stay inside the grid
        int pos = 9;   // (a, c) = (1, 1): the centre
        int exact = 0, finalize = 0;
        double vj[8];
        int bj[8], valj[8];
        int pathv = 0, ns = 0;
        if (!rec) {
            // measured mode: the walk by pointer jumping (no record needed).  A position whose decision
            // is a move that does not end the line continues at its target; every other position ends
            // a chain.  Moves go to strictly larger d, so the chains are acyclic; six doublings cover
            // the 64 positions.  Then lane 9's chain end and step count decide the round.
            const int dpos = dec & 63;
            const bool cont = dpos < CUT_P_STAY && !(dec & 64);
            int jump = cont ? (dec >> 8) & 63 : lane;
            int acc = cont ? 1 : 0;
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                const int jj = __shfl(jump, jump);
                const int aa = __shfl(acc, jump);
                acc += aa;
                jump = jj;
            }
            const int T = __builtin_amdgcn_readlane(jump, 9);
            ns = __builtin_amdgcn_readlane(acc, 9);
            const int wT = __builtin_amdgcn_readlane(dec, T);
            const int dT = wT & 63;
            pos = T;
            if (dT >= WAVE_EXACT) {
                exact = dT == WAVE_EXACT;
            } else {
                ++ns;
                finalize = 1;
                if (dT != CUT_P_STAY) pos = wT >> 8;   // (a move that ends the line: r0 + r1 > 1 after it)
            }
        } else {
            // scalar walk: one readlane per step, the step's record byte parked in lane ns of pathv (one
            // vector store after the walk, no per-step exec-masked store)
            for (int sstep = 0; sstep < 64; ++sstep) {   // (wave-uniform; the grid ends a path: its edge positions stop)
                const int w = __builtin_amdgcn_readlane(dec, pos);
                const int dpos = w & 63;
                if (dpos >= WAVE_EXACT) {   // WAVE_STOP / WAVE_EXACT
                    exact = dpos == WAVE_EXACT;
                    break;
                }
                pathv = lane == ns ? dpos : pathv;
                ++ns;
                if (dpos == CUT_P_STAY) { finalize = 1; break; }
                pos = w >> 8;
                if (w & 64) { finalize = 1; break; }
            }
        }
        if (ns) {
            if (rec && lane < ns && lstep + lane < CUT_PATH) path[(size_t)m * CUT_PATH + lstep + lane] = (uint8_t)pathv;
            n_steps += ns;
            lstep += ns;
            first = 0;
        }
        if (exact) {   // the exact round needs the position's neighbours
            const int pa = pos >> 3, pc = pos & 7;
#pragma unroll
            for (int jn = 0; jn < 8; ++jn) {
                const int l = (pa + nb_da(jn, 0)) * 8 + (pc + nb_da(jn, 1));
                vj[jn] = readlane_f64(dj, l);
                bj[jn] = __builtin_amdgcn_readlane(bok, l);
                valj[jn] = __builtin_amdgcn_readlane(dj_valid, l);
            }
        }
        // the ratios where the walk stopped: that lane's grid values (r + s accumulated, bit for bit)
        r0 = readlane_f64(t0, pos);
        r1 = readlane_f64(t1, pos);
        CUTW_CK(ck_walk);
#ifdef GFPL_CUTW_CLOCK
        ++n_rounds;
#endif
        if (exact) {
            // the reference's evaluation of this step (group 0 = lanes 0-7; the flush uses the wave);
            // the neighbours' values were gathered by the step that stopped
            int myv = 0;
#pragma unroll
            for (int jn = 0; jn < 8; ++jn) myv = lane == jn ? valj[jn] : myv;
            const CutX xr = cut_exact_round(lane < 8, myv, first, m, m_sync, r0, r1, q_cur, lb, -1, mls, rec_l, L.sP,
                                            L.eP, L.covS, L.covE, L.le_obs, L.cut, sumE, tmp[0], &tmp[0][0], Dl,
                                            cam.fx, cam.b, homog, st);
            const int best = __builtin_amdgcn_readfirstlane(xr.best);
            m_sync = __builtin_amdgcn_readfirstlane(xr.m_sync);
            ++n_steps;
            ++n_exact;
            if (rec && lane == 0) {
                if (lstep < CUT_PATH)
                    path[(size_t)m * CUT_PATH + lstep] = (uint8_t)((best >= 0 ? best : CUT_P_STAY) | CUT_P_EXACT);
            }
            ++lstep;
            first = 0;
            if (best < 0) {
                finalize = 1;
            } else {
                double vb = vj[0];
                int bb = bj[0];
#pragma unroll
                for (int jn = 1; jn < 8; ++jn) { vb = best == jn ? vj[jn] : vb; bb = best == jn ? bj[jn] : bb; }
                dc = vb;
                c_ok = bb;
                r0 = r0 + nb_step(best, 0, st);
                r1 = r1 + nb_step(best, 1, st);
                if (!(r0 + r1 <= 1.0)) finalize = 1;
            }
        }
        CUTW_CK(ck_exact);
        if (finalize) {
#ifdef GFPL_CUTW_CLOCK
            ++n_trans;
#endif
#ifdef GFPL_CUTW_TCLOCK
            tk0 = clock64();
#endif
            if (lane == 0) {
                L.cut[2 * q_cur] = r0;
                L.cut[2 * q_cur + 1] = r1;
            }
            // the approximate invCov_sum += the finished line's info (k_cut_search's transition): lane
            // e < 21 forms its entry from the comparison data directly (cut_ours_* expressions, the bits of
            // cut_ours_info over the [v'_s, P_s, v'_e, P_e] vector), or from the reference-order endpoints
            double info = 0.0;
            {
                const int ra = (int)((TRI_ROW >> (3 * lane)) & 7), cb = (int)((TRI_COL >> (3 * lane)) & 7);
                if (fst[PD_OK] != 0.0) {   // (wave-uniform)
                    if (lane < 21) {
                        const double is = rcp_fast(cut_ours_V(fst, 0, r0)), ie = rcp_fast(cut_ours_V(fst, 1, r1));
                        const double psr = cut_ours_P(fst, 0, ra, r0), psc = cut_ours_P(fst, 0, cb, r0);
                        const double per = cut_ours_P(fst, 1, ra, r1), pec = cut_ours_P(fst, 1, cb, r1);
                        info = __builtin_fma(psr * is, psc, (per * ie) * pec);
                    }
                } else {
                    if (lane < 2) {
                        double o7[7];
                        exact_endpoint(cam, homog, Dl, L, q_cur, lane, lane ? r1 : r0, o7);
#pragma unroll
                        for (int i = 0; i < 7; ++i) xsl[7 * lane + i] = o7[i];
                    }
                    wave_lds_sync();
                    if (lane < 21) info = cut_ours_info(xsl, rcp_fast(xsl[0]), rcp_fast(xsl[7]), ra, cb);
                }
            }
            ++m;
            TCK(0);
            if (m < nls) {
                wave_lds_sync();
                if (lane < CUT_FAST) fst[lane] = pf_f0;
                if (lane < 21) sumA[lane] = (sumA[lane] + info) - pf_i0;
                q_cur = lb + __builtin_amdgcn_readfirstlane(pf_q);
                first = 1;
                lstep = 0;
                r0 = 0.0;
                r1 = 0.0;
                wave_lds_sync();
                TCK(1);
                open_line();
                prefetch(m + 1);
            }
        }
        CUTW_CK(ck_trans);
    }
    if (lane == 0) {
        p.scr.bytes[(size_t)STEP_REC * b + 16] = n_steps;
        p.scr.bytes[(size_t)STEP_REC * b + 17] = n_exact;
        p.scr.bytes[(size_t)STEP_REC * b + 19] = 0;
#ifdef GFPL_CUTW_CLOCK
        int64_t* d = p.scr.dbg + 8 * (size_t)b;
        d[0] = ck_eval; d[1] = ck_dec; d[2] = ck_walk; d[3] = ck_exact; d[4] = ck_trans; d[5] = n_rounds; d[6] = n_trans;
        d[7] = n_steps;
#endif
#ifdef GFPL_CUTW_TCLOCK
        for (int i = 0; i < 7; ++i) p.scr.dbg[8 * (size_t)b + i] = (int64_t)tk[i];
#endif
    }
}

// ---------------------------------------------------------------- finish --
// invCovPose of the chosen ratio + updateEndPointByRatio (ledger Q4)
#ifndef GFPL_FIN_WAVES
#define GFPL_FIN_WAVES 4   // waves per SIMD: <= 128 VGPRs (0.855 -> 0.842 ms, profiles/r05_bp)
#endif
__global__ void __launch_bounds__(64, GFPL_FIN_WAVES) k_cut_finish(KParams p) {
    const int b = blockIdx.x;
    const int nls = p.tr.n_matched_ls[b];
    // proven mode (cut_proof 1 / 3): k_cut_verify wrote the proven sequences' invCovPose, this kernel their
    // cut endpoints; the redone ones get both here
    if (nls == 0) return;
    const bool ends_only = (p.cfg.cut_proof == 1 || p.cfg.cut_proof == 3) && p.scr.cut_flag[b] == 0;
    const DevCam& cam = p.cam;
    DevLines& L = p.prev.ls;
    const size_t lb = (size_t)b * p.kl_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    double Dl[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) Dl[i] = p.scr.cut_dtinv[16 * b + i];
    for (int m0 = 0; m0 < nls; m0 += 64) {   // (wave-uniform)
        const int m = m0 + (int)threadIdx.x;
        const bool live = m < nls;
        const size_t q = lb + (live ? mls[m] : 0);
        LineCutData d;
        double r0 = 0.0, r1 = 0.0;
        double info[36];
        if (live && ends_only) {
            load_line(L, q, d);
            r0 = L.cut[2 * q];
            r1 = L.cut[2 * q + 1];
        } else if (live) {
            load_line(L, q, d);
            r0 = L.cut[2 * q];
            r1 = L.cut[2 * q + 1];
            poseInfoOnLine<true>(cam, p.cfg.homog_th, Dl, d, r0, r1, info);
            // 16-B stores: a line's 36 doubles are contiguous and 288-B aligned (carve: 256-B field base)
            // (staged through LDS like k_cut_prep's records they measured 1.01 vs 0.82 ms: the lines of
            // a chunk are scattered over the frame, so the slices do not merge; profiles/r04_u)
            double2* iv = reinterpret_cast<double2*>(L.invcov + 36 * q);
#pragma unroll
            for (int i = 0; i < 18; ++i) iv[i] = make_double2(info[2 * i], info[2 * i + 1]);
        }
        if (live && !(fabs(r0) < 0.0001 && fabs(r1) < 0.0001)) {
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

// ---------------------------------------------------------------- verify --
// Proven mode (cut_proof 1): the measured search (k_cut_search<false>) decided every margined step on
// our comparison operands and recorded its decisions (cut_path); this kernel proves, after the fact,
// that each of those decisions is the reference's, with the agreement bound of DESIGN.md §3 — now
// evaluated with the operands' *actual* differences instead of eager reference operands in the search:
//   * v' (Lemma 2): at every ratio the recorded steps compared, the reference's own endpoint variance
//     (ref_vprime: cut_endpoint_t<double>'s expression tree, scaled by its fgz2) against the quartic the
//     search used, r_v(t) = |v'_ours - v'_ref| / v'_ref plus the scaling's bound (RB, cut_line_bounds);
//   * S (Lemma 3): the search's running invCov_sum (replayed bit for bit in list order: r = 0 infos of
//     k_cut_prep, the search's own info of each finished line — cut_ours_*) against the reference's (the
//     same list order with the reference-order info of each line at its final ratios), their difference
//     whitened by diag(S^-1): eps_S = sum_ik |dS_ik| sqrt(s_i s_k) + our factor's backward error;
//   * P (Lemma 2): the RB error bounds of our polynomial coefficients and of the reference's Jacobian.
// Per line: E = K0 + A1 max(1/v's) + 4.12 bs^2 max(r_v,s / v's) + (end side) <= R0 = tau/8 - 1.01 K0,
// with every maximum over the ratios of the line's margined steps (each step's comparisons then have
// gaps > tau in d, > tau/2 in exact arithmetic (forward bound), > tau/4 between the reference's metrics).
// Steps the search decided exactly need nothing.  A sequence with any line not proven (or a path that
// does not replay to the search's final ratios) is flagged; the eager-proven search then redoes its line
// cut (k_cut_bounds, k_cut_vtab, k_cut_search<true>, k_cut_finish, gated by the flag).  This kernel is
// also k_cut_finish for the proven sequences: invCovPose of every line (written for all; a redone
// sequence overwrites it) and, once the whole sequence is proven, the cut endpoints.
// One wave per sequence; lines in chunks of 64, one per lane.
__device__ __forceinline__ double verify_vref(const KParams& p, const double* Dl, size_t q, int side, double t) {
    return ref_vprime(p.cam, p.cfg.homog_th, Dl, p.prev.ls, q, side, t);
}

// Proven mode, first verification pass: one lane per matched line of every sequence (no serial
// dependence between lines here).  The line's recorded steps are replayed and, at every ratio a
// margined step compared, the reference's own scaled endpoint variance v'_ref (ref_vprime, from
// the line's data held in registers) is set against the quartic v'_ours the search used:
// per side, max 1.01 / min(v'_ours, v'_ref) and max r_v / min(...) with r_v = |v'_ours - v'_ref| / v'_ref.
// k_cut_verify combines these maxima with the line's S-dependent bound terms.
__device__ __forceinline__ double vref_regs(const DevCam& cam, double homog, const double* Dl, const double* P0,
                                            const double* P1, const double* C0, const double* C1, const double* Jl,
                                            double c) {
    double Pt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) Pt[k] = (1.0 - c) * P0[k] + c * P1[k];
    const double a = (1.0 - c) * (1.0 - c), qq = c * c;
    double cov[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) cov[i] = a * C0[i] + qq * C1[i];
    const double v = endpointVar_t<double, true>(cam, Dl, Jl, Pt, cov, 0.0);
    double cur[3];
    se3_apply(Dl, Pt, cur);
    const double f = cam.fx / ref_max(homog, cur[2] * cur[2]);
    return v / (f * f);
}

// The line's replay with a small cache of evaluated ratios per side: the fallback of k_cut_vref for a
// line whose compared ratios leave the key table (a ratio moved back: rare), one lane.
__device__ __forceinline__ void vref_replay(const KParams& p, int b, int m) {
    const double* fd = p.scr.cut_rec + ((size_t)b * p.mls_cap + m) * CUT_REC;
    double* out = p.scr.cut_vmax + ((size_t)b * p.mls_cap + m) * CUT_VMAX;
    const uint8_t* path = p.scr.cut_path + ((size_t)b * p.mls_cap + m) * CUT_PATH;
    const DevLines& L = p.prev.ls;
    const size_t q = (size_t)b * p.kl_cap + p.tr.matched_ls[(size_t)b * p.mls_cap + m];
    const double* Dl = p.scr.cut_dtinv + 16 * (size_t)b;
    const double st = p.cfg.cut_step, rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    double sP[3], eP[3], cS[9], cE[9], Jl[2], qs[5], qe[5];
#pragma unroll
    for (int k = 0; k < 3; ++k) { sP[k] = L.sP[3 * q + k]; eP[k] = L.eP[3 * q + k]; }
#pragma unroll
    for (int k = 0; k < 9; ++k) { cS[k] = L.covS[9 * q + k]; cE[k] = L.covE[9 * q + k]; }
    Jl[0] = L.le_obs[3 * q];
    Jl[1] = L.le_obs[3 * q + 1];
#pragma unroll
    for (int k = 0; k < 5; ++k) { qs[k] = fd[PD_VS + k]; qe[k] = fd[PD_VE + k]; }
    double r0 = 0.0, r1 = 0.0;
    bool done = false;
    // the reference's v' at the last four ratios evaluated per side (t bits, value), in registers:
    // a ratio step moves the window by one, so a step evaluates at most one new ratio per side
    long long ct0[4] = {-1, -1, -1, -1}, ct1[4] = {-1, -1, -1, -1};
    double cv0[4] = {0, 0, 0, 0}, cv1[4] = {0, 0, 0, 0};
    int slot0 = 0, slot1 = 0;
    double ivm[2] = {0.0, 0.0}, rim[2] = {0.0, 0.0};
    int marg = 0, nbad = 0, nev = 0;
    for (int k = 0; k < CUT_PATH && !done; ++k) {
        const int by = path[k];
        if (!(by & CUT_P_EXACT)) {
            ++marg;
            for (int w = 0; w < 6; ++w) {
                const int side = w >= 3 ? 1 : 0, o = w - 3 * side;
                const double rc = side ? r1 : r0;
                const double t = o == 0 ? rc + (-st) : (o == 2 ? rc + st : rc);   // (nb_step's bits)
                if (!(t >= rlo && t <= rhi)) continue;
                const long long tb = __double_as_longlong(t);
                double vr = 0.0;
                bool hit = false;
#pragma unroll
                for (int z = 0; z < 4; ++z) {
                    const bool h = side ? ct1[z] == tb : ct0[z] == tb;
                    vr = h ? (side ? cv1[z] : cv0[z]) : vr;
                    hit = hit || h;
                }
                if (!hit) {
                    vr = side ? vref_regs(p.cam, p.cfg.homog_th, Dl, eP, sP, cE, cS, Jl, t)
                              : vref_regs(p.cam, p.cfg.homog_th, Dl, sP, eP, cS, cE, Jl, t);
                    ++nev;
#pragma unroll
                    for (int z = 0; z < 4; ++z) {
                        if (side && slot1 == z) { ct1[z] = tb; cv1[z] = vr; }
                        if (!side && slot0 == z) { ct0[z] = tb; cv0[z] = vr; }
                    }
                    if (side) slot1 = (slot1 + 1) & 3; else slot0 = (slot0 + 1) & 3;
                }
                const double* qc = side ? qe : qs;
                const double vo = __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, qc[4], qc[3]), qc[2]),
                                                                 qc[1]), qc[0]);   // (cut_ours_V's expression)
                const double lo = fmin(vr, vo);
                const double rv = fabs(vo - vr) / vr;
                if (!(lo > 0.0 && rv < 0.01)) { ++nbad; continue; }
                const double iv = 1.01 / lo;
                ivm[side] = fmax(ivm[side], iv);
                rim[side] = fmax(rim[side], rv * iv);
            }
        }
        if (by & CUT_P_STAY) {
            done = true;
        } else {
            const int jj = by & 7;
            r0 = r0 + nb_step(jj, 0, st);
            r1 = r1 + nb_step(jj, 1, st);
            if (!(r0 + r1 <= 1.0)) done = true;
        }
    }
    // a path that does not end where the search's final ratios are counts as a failure
    if (!done || __double_as_longlong(r0) != __double_as_longlong(L.cut[2 * q]) ||
        __double_as_longlong(r1) != __double_as_longlong(L.cut[2 * q + 1]))
        nbad += 1 << 20;
    out[0] = ivm[0];
    out[1] = rim[0];
    out[2] = ivm[1];
    out[3] = rim[1];
    out[4] = (double)marg + 1024.0 * (double)nev;   // (marg <= CUT_PATH)
    out[5] = (double)nbad;
}


// Lines in chunks of 64 (one wave), in two passes.  (A) lane per line: the recorded steps replayed on
// the ratio-key links (cut_knxt / cut_kprv, the bits of r + s and r - s), marking per side every key a
// margined step compared; (B) the marked (line, side, key) items, compacted in LDS, evaluated by the
// whole wave (consecutive items share a line: its data loads broadcast), the per-side maxima by LDS
// atomics.  A line whose compared ratios leave the table takes vref_replay.
__global__ void __launch_bounds__(64) k_cut_vref(KParams p) {
    __shared__ double keys[CUT_KS];
    __shared__ int8_t knx[CUT_KS], kpv[CUT_KS];
    __shared__ uint16_t items[64 * 2 * CUT_KS];
    __shared__ unsigned long long red[4][64];   // ivm0, rim0, ivm1, rim1 (non-negative doubles' bits)
    __shared__ int nbl[64];
    __shared__ int qln[64];   // each line's index in the prev frame (pass B reads it here: no dependent
                              // global load ahead of the line's data loads)
    const int b = blockIdx.y;
    const int lane = threadIdx.x;
    const int m = blockIdx.x * 64 + lane;
    const int nls = p.tr.n_matched_ls[b];
    if (blockIdx.x * 64 >= nls) return;   // (wave-uniform)
    const int nk = p.cut_nkeys;
    if (lane < CUT_KS) {
        keys[lane] = p.cut_keys[lane];
        knx[lane] = p.cut_knxt[lane];
        kpv[lane] = p.cut_kprv[lane];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[i][lane] = 0ull;
    nbl[lane] = 0;
    wave_lds_sync();
    const bool on = m < nls;
    const double st = p.cfg.cut_step, rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    // (A) replay on the key links
    uint32_t mk[2] = {0u, 0u};
    int marg = 0, nbad = 0;
    bool off = nk == 0;
    if (on && !off) {
        // the line's 64 path bytes in one go (16-byte loads), not a memory round trip per step
        const uint4* pv = reinterpret_cast<const uint4*>(p.scr.cut_path + ((size_t)b * p.mls_cap + m) * CUT_PATH);
        uint32_t pw[CUT_PATH / 4];
#pragma unroll
        for (int i = 0; i < CUT_PATH / 16; ++i) {
            const uint4 v = pv[i];
            pw[4 * i] = v.x; pw[4 * i + 1] = v.y; pw[4 * i + 2] = v.z; pw[4 * i + 3] = v.w;
        }
        double r[2] = {0.0, 0.0};
        int kc[2] = {0, 0};   // (keys[0] is 0.0)
        bool done = false;
        for (int k = 0; k < CUT_PATH && !done && !off; ++k) {
            uint32_t wd = pw[0];
#pragma unroll
            for (int i = 1; i < CUT_PATH / 4; ++i) wd = (k >> 2) == i ? pw[i] : wd;
            const int by = (int)((wd >> (8 * (k & 3))) & 255u);
            if (!(by & CUT_P_EXACT)) {
                ++marg;
#pragma unroll
                for (int side = 0; side < 2; ++side) {
#pragma unroll
                    for (int o = 0; o < 3; ++o) {
                        const double t = o == 0 ? r[side] + (-st) : (o == 2 ? r[side] + st : r[side]);
                        if (!(t >= rlo && t <= rhi)) continue;
                        const int kk = kc[side] < 0 ? -1 : (o == 0 ? kpv[kc[side]] : (o == 2 ? knx[kc[side]] : kc[side]));
                        if (kk < 0 || __double_as_longlong(keys[kk]) != __double_as_longlong(t)) { off = true; continue; }
                        mk[side] |= 1u << kk;
                    }
                }
            }
            if (by & CUT_P_STAY) {
                done = true;
            } else {
                const int jj = by & 7;
#pragma unroll
                for (int side = 0; side < 2; ++side) {
                    const double sv = nb_step(jj, side, st);
                    r[side] = r[side] + sv;
                    if (kc[side] >= 0) kc[side] = sv > 0.0 ? knx[kc[side]] : (sv < 0.0 ? kpv[kc[side]] : kc[side]);
                }
                if (!(r[0] + r[1] <= 1.0)) done = true;
            }
        }
        const int qi = p.tr.matched_ls[(size_t)b * p.mls_cap + m];
        qln[lane] = qi;
        const size_t q = (size_t)b * p.kl_cap + qi;
        // a path that does not end where the search's final ratios are counts as a failure
        if (!done || __double_as_longlong(r[0]) != __double_as_longlong(p.prev.ls.cut[2 * q]) ||
            __double_as_longlong(r[1]) != __double_as_longlong(p.prev.ls.cut[2 * q + 1]))
            nbad += 1 << 20;
    }
    if (off) mk[0] = mk[1] = 0u;
    // compaction: the lane's items at its exclusive prefix of the counts
    const int cnt = __popc(mk[0]) + __popc(mk[1]);
    int inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o);
        if (lane >= o) inc += v;
    }
    const int total = __shfl(inc, 63);
    {
        int w = inc - cnt;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            uint32_t x = mk[side];
            while (x) {
                const int kk = __ffs(x) - 1;
                x &= x - 1u;
                items[w++] = (uint16_t)((lane << 6) | (side << 5) | kk);
            }
        }
    }
    wave_lds_sync();
    // (B) the items, one per lane per round
    const DevLines& L = p.prev.ls;
    const double* Dl = p.scr.cut_dtinv + 16 * (size_t)b;
    for (int i0 = 0; i0 < total; i0 += 64) {   // (wave-uniform)
        const int i = i0 + lane;
        if (i < total) {
            const int it = items[i];
            const int ln = it >> 6, side = (it >> 5) & 1, kk = it & 31;
            const int mm = blockIdx.x * 64 + ln;
            const size_t q = (size_t)b * p.kl_cap + qln[ln];
            const double* fd = p.scr.cut_rec + ((size_t)b * p.mls_cap + mm) * CUT_REC;
            double P0[3], P1[3], C0[9], C1[9], Jl[2], qc[5];
            const double* A3 = side ? L.eP : L.sP;
            const double* B3 = side ? L.sP : L.eP;
            const double* A9 = side ? L.covE : L.covS;
            const double* B9 = side ? L.covS : L.covE;
#pragma unroll
            for (int k = 0; k < 3; ++k) { P0[k] = A3[3 * q + k]; P1[k] = B3[3 * q + k]; }
#pragma unroll
            for (int k = 0; k < 9; ++k) { C0[k] = A9[9 * q + k]; C1[k] = B9[9 * q + k]; }
            Jl[0] = L.le_obs[3 * q];
            Jl[1] = L.le_obs[3 * q + 1];
#pragma unroll
            for (int k = 0; k < 5; ++k) qc[k] = fd[(side ? PD_VE : PD_VS) + k];
            const double t = keys[kk];
            const double vr = vref_regs(p.cam, p.cfg.homog_th, Dl, P0, P1, C0, C1, Jl, t);
            const double vo = __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, __builtin_fma(t, qc[4], qc[3]), qc[2]),
                                                             qc[1]), qc[0]);   // (cut_ours_V's expression)
            const double lo = fmin(vr, vo);
            const double rv = fabs(vo - vr) / vr;
            if (!(lo > 0.0 && rv < 0.01)) {
                atomicAdd(&nbl[ln], 1);
            } else {
                const double iv = 1.01 / lo;
                atomicMax(&red[2 * side][ln], (unsigned long long)__double_as_longlong(iv));
                atomicMax(&red[2 * side + 1][ln], (unsigned long long)__double_as_longlong(rv * iv));
            }
        }
    }
    wave_lds_sync();
    if (!on) return;
    double* out = p.scr.cut_vmax + ((size_t)b * p.mls_cap + m) * CUT_VMAX;
    if (off) {   // (k_cut_vref_off replays the line: appended to its list)
        const int slot = atomicAdd(p.scr.cut_offl, 1);
        p.scr.cut_offl[1 + slot] = b * p.mls_cap + m;
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = __longlong_as_double((long long)red[i][lane]);
    out[4] = (double)marg + 1024.0 * (double)cnt;   // (marg <= CUT_PATH)
    out[5] = (double)(nbad + nbl[lane]);
}

// the lines k_cut_vref left (a compared ratio off the key table: rare), from its list, one lane each;
// its own kernel, so that the replay's registers do not set k_cut_vref's occupancy, over a fixed grid
__global__ void __launch_bounds__(64) k_cut_vref_off(KParams p) {
    const int n = p.scr.cut_offl[0];
    for (int i = blockIdx.x * 64 + threadIdx.x; i < n; i += gridDim.x * 64) {
        const int e = p.scr.cut_offl[1 + i];
        vref_replay(p, e / p.mls_cap, e % p.mls_cap);
    }
}

// Proven mode: the operand error bounds of every matched line (cut_line_bounds_p, P only) into
// cut_vmax[6..13] as 14 floats, one lane per line — no dependence between lines, so out of
// k_cut_verify's serial sequence pass (and its register budget)
__global__ void __launch_bounds__(64) k_cut_ebound(KParams p) {
    const int b = blockIdx.y;
    const int m = blockIdx.x * 64 + threadIdx.x;
    if (m >= p.tr.n_matched_ls[b]) return;
    const double* fd = p.scr.cut_rec + ((size_t)b * p.mls_cap + m) * CUT_REC;
    if (fd[PD_OK] == 0.0) return;
    const size_t q = (size_t)b * p.kl_cap + p.tr.matched_ls[(size_t)b * p.mls_cap + m];
    double Dl[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) Dl[i] = p.scr.cut_dtinv[16 * b + i];
    float eb[14];
    cut_line_bounds_p(p, q, true, Dl, eb);
    float* o = reinterpret_cast<float*>(p.scr.cut_vmax + ((size_t)b * p.mls_cap + m) * CUT_VMAX + 6);
#pragma unroll
    for (int i = 0; i < 14; ++i) o[i] = eb[i];
}

// A recorded step the bound does not cover, checked with the reference's own arithmetic: its 6
// endpoint slots (reference order), every valid neighbour's logdet(S_ref + info) and the centre
// metric (logdet(invCov_sum) on a line's first step), the reference's first strict maximum against
// the recorded decision.  Out of line: rare, and its two 6x6 LLTs per neighbour would set the
// register budget of the replay.  Returns 1 when the decisions agree.
__device__ __attribute__((noinline)) int verify_exact_step(const KParams& p, const double* Dl, size_t q, double r0,
                                                           double r1, int first, const double* Sref, const double* Sfull,
                                                           int recorded) {
    const double st = p.cfg.cut_step, rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    double ep[6][7];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int side = j < 3 ? 0 : 1;
        const double eoff = (j % 3) == 0 ? -st : ((j % 3) == 2 ? st : 0.0);
        exact_endpoint(p.cam, p.cfg.homog_th, Dl, p.prev.ls, q, side, (side == 0 ? r0 : r1) + eoff, ep[j]);
    }
    double tot[21], tmp[21];
    double mc;
    if (first) {
#pragma unroll
        for (int i = 0; i < 21; ++i) tot[i] = Sfull[i];
    } else {
        cut_assemble<false>(ep[1], ep[4], tmp);
#pragma unroll
        for (int i = 0; i < 21; ++i) tot[i] = tmp[i] + Sref[i];
    }
    mc = logdet6_lower(tot);
    double mx = -__builtin_inf();
    int best = -1;
    for (int jn = 0; jn < 8; ++jn) {
        const double t0 = r0 + nb_step(jn, 0, st), t1 = r1 + nb_step(jn, 1, st);
        if (t0 + t1 > 1.0 || t0 < rlo || t0 > rhi || t1 < rlo || t1 > rhi) continue;
        cut_assemble<false>(ep[nb_slot(jn, 0)], ep[3 + nb_slot(jn, 1)], tmp);
#pragma unroll
        for (int i = 0; i < 21; ++i) tot[i] = tmp[i] + Sref[i];
        const double v = logdet6_lower(tot);
        if (v == v && v > mx) { mx = v; best = jn; }   // the first strict maximum (ties: lowest j)
    }
    const int ref = (best >= 0 && mx > mc) ? best : CUT_P_STAY;
    return ref == recorded ? 1 : 0;
}

// k_cut_verify's step-by-step replay of one line the line-level bound did not cover (rare): per margined
// step the reference's v' at the step's ratios and the step's own bound, a step no bound covers
// re-decided by the reference's arithmetic (verify_exact_step).  Sfull: the LDS column of the
// reference's whole invCov_sum at the line's start (stride 65).  Returns a reason mask.
__device__ __attribute__((noinline)) int verify_line_detail(const KParams& p, const double* Dl, size_t q,
                                                            const uint8_t* path_m, const double* fd, double r0f,
                                                            double r1f, double K0, double A1, double B1, double cs,
                                                            double ce, double R0, double rts, double rte, bool line_ok,
                                                            const double* Scol, int sstride, int& n_xchk) {
    const double st = p.cfg.cut_step, rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    const bool pdok = fd[PD_OK] != 0.0;
    int bad = 0;
    {
            double r0 = 0.0, r1 = 0.0;
            bool done = false;
            int first = 1;
            // the reference's v' at the last ratios evaluated, per side (t bits, value); the quartic is
            // re-evaluated (four FMAs)
            double ct[2][4], cv[2][4];
            int cn[2] = {0, 0};
            for (int k = 0; k < CUT_PATH && !done; ++k) {
                const int by = path_m[k];
                if (!(by & CUT_P_EXACT)) {
                    // (a margined step)
                    double ivm[2] = {0.0, 0.0}, rim[2] = {0.0, 0.0};
                    bool vok = pdok;
                    for (int w = 0; w < 6 && vok; ++w) {
                        const int side = w / 3, o = w % 3;
                        const double rc = side ? r1 : r0;
                        const double t = o == 0 ? rc + (-st) : (o == 2 ? rc + st : rc);   // (nb_step's bits)
                        if (!(t >= rlo && t <= rhi)) continue;
                        double vr = 0.0;
                        bool hit = false;
                        for (int z = 0; z < cn[side]; ++z)
                            if (__double_as_longlong(ct[side][z]) == __double_as_longlong(t)) { vr = cv[side][z]; hit = true; }
                        if (!hit) {
                            vr = verify_vref(p, Dl, q, side, t);
                            const int z = cn[side] < 4 ? cn[side]++ : (k & 3);
                            ct[side][z] = t;
                            cv[side][z] = vr;
                        }
                        const double vo = cut_ours_V(fd, side, t);
                        const double lo = fmin(vr, vo);
                        const double rv = fabs(vo - vr) / vr;
                        if (!(lo > 0.0 && rv < 0.01)) { vok = false; continue; }
                        const double iv = 1.01 / lo;
                        ivm[side] = fmax(ivm[side], iv);
                        rim[side] = fmax(rim[side], (1.01 * rv + (side ? rte : rts)) * iv);
                    }
                    const double E = K0 + A1 * ivm[0] + cs * rim[0] + B1 * ivm[1] + ce * rim[1];
                    if (!(vok && line_ok && E * 1.0001 <= R0)) {
                        // not covered by the bound: the reference's own evaluation of the step
                        double Sref[21], Sfull[21];
#pragma unroll
                        for (int e = 0; e < 21; ++e) { Sfull[e] = Scol[sstride * e]; Sref[e] = Sfull[e] - fd[CUT_FAST + e]; }
                        ++n_xchk;
                        if (!verify_exact_step(p, Dl, q, r0, r1, first, Sref, Sfull, (by & CUT_P_STAY) ? CUT_P_STAY : (by & 7)))
                            bad |= 512;
                    }
                }
                first = 0;
                if (by & CUT_P_STAY) {
                    done = true;
                } else {
                    const int jj = by & 7;
                    r0 = r0 + nb_step(jj, 0, st);
                    r1 = r1 + nb_step(jj, 1, st);
                    if (!(r0 + r1 <= 1.0)) done = true;
                }
            }
            // the replay must end where the search did
            if (!done || __double_as_longlong(r0) != __double_as_longlong(r0f) ||
                __double_as_longlong(r1) != __double_as_longlong(r1f))
                bad |= 1;
        }
    return bad;
}

// k_cut_verify: the S-dependent bound terms of one line from S_ours (LDS column So),
// the reference's whole sum at the line's start (column Sf; S_ref = Sf - i0) and the operand bounds.
// Out of line: its unrolled 6 x 6 loops would otherwise set the kernel's register budget.
struct LineBound {
    double K0, A1, B1, cs, ce, R0, rts, rte, epsS, kt;
    int ok;
};
__device__ __forceinline__ LineBound verify_line_bound(const KParams& p, size_t q, const double* fd, const double* vmx,
                                                      const double* Dl, const double* So, const double* Sf) {
    const double rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    const double T = fmax(fabs(rlo), fabs(rhi));
    const double tau = p.cfg.cut_certify;
    constexpr double u = 0x1p-53;
    LineBound lbd;
    double K0, A1, B1, cs, ce, R0, rts, rte, epsS_l, kt_l;
    bool line_ok;
        float eb[14];
        {
            const float* ebg = reinterpret_cast<const float*>(vmx + 6);   // (k_cut_ebound's)
#pragma unroll
            for (int i = 0; i < 14; ++i) eb[i] = ebg[i];
        }
        double o28[28];
        {
            double S[21];
#pragma unroll
            for (int e = 0; e < 21; ++e) S[e] = So[65 * e];
            chol_s(S, o28);   // (the search's factorization: pivots >= 1e-2 of the diagonal, 1 / L_kk)
        }
        double sg[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double x[6], a = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double uu = i == j ? 1.0 : 0.0;
#pragma unroll
                for (int k = 0; k < i; ++k) uu = uu - o28[tri(i, k)] * x[k];
                x[i] = uu * o28[21 + i];
                a = a + x[i] * x[i];
            }
            sg[j] = 1.002 * a;
        }
        double Bn[2] = {0.0, 0.0};
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            double tk = 1.0;
#pragma unroll
            for (int kk = 0; kk < 3; ++kk) {
                double w[6], a = 0.0;
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    double uu = fd[(side ? PD_PE : PD_PS) + 6 * kk + i];
#pragma unroll
                    for (int k = 0; k < i; ++k) uu = uu - o28[tri(i, k)] * w[k];
                    w[i] = uu * o28[21 + i];
                    a = a + w[i] * w[i];
                }
                Bn[side] = Bn[side] + 1.01 * sqrt(a) * tk;
                tk = tk * T;
            }
        }
        double Kc = 0.0, xi = 0.0, Qs = 0.0, Qe = 0.0, hs0 = 0.0, he0 = 0.0, Lam = 0.0, dSn = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double Sii = So[65 * tri(i, i)];
            const double es = eb[i], ee = eb[7 + i];
            const double ps = fabs(fd[PD_PS + i]) + T * (fabs(fd[PD_PS + 6 + i]) + T * fabs(fd[PD_PS + 12 + i])) + es;
            const double pe = fabs(fd[PD_PE + i]) + T * (fabs(fd[PD_PE + 6 + i]) + T * fabs(fd[PD_PE + 12 + i])) + ee;
            const double kc = Sii * sg[i];
            Kc = Kc + kc;
            xi = xi + sqrt(kc);
            Qs = Qs + sg[i] * ps * ps;
            Qe = Qe + sg[i] * pe * pe;
            hs0 = hs0 + es * sqrt(sg[i]);
            he0 = he0 + ee * sqrt(sg[i]);
            Lam = Lam + ((Sii > 0.0 && Sii < 1e300) ? 0.6931471805599453 * (double)(abs(__builtin_amdgcn_frexp_exp(Sii)) + 1)
                                                     : __builtin_inf());
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                // |S_ours - S_ref| of entry (i, k), S_ref = sE - i0 as the reference forms it; the
                // difference of two such close values is exact (Sterbenz), 2u |.| covers the rest
                const int e = tri(i > k ? i : k, i > k ? k : i);
                const double sref = Sf[65 * e] - fd[CUT_FAST + e];
                const double dd = 1.0000000000000004 * fabs(So[65 * e] - sref);
                dSn = dSn + dd * sqrt(sg[i] * sg[k]);
            }
        }
        const double epsS = 1.01 * dSn + (7.01 * u) * xi * xi;
        const double hs = hs0 + (6.01 * u) * Bn[0] * xi, he = he0 + (6.01 * u) * Bn[1] * xi;
        const double ck = 110.0 * u;
        K0 = 1.002 * epsS + ck * Kc + (7.1 * u) * Lam;
        const double bs = Bn[0] + hs, be = Bn[1] + he;
        // the v'-table's own error (the blended depth's relative error x 4 + the scaling's roundings)
        rts = 4.1 * (double)eb[6] + 16.0 * u;
        rte = 4.1 * (double)eb[13] + 16.0 * u;
        A1 = 1.03 * (2.0 * ck * Qs + 4.0 * hs * bs);
        B1 = 1.03 * (2.0 * ck * Qe + 4.0 * he * be);
        cs = 4.12 * bs * bs;
        ce = 4.12 * be * be;
        R0 = fmin(0.125 * tau, 1e-3) - 1.01 * K0;
        line_ok = o28[27] != 0.0 && epsS <= 1e-3 && Kc <= 1e8 && R0 > 0.0 && rlo >= 0.0 && rhi <= 1.0 &&
                  tau > 0.0 && rts + rte <= 0.01;
        epsS_l = 1.002 * epsS;
        kt_l = ck * Kc + (7.1 * u) * Lam;

    lbd.K0 = K0; lbd.A1 = A1; lbd.B1 = B1; lbd.cs = cs; lbd.ce = ce; lbd.R0 = R0; lbd.rts = rts; lbd.rte = rte;
    lbd.epsS = epsS_l; lbd.kt = kt_l; lbd.ok = line_ok ? 1 : 0;
    return lbd;
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_cut_verify(KParams p) {
    __shared__ double fo[21][65];   // the chunk's lines: our info, then S_ours of the line
    __shared__ double fr[21][65];   // the reference's info, then its whole invCov_sum at the line's start
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int nls = p.tr.n_matched_ls[b];
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    DevLines& L = p.prev.ls;
    const size_t lb = (size_t)b * p.kl_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    const double* rec_l = p.scr.cut_rec + (size_t)b * p.mls_cap * CUT_REC;
    double Dl[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) Dl[i] = p.scr.cut_dtinv[16 * b + i];
    int bad = p.cfg.cut_proof == 3 ? 256 : 0;   // (cut_proof 3: every sequence redone eagerly — a test hook)
    // bad is a reason mask (diagnostics, scr.dbg): 1 replay != search, 2 v' <= 0 or r_v >= 1/4, 512 a step
    // the bound does not cover decided otherwise by the reference's arithmetic
    double worst = 0.0;   // max E / R0 over the margined steps
    double tS = 0.0, tK = 0.0, tA = 0.0, tV = 0.0;   // its terms: eps_S, K0's rest, A1 / B1, the v' terms
    int64_t n_marg = 0, n_eval = 0, n_mline = 0, n_xchk = 0, n_dline = 0;
    // the running sums of the search (sA: ours, S of the line being opened) and of the reference (sE:
    // the whole sum before the line's r = 0 info is taken out), lanes 0-20 hold entry lane
    double sA = 0.0, sE = 0.0;
    if (nls > 0 && lane < 21) {
        const double s0 = p.scr.cut_sum[24 * b + lane];
        sA = s0 - rec_l[CUT_FAST + lane];
        sE = s0;
    }
#ifdef GFPL_VERIFY_CLOCK   // (diagnostic build: shader-clock cycles per phase in scr.dbg 0-4)
    uint64_t vk[5] = {0, 0, 0, 0, 0};
    uint64_t vk0 = clock64();
#define VK(i) do { const uint64_t vk1 = clock64(); vk[i] += vk1 - vk0; vk0 = vk1; } while (0)
#else
#define VK(i) do { } while (0)
#endif
    for (int c0 = 0; c0 < nls; c0 += 64) {   // (wave-uniform)
        const int m = c0 + lane;
        const bool on = m < nls;
        const size_t q = lb + (on ? mls[m] : mls[0]);
        const double* fd = rec_l + (size_t)(on ? m : 0) * CUT_REC;
        const double r0f = L.cut[2 * q], r1f = L.cut[2 * q + 1];
        // (1) the reference's info at the final ratios: invCovPose (k_cut_finish's), and its lower triangle
        {
            LineCutData d;
            load_line(L, q, d);
            double info[36];
            poseInfoOnLine<true>(cam, homog, Dl, d, r0f, r1f, info);
            if (on) {
                double2* iv = reinterpret_cast<double2*>(L.invcov + 36 * q);
#pragma unroll
                for (int i = 0; i < 18; ++i) iv[i] = make_double2(info[2 * i], info[2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 6; ++i)
#pragma unroll
                    for (int k = 0; k <= i; ++k) fr[tri(i, k)][lane] = info[i * 6 + k];
            }
        }
        VK(0);
        // (2) the search's own info of the line (its transition's expressions, cut_ours_*)
        const bool pdok = fd[PD_OK] != 0.0;
        {
            double xs[14];
            if (pdok) {
                xs[0] = cut_ours_V(fd, 0, r0f);
                xs[7] = cut_ours_V(fd, 1, r1f);
#pragma unroll
                for (int i = 0; i < 6; ++i) { xs[1 + i] = cut_ours_P(fd, 0, i, r0f); xs[8 + i] = cut_ours_P(fd, 1, i, r1f); }
            } else {
                exact_endpoint(cam, homog, Dl, L, q, 0, r0f, xs);
                exact_endpoint(cam, homog, Dl, L, q, 1, r1f, xs + 7);
            }
            const double is = rcp_fast(xs[0]), ie = rcp_fast(xs[7]);
            if (on) {
#pragma unroll
                for (int i = 0; i < 6; ++i)
#pragma unroll
                    for (int k = 0; k <= i; ++k) fo[tri(i, k)][lane] = cut_ours_info(xs, is, ie, i, k);
            }
        }
        wave_lds_sync();
        VK(1);
        // (3) the two running sums in list order (lanes 0-20, entry lane): S_ours and the reference's
        //     whole sum at each line's start replace its infos in fo / fr
        const int cnt = min(64, nls - c0);
        if (lane < 21) {
            // the r = 0 infos are fetched 16 lines at a time (one memory round trip per batch, not per line)
            auto fetch = [&](int l0, double* v) {
#pragma unroll
                for (int k = 0; k < 17; ++k) {
                    const int mm = c0 + l0 + k;
                    v[k] = (l0 + k <= cnt && mm < nls) ? rec_l[(size_t)mm * CUT_REC + CUT_FAST + lane] : 0.0;
                }
            };
            // (a double-buffered fetch, the next batch's loads issued before this batch's sums, measured
            // 2.21 vs 1.99 ms: its 34 live registers cost 35 more spills)
            double iv[17];
            for (int l0 = 0; l0 < cnt; l0 += 16) {
                fetch(l0, iv);
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int l = l0 + k;
                    if (l < cnt) {
                        const double sref = sE - iv[k];                // the reference's S of line c0 + l
                        const double f_o = fo[lane][l], f_r = fr[lane][l];
                        fo[lane][l] = sA;
                        fr[lane][l] = sE;
                        sE = sref + f_r;
                        sA = (sA + f_o) - iv[k + 1];
                    }
                }
            }
        }
        wave_lds_sync();
        VK(2);
        // (4) the line's bound terms from S_ours, S_ref = sE - i0, and the operand bounds
        double K0 = 0.0, A1 = 0.0, B1 = 0.0, cs = 0.0, ce = 0.0, R0 = -1.0, rts = 0.0, rte = 0.0;
        double epsS_l = 0.0, kt_l = 0.0;
        bool line_ok = false;
        if (on && pdok) {
            const LineBound lbd = verify_line_bound(p, q, fd, p.scr.cut_vmax + ((size_t)b * p.mls_cap + m) * CUT_VMAX, Dl,
                                                    &fo[0][0] + lane, &fr[0][0] + lane);
            K0 = lbd.K0; A1 = lbd.A1; B1 = lbd.B1; cs = lbd.cs; ce = lbd.ce; R0 = lbd.R0; rts = lbd.rts; rte = lbd.rte;
            epsS_l = lbd.epsS; kt_l = lbd.kt; line_ok = lbd.ok != 0;
        }
        VK(3);
        // (5) the line's margined steps: with k_cut_vref's maxima over the compared ratios, one bound for
        //     every step of the line; a line it does not cover is replayed step by step (the reference's v'
        //     at each step's ratios, the step's own bound) and a step no bound covers is re-decided exactly
        int marg = 0;
        bool detail = false;
        if (on) {
            const double* vm = p.scr.cut_vmax + ((size_t)b * p.mls_cap + m) * CUT_VMAX;
            const double mv = vm[4];
            marg = (int)fmod(mv, 1024.0);
            n_eval += (int64_t)(mv / 1024.0);
            if (marg) {
                const double E = K0 + A1 * vm[0] + cs * (1.01 * vm[1] + rts * vm[0]) + B1 * vm[2] +
                                 ce * (1.01 * vm[3] + rte * vm[2]);
                detail = !(vm[5] == 0.0 && line_ok && E * 1.0001 <= R0);
                if (!detail && E / R0 > worst) {   // (diagnostics: the worst line's terms, relative to R0)
                    worst = E / R0;
                    tS = epsS_l / R0;
                    tK = kt_l / R0;
                    tA = (A1 * vm[0] + B1 * vm[2]) / R0;
                    tV = (cs * (1.01 * vm[1] + rts * vm[0]) + ce * (1.01 * vm[3] + rte * vm[2])) / R0;
                }
            }
            n_marg += marg;
            n_mline += marg ? 1 : 0;
            n_dline += detail ? 1 : 0;
        }
        VK(4);
        if (detail) {   // to k_cut_verify_detail's list (out of this kernel's register budget); a full list: redo
            const int slot = atomicAdd(p.scr.cut_dtln, 1);
            if (slot < CUT_DTL * p.B) {
                double* e = p.scr.cut_dtl + (size_t)slot * 32;
#pragma unroll
                for (int i = 0; i < 21; ++i) e[i] = fr[i][lane];
                e[21] = K0; e[22] = A1; e[23] = B1; e[24] = cs; e[25] = ce; e[26] = R0; e[27] = rts; e[28] = rte;
                e[29] = line_ok ? 1.0 : 0.0;
                p.scr.cut_dtln[1 + slot] = b * p.mls_cap + m;
            } else {
                bad |= 1024;
            }
        }
        wave_lds_sync();
    }
    // the reason mask and the worst E / R0 over the wave's lanes (diagnostics)
    int mask = bad;
    int wl = lane;   // the lane holding the worst step
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mask |= __shfl_xor(mask, o);
        const double ow = __shfl_xor(worst, o);
        const int ol = __shfl_xor(wl, o);
        if (ow > worst || (ow == worst && ol < wl)) { worst = ow; wl = ol; }
    }
    tS = __shfl(tS, wl); tK = __shfl(tK, wl); tA = __shfl(tA, wl); tV = __shfl(tV, wl);
    bad = mask != 0 ? 1 : 0;
    // (the cut endpoints of a proven sequence: k_cut_finish, after k_cut_verify_detail has had its say)
    // counters: lanes' partial counts summed
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        n_marg += __shfl_xor(n_marg, o);
        n_eval += __shfl_xor(n_eval, o);
        n_mline += __shfl_xor(n_mline, o);
        n_xchk += __shfl_xor(n_xchk, o);
        n_dline += __shfl_xor(n_dline, o);
    }
    if (lane == 0) {
        p.scr.cut_flag[b] = bad;
        p.scr.bytes[(size_t)STEP_REC * b + 20] = bad;
        p.scr.bytes[(size_t)STEP_REC * b + 21] = n_marg;
        p.scr.bytes[(size_t)STEP_REC * b + 22] = n_eval;
        p.scr.bytes[(size_t)STEP_REC * b + 23] = n_mline;
        p.scr.dbg[8 * (size_t)b + 4] = mask;
        p.scr.dbg[8 * (size_t)b + 5] = __double_as_longlong(worst);
        p.scr.dbg[8 * (size_t)b + 6] = n_xchk;
        p.scr.dbg[8 * (size_t)b + 7] = n_dline;
        p.scr.dbg[8 * (size_t)b + 0] = __double_as_longlong(tS);
        p.scr.dbg[8 * (size_t)b + 1] = __double_as_longlong(tK);
        p.scr.dbg[8 * (size_t)b + 2] = __double_as_longlong(tA);
        p.scr.dbg[8 * (size_t)b + 3] = __double_as_longlong(tV);
#ifdef GFPL_VERIFY_CLOCK
        for (int i = 0; i < 5; ++i) p.scr.dbg[8 * (size_t)b + i] = (int64_t)vk[i];
#endif
    }
}

// The lines k_cut_verify's line-level bound did not cover, from its list, one lane each: the recorded
// steps replayed with each step's own bound, and a step no bound covers re-decided with the
// reference's arithmetic (verify_line_detail).  A failure flags the sequence for the eager redo.
__global__ void __launch_bounds__(64) k_cut_verify_detail(KParams p) {
    const int n = min(p.scr.cut_dtln[0], CUT_DTL * p.B);
    for (int i = blockIdx.x * 64 + threadIdx.x; i < n; i += gridDim.x * 64) {
        const int e = p.scr.cut_dtln[1 + i];
        const int b = e / p.mls_cap, m = e % p.mls_cap;
        const double* pl = p.scr.cut_dtl + (size_t)i * 32;
        const size_t q = (size_t)b * p.kl_cap + p.tr.matched_ls[(size_t)b * p.mls_cap + m];
        const double* fd = p.scr.cut_rec + ((size_t)b * p.mls_cap + m) * CUT_REC;
        const uint8_t* path = p.scr.cut_path + ((size_t)b * p.mls_cap + m) * CUT_PATH;
        double Dl[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) Dl[k] = p.scr.cut_dtinv[16 * b + k];
        int nx = 0;
        const int bad = verify_line_detail(p, Dl, q, path, fd, p.prev.ls.cut[2 * q], p.prev.ls.cut[2 * q + 1], pl[21],
                                           pl[22], pl[23], pl[24], pl[25], pl[26], pl[27], pl[28], pl[29] != 0.0, pl, 1,
                                           nx);
        if (bad) {
            atomicOr(&p.scr.cut_flag[b], 1);
            atomicOr(reinterpret_cast<unsigned long long*>(&p.scr.bytes[(size_t)STEP_REC * b + 20]), 1ull);
        }
        if (nx) atomicAdd(reinterpret_cast<unsigned long long*>(&p.scr.dbg[8 * (size_t)b + 6]), (unsigned long long)nx);
    }
}

// the batch size up to which the one-sequence-per-wave search runs (GFPL_CUT_WAVE_MAX_B overrides:
// tests run both searches on the same batch)
static int cut_wave_max_b() {
    const char* e = getenv("GFPL_CUT_WAVE_MAX_B");
    return e ? atoi(e) : CUT_WAVE_MAX_B;
}

// the batch size up to which k_cut_prep runs 8 waves per sequence (GFPL_CUT_PREP_W8_MAX_B overrides)
static int cut_prep_w8_max_b() {
    const char* e = getenv("GFPL_CUT_PREP_W8_MAX_B");
    return e ? atoi(e) : 256;
}

hipError_t launch_line_cut(const KParams& p, hipStream_t s, const hipEvent_t* marks) {
    const int mode = p.cfg.cut_proof;   // 0 measured, 1 proven (recorded search + verify), 2 eager-proven, 3 (test)
    const dim3 gsearch((p.B + CUT_G - 1) / CUT_G);
    if (p.B <= cut_prep_w8_max_b()) {   // small batches: 8 waves per sequence
        static std::atomic<unsigned long long> attr{0};
        const hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(k_cut_prep<8>), (int)cut_prep_lds(8), &attr);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_cut_prep<8>, dim3(p.B), dim3(512), cut_prep_lds(8), s, p);
    } else {
        hipLaunchKernelGGL(k_cut_prep<1>, dim3(p.B), dim3(64), cut_prep_lds(1), s, p);
    }
    if (mode == 2) {   // the per-line operand error bounds the eager agreement bound starts from
        hipLaunchKernelGGL(k_cut_bounds, dim3((p.mls_cap + 63) / 64, p.B), dim3(64), 0, s, p);
        hipLaunchKernelGGL(k_cut_vtab, dim3(p.B), dim3(256), 0, s, p);
    }
    if (marks) (void)hipEventRecord(marks[0], s);
    if (mode == 2)
        hipLaunchKernelGGL(k_cut_search<true>, gsearch, dim3(64), 0, s, p);
    else if (p.B <= cut_wave_max_b())   // small batches: one sequence per wave, several steps per round
        hipLaunchKernelGGL(k_cut_search_w, dim3(p.B), dim3(64), 0, s, p);
    else if (mode == 1 || mode == 3)   // (the recorded search)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_cut_search<false, true>), gsearch, dim3(64), 0, s, p);
    else
        hipLaunchKernelGGL(k_cut_search<false>, gsearch, dim3(64), 0, s, p);
    if (marks) (void)hipEventRecord(marks[1], s);
    if (mode == 1 || mode == 3) {
        // prove the recorded decisions (and finish those sequences); redo the others eagerly
        if (hipMemsetAsync(p.scr.cut_offl, 0, sizeof(int32_t), s) != hipSuccess) return hipGetLastError();
        hipLaunchKernelGGL(k_cut_vref, dim3((p.mls_cap + 63) / 64, p.B), dim3(64), 0, s, p);
        hipLaunchKernelGGL(k_cut_vref_off, dim3(256), dim3(64), 0, s, p);
        hipLaunchKernelGGL(k_cut_ebound, dim3((p.mls_cap + 63) / 64, p.B), dim3(64), 0, s, p);
        if (hipMemsetAsync(p.scr.cut_dtln, 0, sizeof(int32_t), s) != hipSuccess) return hipGetLastError();
        hipLaunchKernelGGL(k_cut_verify, dim3(p.B), dim3(64), 0, s, p);
        hipLaunchKernelGGL(k_cut_verify_detail, dim3(256), dim3(64), 0, s, p);
        hipLaunchKernelGGL(k_cut_bounds, dim3((p.mls_cap + 63) / 64, p.B), dim3(64), 0, s, p);
        hipLaunchKernelGGL(k_cut_vtab, dim3(p.B), dim3(256), 0, s, p);
        hipLaunchKernelGGL(k_cut_search<true>, gsearch, dim3(64), 0, s, p);
    }
    hipLaunchKernelGGL(k_cut_finish, dim3(p.B), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace gfpl
