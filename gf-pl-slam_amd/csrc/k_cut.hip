// k_cut.hip — good-line-cut: estimateProjUncertainty_submodular(0.05, {0,1})
// (src/stereoFrameHandler.cpp:1618-1764) with getPoseInfoOnLine (:1342-1411),
// getPoseInfoPoint (:1414-1447), updateEndPointByRatio (:1451-1470) and logdet
// (include/linespec.h:43-56).
//
// The search is a serial chain over matched lines: each line's greedy search
// reads invCov_sum after all earlier lines were cut.  Three kernels:
//  k_cut_prep   (one wave / sequence) r = (0,0) infos of lines and points and
//               invCov_sum, each entry summed in list order (lines, then points)
//               by one lane over 64-entry chunks staged in LDS, plus the metric
//               logdet(invCov_sum) that opens the first line;
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

// ------------------------------------------------------------------ prep --
__global__ void __launch_bounds__(64) k_cut_prep(KParams p) {
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
    __syncthreads();
    if (lane == 0) {   // metric of the first line's search: logdet(invCov_sum) (:1671)
        double a[21];
#pragma unroll
        for (int i = 0; i < 21; ++i) a[i] = p.scr.cut_sum[24 * b + i];
        p.scr.cut_sum[24 * b + 21] = logdet6_lower(a);
    }
}

// ---------------------------------------------------------------- search --
// 8 sequences per wave, 8 lanes each; every wave iteration is one greedy step
// of each of its 8 chains, in three phases separated by wave barriers:
//   E  lanes 0-2 of a group compute the start endpoint at t0 = r0 + {-s, 0, +s},
//      lanes 3-5 the end endpoint at t1 = r1 + {-s, 0, +s} (cut_endpoint: blend,
//      projected variance, pose Jacobian).  A neighbour's start terms depend on
//      t0 only and its end terms on t1 only, so the 8 neighbours share these 6;
//   C  lane j assembles neighbour j's info from its two endpoints, adds
//      invCov_sum and takes the logdet (first failing LLT pivot kept, Q11);
//   D  the group takes the first strict maximum over the valid neighbours (the
//      reference's j-loop); no improvement finalises the line: invCov_sum +=
//      info of the chosen ratio (re-assembled from the middle endpoints, the
//      same arithmetic as the chosen candidate's), the cut ratio is stored and
//      the next line opens at (0, 0).
// The metric that opens line m+1, logdet(invCov_sum), equals line m's final
// metric whenever line m moved: invCov_sum' = (sum - info_m) + chosen has the
// bits of the chosen candidate's own total chosen + (sum - info_m).  Only when a
// line never moved and the sum did not come back bit-identical is it evaluated
// (one extra "setup" iteration, lane 0 of the group).
#define CUT_G 8   // sequences per wave (8 lanes each)

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
__device__ __forceinline__ bool same_bits(double a, double b) {
    return __double_as_longlong(a) == __double_as_longlong(b);
}

__global__ void __launch_bounds__(64) k_cut_search(KParams p) {
    // per-group rows padded by one double so the 8 groups of a wave sit in
    // different LDS banks when their lanes read the same entry
    __shared__ double sum[CUT_G][25];
    __shared__ double sumb[CUT_G][25];
    __shared__ double epf[CUT_G * 49];   // group g, slot j: epf + 49 g + 8 j (v, J[6])
    __shared__ double val[CUT_G][9];
    __shared__ int vld[CUT_G][8];
    __shared__ double nxt[CUT_G][49];    // prefetched next line: sP eP covS covE Jl (26) | r=0 info (21)
    const int lane = threadIdx.x;
    const int g = lane >> 3, j = lane & 7;
    const int b = blockIdx.x * CUT_G + g;
    const bool live = b < p.B;
    const int nls = live ? p.tr.n_matched_ls[b] : 0;
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    DevLines& L = p.prev.ls;
    const size_t lb = (size_t)(live ? b : 0) * p.kl_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)(live ? b : 0) * p.mls_cap;
    const double* scr_l = p.scr.cut_ls + (size_t)(live ? b : 0) * p.mls_cap * 21;
    double Dl[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) Dl[i] = live && nls > 0 ? p.scr.cut_dtinv[16 * b + i] : 0.0;
    const double st = p.cfg.cut_step;
    const double rlo = p.cfg.cut_rng[0], rhi = p.cfg.cut_rng[1];
    // E role of this lane
    const int eside = j < 3 ? 0 : 1;
    const double eoff = (j % 3) == 0 ? -st : ((j % 3) == 2 ? st : 0.0);
    // C role: neighbour j
    const double nb0 = nb_step(j, 0, st), nb1 = nb_step(j, 1, st);
    const int cs = nb_slot(j, 0), ce = 3 + nb_slot(j, 1);
    // group state (identical in the 8 lanes of a group)
    int m = 0;
    int setup = 0;       // 1: this iteration evaluates logdet(invCov_sum) only
    int moved = 0;
    double r0 = 0.0, r1 = 0.0, mb = 0.0, mb_init = 0.0;
    LineCutData d;
    // Next-line prefetch: lane j loads elements j, j+8, ... of the 47-element vector
    // [line data | r = 0 info] of the group's next line right after a line opens;
    // the values land in LDS one iteration later, so opening a line never waits on HBM.
    double pf[6];
    int pending = 0;
    auto pf_issue = [&](int mm) {
        const size_t q = lb + mls[mm];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int e = j + 8 * k;
            const double* src;
            size_t off;
            if (e < 3) { src = L.sP; off = 3 * q + e; }
            else if (e < 6) { src = L.eP; off = 3 * q + (e - 3); }
            else if (e < 15) { src = L.covS; off = 9 * q + (e - 6); }
            else if (e < 24) { src = L.covE; off = 9 * q + (e - 15); }
            else if (e < 26) { src = L.le_obs; off = 3 * q + (e - 24); }
            else { src = scr_l; off = (size_t)mm * 21 + (size_t)(e < 47 ? e - 26 : 0); }
            pf[k] = src[off];
        }
        pending = 1;
    };
    if (m < nls) {
        load_line(L, lb + mls[m], d);
        for (int e = j; e < 21; e += 8) {
            const double s0 = p.scr.cut_sum[24 * b + e];
            sumb[g][e] = s0;
            sum[g][e] = s0 - scr_l[e];
        }
        mb = p.scr.cut_sum[24 * b + 21];   // logdet(invCov_sum) from k_cut_prep
        mb_init = mb;
        if (nls > 1) pf_issue(1);
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) { d.sP[k] = 0.0; d.eP[k] = 1.0; }
#pragma unroll
        for (int k = 0; k < 9; ++k) { d.covS[k] = 0.0; d.covE[k] = 0.0; }
        d.Jl[0] = 0.0; d.Jl[1] = 0.0;
    }
    __syncthreads();
    while (__any(m < nls)) {   // wave-uniform loop; groups that are done idle
        const bool act = m < nls;
        // ---- E: the six endpoints of this step
        if (j < 6) {
            const double t = (eside == 0 ? r0 : r1) + eoff;
            double out[7];
            if (eside == 0) cut_endpoint(cam, homog, Dl, d.Jl, d.sP, d.eP, d.covS, d.covE, t, out);
            else cut_endpoint(cam, homog, Dl, d.Jl, d.eP, d.sP, d.covE, d.covS, t, out);
#pragma unroll
            for (int i = 0; i < 7; ++i) epf[49 * g + 8 * j + i] = out[i];
        }
        __syncthreads();
        // ---- C: neighbour j (or the setup logdet)
        {
            const double t0 = r0 + nb0, t1 = r1 + nb1;
            int valid = 1;
            if (t0 + t1 > 1.0) valid = 0;
            if (t0 < rlo || t0 > rhi) valid = 0;
            if (t1 < rlo || t1 > rhi) valid = 0;
            double tot[21];
            if (setup) {
#pragma unroll
                for (int i = 0; i < 21; ++i) tot[i] = sumb[g][i];
            } else {
                double tmp[21];
                cut_assemble<false>(epf + 49 * g + 8 * cs, epf + 49 * g + 8 * ce, tmp);
#pragma unroll
                for (int i = 0; i < 21; ++i) tot[i] = tmp[i] + sum[g][i];
            }
            const double v = logdet6_lower(tot);
            if (act) {
                val[g][j] = v;
                vld[g][j] = setup ? 0 : valid;
            }
        }
        __syncthreads();
        // ---- land the prefetched next line in LDS (its loads were issued >= 1 iteration ago)
        if (pending) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (j + 8 * k < 47) nxt[g][j + 8 * k] = pf[k];
            pending = 0;
        }
        __syncthreads();
        // ---- D: group decision (all 8 lanes compute it identically)
        int finalize = 0, stale_mid = 0;
        if (act) {
            if (setup) {
                mb = val[g][0];
                mb_init = mb;
                setup = 0;
            } else {
                double mi = mb;
                int best = -1;
#pragma unroll
                for (int jj = 0; jj < 8; ++jj)
                    if (vld[g][jj] && val[g][jj] > mi) { mi = val[g][jj]; best = jj; }
                if (best >= 0) {
                    r0 = r0 + nb_step(best, 0, st);
                    r1 = r1 + nb_step(best, 1, st);
                    mb = mi;
                    moved = 1;
                    if (!(r0 + r1 <= 1.0)) { finalize = 1; stale_mid = 1; }   // while-condition
                } else {
                    finalize = 1;   // the middle endpoints of this step are (r0 + 0, r1 + 0) = (r0, r1)
                }
            }
        }
        if (act && finalize) {
            // invCov_sum += info of the chosen ratio
            double S7[7], E7[7];
            if (!stale_mid) {
#pragma unroll
                for (int i = 0; i < 7; ++i) { S7[i] = epf[49 * g + 8 + i]; E7[i] = epf[49 * g + 32 + i]; }
            } else {
                cut_endpoint(cam, homog, Dl, d.Jl, d.sP, d.eP, d.covS, d.covE, r0, S7);
                cut_endpoint(cam, homog, Dl, d.Jl, d.eP, d.sP, d.covE, d.covS, r1, E7);
            }
            double info[21];
            cut_assemble<false>(S7, E7, info);
            int differs = 0;
#pragma unroll
            for (int e = 0; e < 21; ++e) {   // lane j owns entries j, j+8, j+16 (compile-time register index)
                if ((e & 7) == j) {
                    const double ns = sum[g][e] + info[e];
                    differs |= same_bits(ns, sumb[g][e]) ? 0 : 1;
                    sum[g][e] = ns;
                }
            }
            // group-level "the sum came back bit-identical" (consulted only if the line never moved)
            const unsigned long long bad = __ballot(differs);
            const bool same = ((bad >> (8 * g)) & 0xFFull) == 0;
            if (j == 0) {
                const size_t q = lb + mls[m];
                L.cut[2 * q] = r0;
                L.cut[2 * q + 1] = r1;
            }
            ++m;
            if (m < nls) {
                if (!moved) {
                    if (same) mb = mb_init;   // logdet of a bit-identical sum
                    else setup = 1;           // evaluated next iteration
                }
                moved = 0;
                r0 = 0.0;
                r1 = 0.0;
                // line m from the prefetch buffer (same values load_line would read)
#pragma unroll
                for (int k = 0; k < 3; ++k) { d.sP[k] = nxt[g][k]; d.eP[k] = nxt[g][3 + k]; }
#pragma unroll
                for (int k = 0; k < 9; ++k) { d.covS[k] = nxt[g][6 + k]; d.covE[k] = nxt[g][15 + k]; }
                d.Jl[0] = nxt[g][24];
                d.Jl[1] = nxt[g][25];
                // open line m: sumb = invCov_sum, sum = invCov_sum - info(line m, r = 0)
                for (int e = j; e < 21; e += 8) {
                    const double s0 = sum[g][e];
                    sumb[g][e] = s0;
                    sum[g][e] = s0 - nxt[g][26 + e];
                }
                if (!setup) mb_init = mb;
                if (m + 1 < nls) pf_issue(m + 1);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- finish --
// invCovPose of the chosen ratio + updateEndPointByRatio (ledger Q4)
__global__ void __launch_bounds__(64) k_cut_finish(KParams p) {
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
        for (int i = 0; i < 36; ++i) L.invcov[36 * q + i] = info[i];
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
