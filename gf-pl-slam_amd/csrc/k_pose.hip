// k_pose.hip — robust Gauss-Newton pose: optimizePose(prev_frame->DT)
// (src/stereoFrameHandler.cpp:1939-2030) with gaussNewtonOptimization (:2032-2056),
// optimizeFunctions (:2118-2245), removeOutliers (:2058-2116) and
// vector_stdv_mad (src/auxiliar.cpp:521-537).
//
// One 256-thread workgroup owns one sequence for the whole two-stage solve:
//  * every GN iteration all threads evaluate the per-feature Jacobian rows
//    (J[6], |e|, Cauchy weight) of the matched list into LDS;
//  * 56 threads then form the 6x6 J^T W J reduction (21 unique H entries + 6 g
//    + 1 e, separately for points and lines), each summing one entry over the
//    list in list order — the reference's accumulation order, so H is bit-identical;
//  * thread 0 solves the 6x6 LDLT, applies the SE(3) update and tests convergence.
// The outlier pass sorts residuals in LDS (bitonic) for the MAD medians.
#include "gfpl_kernels.hpp"

namespace gfpl {

struct PoseLDS {
    double DT[16];
    double DTini[16];
    double H[36];
    double part[56];
    int npart[2];
    int brk;
    int ninl;
    double err;
};

// feature rows: feat[f*8 + 0..5] = J, [6] = |e|, [7] = w;  act[f] = inlier
__device__ void eval_features(const KParams& p, int b, const double* DT, double* feat, uint8_t* act, int npt,
                              int nls) {
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    const DevPoints& P = p.prev.pt;
    const DevLines& L = p.prev.ls;
    const int32_t* mpt = p.tr.matched_pt + (size_t)b * p.mpt_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    const size_t pb = (size_t)b * p.kp_cap, lb = (size_t)b * p.kl_cap;
    for (int f = threadIdx.x; f < npt + nls; f += blockDim.x) {
        double J[6], n, w;
        if (f < npt) {
            const size_t q = pb + mpt[f];
            if (!P.inlier[q]) { act[f] = 0; continue; }
            double Pp[3] = {P.P[3 * q], P.P[3 * q + 1], P.P[3 * q + 2]};
            double Pc[3], uv[2];
            se3_apply(DT, Pp, Pc);
            projection(cam, Pc, uv);
            const double ex = uv[0] - P.pl_obs[2 * q], ey = uv[1] - P.pl_obs[2 * q + 1];
            n = sqrt(ex * ex + ey * ey);
            poseJac(cam, homog, Pc, ex, ey, J);
            const double m = ref_max(homog, n);
#pragma unroll
            for (int i = 0; i < 6; ++i) J[i] = J[i] / m;
            w = 1.0 / (1.0 + (n * n) * P.sigma2[q]);
        } else {
            const size_t q = lb + mls[f - npt];
            if (!L.inlier[q]) { act[f] = 0; continue; }
            double sP[3] = {L.sP[3 * q], L.sP[3 * q + 1], L.sP[3 * q + 2]};
            double eP[3] = {L.eP[3 * q], L.eP[3 * q + 1], L.eP[3 * q + 2]};
            double sc[3], ec[3], su[2], eu[2];
            se3_apply(DT, sP, sc);
            projection(cam, sc, su);
            se3_apply(DT, eP, ec);
            projection(cam, ec, eu);
            const double l0 = L.le_obs[3 * q], l1 = L.le_obs[3 * q + 1], l2 = L.le_obs[3 * q + 2];
            const double ds = (l0 * su[0] + l1 * su[1]) + l2;
            const double de = (l0 * eu[0] + l1 * eu[1]) + l2;
            n = sqrt(ds * ds + de * de);
            double Js[6], Je[6];
            poseJac(cam, homog, sc, l0, l1, Js);
            poseJac(cam, homog, ec, l0, l1, Je);
            const double m = ref_max(homog, n);
#pragma unroll
            for (int i = 0; i < 6; ++i) J[i] = (Js[i] * ds + Je[i] * de) / m;
            w = 1.0 / (1.0 + (n * n) * L.sigma2[q]);
        }
        act[f] = 1;
        double* o = feat + (size_t)f * 8;
#pragma unroll
        for (int i = 0; i < 6; ++i) o[i] = J[i];
        o[6] = n;
        o[7] = w;
    }
}

// one reduction entry e in [0,28): H lower (i,j), g_i, e
__device__ __forceinline__ double term(const double* o, int e, int ti, int tj) {
    if (e < 21) return (o[ti] * o[tj]) * o[7];
    if (e < 27) return (o[e - 21] * o[6]) * o[7];
    return (o[6] * o[6]) * o[7];
}

// gaussNewtonOptimization; returns via S: DT updated in place, H (last evaluated), err
__device__ void gauss_newton(const KParams& p, int b, PoseLDS& S, double* feat, uint8_t* act, int npt, int nls,
                             int max_iters) {
    const int tid = threadIdx.x;
    double err_prev = 999999999.9;   // thread 0 only
    if (tid == 0) S.err = 0.0;
    for (int it = 0; it < max_iters; ++it) {
        double DT[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) DT[i] = S.DT[i];
        eval_features(p, b, DT, feat, act, npt, nls);
        __syncthreads();
        if (tid < 56) {
            const int list = tid / 28, e = tid % 28;
            int ti = 0, tj = 0;
            if (e < 21) { ti = 0; while ((ti + 1) * (ti + 2) / 2 <= e) ++ti; tj = e - ti * (ti + 1) / 2; }
            const int f0 = list == 0 ? 0 : npt, f1 = list == 0 ? npt : npt + nls;
            double s = 0.0;
            int cnt = 0;
#pragma unroll 4
            for (int f = f0; f < f1; ++f) {
                const double t = term(feat + (size_t)f * 8, e, ti, tj);
                const bool a = act[f] != 0;
                s = a ? s + t : s;
                cnt += a ? 1 : 0;
            }
            S.part[tid] = s;
            if (e == 0) S.npart[list] = cnt;
        }
        __syncthreads();
        if (tid == 0) {
            double H[36], g[6];
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j <= i; ++j) {
                    const double v = S.part[tri(i, j)] + S.part[28 + tri(i, j)];
                    H[i * 6 + j] = v; H[j * 6 + i] = v;
                }
            for (int i = 0; i < 6; ++i) g[i] = S.part[21 + i] + S.part[28 + 21 + i];
            double e = S.part[27] + S.part[28 + 27];
            e = e / (double)(S.npart[1] + S.npart[0]);
            for (int i = 0; i < 36; ++i) S.H[i] = H[i];
            S.err = e;
            int brk = 0;
            if ((fabs(e - err_prev) < p.cfg.min_error_change) || (e < p.cfg.min_error)) {
                brk = 1;
            } else {
                double inc[6], E[16], Ei[16], Dn[16];
                ldlt_solve6(H, g, inc);
                expmap_se3(inc, E);
                inverse_se3(E, Ei);
                mat4_mul(DT, Ei, Dn);
                for (int i = 0; i < 16; ++i) S.DT[i] = Dn[i];
                const double nrm = sqrt(((((inc[0] * inc[0] + inc[1] * inc[1]) + inc[2] * inc[2]) + inc[3] * inc[3]) +
                                         inc[4] * inc[4]) + inc[5] * inc[5]);
                if (nrm < 2.220446049250313e-16) brk = 1;
                err_prev = e;
            }
            S.brk = brk;
        }
        __syncthreads();
        if (S.brk) break;
    }
}

// vector_stdv_mad on res[0..n) (LDS, destroyed); scratch buf has NP2 entries
__device__ double stdv_mad(double* buf, int n, int NP2) {
    if (n == 0) return 0.0;   // uniform
    for (int i = threadIdx.x + n; i < NP2; i += blockDim.x) buf[i] = __builtin_inf();
    __syncthreads();
    for (int k = 2; k <= NP2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < NP2; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    bool up = ((i & k) == 0);
                    double x = buf[i], y = buf[ixj];
                    if ((x > y) == up) { buf[i] = y; buf[ixj] = x; }
                }
            }
            __syncthreads();
        }
    const double median = buf[n / 2];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) buf[i] = (double)fabsf((float)(buf[i] - median));
    __syncthreads();
    for (int k = 2; k <= NP2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < NP2; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    bool up = ((i & k) == 0);
                    double x = buf[i], y = buf[ixj];
                    if ((x > y) == up) { buf[i] = y; buf[ixj] = x; }
                }
            }
            __syncthreads();
        }
    const double mad = buf[n / 2];
    __syncthreads();
    return 1.4826 * mad;
}

// dynamic LDS: feat[(mpt+mls)*8] f64 (reused for residual sorts) | act[mpt+mls] u8
__global__ void __launch_bounds__(256) k_pose(KParams p, int NP2, int featN) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ PoseLDS S;
    __shared__ int cnt[4];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int npt = p.tr.n_matched_pt[b], nls = p.tr.n_matched_ls[b];
    double* feat = (double*)smem;
    uint8_t* act = (uint8_t*)(feat + featN);
    DevPose& CP = p.curr.pose;
    const DevPose& PP = p.prev.pose;
    if (tid < 16) { S.DTini[tid] = PP.DT[16 * b + tid]; S.DT[tid] = S.DTini[tid]; }   // Q2
    if (tid == 0) { S.ninl = p.tr.n_inliers[b]; cnt[0] = cnt[1] = 0; }
    __syncthreads();
    int ok = 0;        // 1: stage-2 DT usable
    double err = 0.0;  // err of the last GN run (reference: uninitialised when no GN runs, pinned 0)
    if (S.ninl > p.cfg.min_features) {
        gauss_newton(p, b, S, feat, act, npt, nls, p.cfg.max_iters);
        err = S.err;
        double DTs[16];
        for (int i = 0; i < 16; ++i) DTs[i] = S.DT[i];
        bool fin = true;
        for (int i = 0; i < 16; ++i) { double d = DTs[i] - DTs[i]; if (!(d == d)) fin = false; }
        if (fin) {
            // removeOutliers(DT_): residuals of every list entry
            const DevPoints& P = p.prev.pt;
            const DevLines& L = p.prev.ls;
            const int32_t* mpt = p.tr.matched_pt + (size_t)b * p.mpt_cap;
            const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
            const size_t pb = (size_t)b * p.kp_cap, lb = (size_t)b * p.kl_cap;
            double* rp = feat;                 // [npt] residuals (kept)
            double* rl = feat + NP2;           // [nls]
            double* buf = feat + 2 * NP2;      // sort scratch [NP2]
            for (int k = tid; k < npt; k += blockDim.x) {
                const size_t q = pb + mpt[k];
                double Pp[3] = {P.P[3 * q], P.P[3 * q + 1], P.P[3 * q + 2]}, Pc[3], uv[2];
                se3_apply(DTs, Pp, Pc);
                projection(p.cam, Pc, uv);
                const double ex = uv[0] - P.pl_obs[2 * q], ey = uv[1] - P.pl_obs[2 * q + 1];
                rp[k] = sqrt(ex * ex + ey * ey) * sqrt(P.sigma2[q]);
            }
            for (int k = tid; k < nls; k += blockDim.x) {
                const size_t q = lb + mls[k];
                double sP[3] = {L.sP[3 * q], L.sP[3 * q + 1], L.sP[3 * q + 2]};
                double eP[3] = {L.eP[3 * q], L.eP[3 * q + 1], L.eP[3 * q + 2]};
                double sc[3], ec[3], su[2], eu[2];
                se3_apply(DTs, sP, sc);
                se3_apply(DTs, eP, ec);
                projection(p.cam, sc, su);
                projection(p.cam, ec, eu);
                const double l0 = L.le_obs[3 * q], l1 = L.le_obs[3 * q + 1], l2 = L.le_obs[3 * q + 2];
                const double e0 = (l0 * su[0] + l1 * su[1]) + l2;
                const double e1 = (l0 * eu[0] + l1 * eu[1]) + l2;
                rl[k] = sqrt(e0 * e0 + e1 * e1) * sqrt(L.sigma2[q]);
            }
            __syncthreads();
            for (int k = tid; k < npt; k += blockDim.x) buf[k] = rp[k];
            __syncthreads();
            const double th_p = p.cfg.inlier_k * stdv_mad(buf, npt, NP2);
            for (int k = tid; k < nls; k += blockDim.x) buf[k] = rl[k];
            __syncthreads();
            const double th_l = p.cfg.inlier_k * stdv_mad(buf, nls, NP2);
            for (int k = tid; k < npt; k += blockDim.x)
                if (rp[k] > th_p) { p.prev.pt.inlier[pb + mpt[k]] = 0; atomicAdd(&cnt[0], 1); }
            for (int k = tid; k < nls; k += blockDim.x)
                if (rl[k] > th_l) { p.prev.ls.inlier[lb + mls[k]] = 0; atomicAdd(&cnt[1], 1); }
            __syncthreads();
            if (tid == 0) {
                S.ninl = S.ninl - cnt[0] - cnt[1];
                p.tr.n_inliers[b] = S.ninl;
                p.tr.n_inliers_pt[b] -= cnt[0];
                p.tr.n_inliers_ls[b] -= cnt[1];
            }
            __syncthreads();
            if (S.ninl > p.cfg.min_features) {
                if (tid < 16) S.DT[tid] = S.DTini[tid];   // Q3: stage 2 restarts from DT_ini
                __syncthreads();
                gauss_newton(p, b, S, feat, act, npt, nls, p.cfg.max_iters_ref);
                err = S.err;
                ok = 1;
            }
        }
    }
    if (tid == 0) {
        for (int i = 0; i < 16; ++i) p.scr.pose_DT[16 * b + i] = S.DT[i];
        for (int i = 0; i < 36; ++i) p.scr.pose_H[36 * b + i] = S.H[i];
        p.scr.pose_err[b] = err;
        p.scr.pose_ok[b] = ok;
    }
}

// Final bookkeeping of optimizePose (src/stereoFrameHandler.cpp:1983-2028), one
// lane per sequence: inverse_se3, motion-step gate, Tfw, DT_cov = H^-1 (Q13),
// its eigenvalues, Tfw_cov = unccomp_se3, err_norm, numFrameLoss.
__global__ void __launch_bounds__(64) k_pose_finish(KParams p) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    DevPose& CP = p.curr.pose;
    const DevPose& PP = p.prev.pose;
    const int ok = p.scr.pose_ok[b];
    const double err = p.scr.pose_err[b];
    double DT[16], DT_cov[36];
    if (ok) {
        double H[36];
#pragma unroll
        for (int i = 0; i < 16; ++i) DT[i] = p.scr.pose_DT[16 * b + i];
#pragma unroll
        for (int i = 0; i < 36; ++i) H[i] = p.scr.pose_H[36 * b + i];
        inverse6(H, DT_cov);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) DT[i] = (i % 5 == 0) ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < 36; ++i) DT_cov[i] = 0.0;
    }
    bool fin = true;
#pragma unroll
    for (int i = 0; i < 16; ++i) { double d = DT[i] - DT[i]; if (!(d == d)) fin = false; }
    double Tp[16], Tpc[36];
#pragma unroll
    for (int i = 0; i < 16; ++i) Tp[i] = PP.Tfw[16 * b + i];
#pragma unroll
    for (int i = 0; i < 36; ++i) Tpc[i] = PP.Tfw_cov[36 * b + i];
    double cDT[16], Tfw[16], Tcov[36], eig[6];
    double err_norm;
    bool moved = false;
    if (fin) {
        inverse_se3(DT, cDT);
        const double tn = sqrt((cDT[3] * cDT[3] + cDT[7] * cDT[7]) + cDT[11] * cDT[11]);
        moved = tn < p.cfg.motion_step_th * (CP.time_stamp[b] - PP.time_stamp[b]);
        p.tr.num_frame_loss[b] = 0;
    } else {
        p.tr.num_frame_loss[b] = p.tr.num_frame_loss[b] + 1;
    }
    if (moved) {
        mat4_mul(Tp, cDT, Tfw);
        // unccomp_se3(prev.Tfw, prev.Tfw_cov, DT_cov) (src/auxiliar.cpp:216-238)
        double Ad[36], R[9], t[3] = {Tp[3], Tp[7], Tp[11]}, Sk[9], SR[9];
#pragma unroll
        for (int i = 0; i < 36; ++i) Ad[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) R[i * 3 + j] = Tp[i * 4 + j];
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
        double AS[36];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double s = Ad[i * 6 + 0] * DT_cov[0 * 6 + j];
#pragma unroll
                for (int k = 1; k < 6; ++k) s = s + Ad[i * 6 + k] * DT_cov[k * 6 + j];
                AS[i * 6 + j] = s;
            }
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double s = AS[i * 6 + 0] * Ad[j * 6 + 0];
#pragma unroll
                for (int k = 1; k < 6; ++k) s = s + AS[i * 6 + k] * Ad[j * 6 + k];
                Tcov[i * 6 + j] = Tpc[i * 6 + j] + s;
            }
        err_norm = err;
    } else {
        // rejected step or non-finite pose: identity, prev pose kept, err_norm = -1
#pragma unroll
        for (int i = 0; i < 16; ++i) { cDT[i] = (i % 5 == 0) ? 1.0 : 0.0; Tfw[i] = Tp[i]; }
#pragma unroll
        for (int i = 0; i < 36; ++i) Tcov[i] = Tpc[i];
        err_norm = -1.0;
    }
    eig_sym<6>(DT_cov, eig);
#pragma unroll
    for (int i = 0; i < 16; ++i) { CP.DT[16 * b + i] = cDT[i]; CP.Tfw[16 * b + i] = Tfw[i]; }
#pragma unroll
    for (int i = 0; i < 36; ++i) { CP.DT_cov[36 * b + i] = DT_cov[i]; CP.Tfw_cov[36 * b + i] = Tcov[i]; }
#pragma unroll
    for (int i = 0; i < 6; ++i) CP.DT_cov_eig[6 * b + i] = eig[i];
    CP.err_norm[b] = err_norm;
}

hipError_t launch_pose(const KParams& p, hipStream_t s) {
    int NP2 = 1;
    while (NP2 < p.mpt_cap || NP2 < p.mls_cap) NP2 <<= 1;
    size_t feat = (size_t)(p.mpt_cap + p.mls_cap) * 8;
    if (feat < (size_t)3 * NP2) feat = (size_t)3 * NP2;
    const size_t lds = feat * 8 + (size_t)(p.mpt_cap + p.mls_cap) + 16;
    hipLaunchKernelGGL(k_pose, dim3(p.B), dim3(256), lds, s, p, NP2, (int)feat);
    hipLaunchKernelGGL(k_pose_finish, dim3((p.B + 63) / 64), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace gfpl
