// k_cross.hip — cross-frame matching (gfx950).
//
//  k_cross_points : predictFramePose (src/stereoFrameHandler.cpp:153-157) +
//                   crossFrameMatching_Hybrid points (:451-603) + projectPrev3DPoint
//                   (src/stereoFrame.cpp:1550-1570).  The reference's radiusMatch(50) +
//                   10 px projection gate + multimap resolution is restated as: for every
//                   current point t, the lexicographic minimum (dist, q) over previous
//                   points q passing both gates (ledger U3: distinct keys ascending;
//                   ties -> earliest inserted = lowest q); the first max_point_match_num
//                   t with a candidate form matched_pt (ledger Q12: duplicates allowed,
//                   pl_obs of a duplicated q comes from its largest accepted t).
//  k_cross_lines  : crossFrameMatching_Hybrid lines (:605-690): knn-2 NORM_HAMMING both
//                   ways, lineDescriptorMAD + lineDescriptorBudgetThres via 257-bin LDS
//                   histograms (the medians are order statistics of small integers),
//                   mutual check, first max_line_match_num accepted in prev order.
#include "gfpl_kernels.hpp"

namespace gfpl {

// dynamic LDS: projx[cap] projy[cap] f64 | lastT[cap] i32 | Tinv[16] f64 | misc[64] i32
__global__ void __launch_bounds__(1024) k_cross_points(KParams p) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int b = blockIdx.x;
    const int cap = p.kp_cap;
    double* projx = (double*)smem;
    double* projy = projx + cap;
    double* Tinv = projy + cap;
    double* prevT = Tinv + 16;
    int* lastT = (int*)(prevT + 16);
    int* misc = lastT + cap;
    const int tid = threadIdx.x;
    const int Sp = p.prev.pt.n[b], Sc = p.curr.pt.n[b];
    if (tid == 0) {
        // predictFramePose: curr.Tfw = prev.Tfw * prev.DT
        double T[16], A[16], Bm[16];
        for (int i = 0; i < 16; ++i) { A[i] = p.prev.pose.Tfw[16 * b + i]; Bm[i] = p.prev.pose.DT[16 * b + i]; }
        mat4_mul(A, Bm, T);
        for (int i = 0; i < 16; ++i) { p.curr.pose.Tfw[16 * b + i] = T[i]; prevT[i] = A[i]; }
        mat4_inv(T, Tinv);
    }
    __syncthreads();
    int total = 0;
    if (Sp > 0 && Sc > 0) {
        const DevPoints& P = p.prev.pt;
        const DevPoints& Cc = p.curr.pt;
        const size_t pb = (size_t)b * cap;
        for (int q = tid; q < Sp; q += blockDim.x) {
            double v[4] = {P.P[3 * (pb + q)], P.P[3 * (pb + q) + 1], P.P[3 * (pb + q) + 2], 1.0};
            mat4_vec(prevT, v, v);
            mat4_vec(Tinv, v, v);
            double uv[2];
            projection(p.cam, v, uv);
            projx[q] = uv[0];
            projy[q] = uv[1];
            lastT[q] = -1;
        }
        __syncthreads();
        const double gate = p.cfg.proj_gate_px;
        const double pre = gate + 0.5;   // exact pre-filter: |dx| > gate+0.5 implies norm > gate
        const float radius = (float)p.cfg.point_match_radius;
        const int cap_m = p.cfg.max_point_match_num;
        const uint8_t* PD = P.desc + pb * 32;
        int off = 0;
        for (int c0 = 0; c0 < Sc; c0 += blockDim.x) {
            const int t = c0 + tid;
            int bestq = -1;
            if (t < Sc) {
                const double plx = Cc.pl[2 * (pb + t)], ply = Cc.pl[2 * (pb + t) + 1];
                uint32_t dt[8];
                load_desc(Cc.desc + (pb + t) * 32, dt);
                int bestd = 0x7FFFFFFF;
                for (int q = 0; q < Sp; ++q) {
                    const double dx = projx[q] - plx, dy = projy[q] - ply;
                    if (fabs(dx) > pre || fabs(dy) > pre) continue;
                    if (sqrt(dx * dx + dy * dy) > gate) continue;
                    uint32_t dq[8];
                    load_desc(PD + (size_t)q * 32, dq);
                    const int d = hamming8<1>(dq, dt);
                    if ((float)d <= radius && d < bestd) { bestd = d; bestq = q; }
                }
            }
            const int has = bestq >= 0 ? 1 : 0;
            int tot;
            const int rank = off + block_exclusive_scan<1024>(has, misc, &tot);
            if (has && rank < cap_m) {
                p.tr.matched_pt[(size_t)b * p.mpt_cap + rank] = bestq;
                Cc.idx[pb + t] = P.idx[pb + bestq];
                atomicMax(&lastT[bestq], t);
            }
            off += tot;
            if (off >= cap_m) break;   // uniform: every thread sees the same off
        }
        total = off < cap_m ? off : cap_m;
        __syncthreads();
        for (int q = tid; q < Sp; q += blockDim.x) {
            const int t = lastT[q];
            if (t >= 0) {
                P.pl_obs[2 * (pb + q)] = Cc.pl[2 * (pb + t)];
                P.pl_obs[2 * (pb + q) + 1] = Cc.pl[2 * (pb + t) + 1];
                P.inlier[pb + q] = 1;
            }
        }
    }
    if (tid == 0) {
        p.tr.n_matched_pt[b] = total;
        p.tr.n_inliers_pt[b] = total;
    }
}

template <int CELL>
__device__ __forceinline__ void knn2_lds(const uint32_t* q, const uint32_t* T, int nt, int& i0, int& d0, int& d1) {
    int dist0 = 2147483647, dist1 = 2147483647, idx0 = -1;
    for (int j = 0; j < nt; ++j) {
        const int d = hamming8<CELL>(q, T + 8 * j);
        if (d < dist1) {
            if (dist0 > d) { dist1 = dist0; dist0 = d; idx0 = j; }
            else { dist1 = d; }
        }
    }
    i0 = idx0; d0 = dist0; d1 = dist1;
}

__device__ int hist_rank_c(const int* h, int r) {
    int c = 0;
    for (int v = 0; v <= 256; ++v) { c += h[v]; if (c > r) return v; }
    return 256;
}

// dynamic LDS: dp[cap*8] dc[cap*8] u32 | i12 d0 d1 i21 [cap] | h12[260] h0[260] | misc[64]
__global__ void __launch_bounds__(512) k_cross_lines(KParams p) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int b = blockIdx.x;
    const int cap = p.kl_cap;
    uint32_t* dp = (uint32_t*)smem;
    uint32_t* dc = dp + cap * 8;
    int* i12 = (int*)(dc + cap * 8);
    int* d012 = i12 + cap;
    int* d112 = d012 + cap;
    int* i21 = d112 + cap;
    int* h12 = i21 + cap;
    int* h0 = h12 + 260;
    int* misc = h0 + 260;
    const int tid = threadIdx.x;
    const int Sl = p.prev.ls.n[b], Sc = p.curr.ls.n[b];
    int total = 0;
    if (Sl >= 2 && Sc >= 2) {   // empty lists: skipped by the reference; 1 row: U4 guard
        DevLines& P = p.prev.ls;
        DevLines& Cc = p.curr.ls;
        const size_t pb = (size_t)b * cap;
        for (int i = tid; i < Sl * 2; i += blockDim.x) reinterpret_cast<uint4*>(dp)[i] = reinterpret_cast<const uint4*>(P.desc + pb * 32)[i];
        for (int i = tid; i < Sc * 2; i += blockDim.x) reinterpret_cast<uint4*>(dc)[i] = reinterpret_cast<const uint4*>(Cc.desc + pb * 32)[i];
        for (int i = tid; i < 520; i += blockDim.x) h12[i] = 0;
        __syncthreads();
        for (int i = tid; i < Sl; i += blockDim.x) {
            int a, d0, d1;
            knn2_lds<1>(dp + 8 * i, dc, Sc, a, d0, d1);
            i12[i] = a; d012[i] = d0; d112[i] = d1;
            atomicAdd(&h12[d1 - d0], 1);
            atomicAdd(&h0[d0], 1);
        }
        for (int j = tid; j < Sc; j += blockDim.x) {
            int a, d0, d1;
            knn2_lds<1>(dc + 8 * j, dp, Sl, a, d0, d1);
            i21[j] = a;
        }
        __syncthreads();
        if (tid == 0) {
            const int v = hist_rank_c(h12, Sl / 2);
            reinterpret_cast<double*>(misc + 16)[0] = (1.4826 * (double)(float)v) * p.cfg.desc_th_l;
            const int k = min(p.cfg.max_line_match_num, Sl) - 1;
            reinterpret_cast<double*>(misc + 16)[1] = (double)(float)hist_rank_c(h0, k);
        }
        __syncthreads();
        const double nn12 = reinterpret_cast<double*>(misc + 16)[0];
        const double budget = reinterpret_cast<double*>(misc + 16)[1];
        const int cap_m = p.cfg.max_line_match_num;
        int off = 0;
        for (int c0 = 0; c0 < Sl; c0 += 512) {
            const int i = c0 + tid;
            int acc = 0, t = 0;
            if (i < Sl) {
                t = i12[i];
                const int rl = i21[t];
                const bool over = (double)(float)d012[i] > 1.2 * budget;
                const double dist_12 = (double)((float)d112[i] - (float)d012[i]);
                acc = (!over && i == rl && dist_12 > nn12) ? 1 : 0;
            }
            int tot;
            const int rank = off + block_exclusive_scan<512>(acc, misc, &tot);
            if (acc && rank < cap_m) {
                const size_t qi = pb + i, qt = pb + t;
                P.sdisp_obs[qi] = Cc.sdisp[qt];
                P.edisp_obs[qi] = Cc.edisp[qt];
                P.spl_obs[2 * qi] = Cc.spl[2 * qt]; P.spl_obs[2 * qi + 1] = Cc.spl[2 * qt + 1];
                P.epl_obs[2 * qi] = Cc.epl[2 * qt]; P.epl_obs[2 * qi + 1] = Cc.epl[2 * qt + 1];
                for (int k = 0; k < 3; ++k) P.le_obs[3 * qi + k] = Cc.le[3 * qt + k];
                P.inlier[qi] = 1;
                p.tr.matched_ls[(size_t)b * p.mls_cap + rank] = i;
                Cc.idx[qt] = P.idx[qi];
            }
            off += tot;
            if (off >= cap_m) break;
        }
        total = off < cap_m ? off : cap_m;
    }
    if (tid == 0) {
        p.tr.n_matched_ls[b] = total;
        p.tr.n_inliers_ls[b] = total;
        p.tr.n_inliers[b] = p.tr.n_inliers_pt[b] + total;
    }
}

hipError_t launch_cross_points(const KParams& p, hipStream_t s) {
    const size_t lds = (size_t)p.kp_cap * 16 + 32 * 8 + (size_t)p.kp_cap * 4 + 64 * 4;
    hipLaunchKernelGGL(k_cross_points, dim3(p.B), dim3(1024), lds, s, p);
    return hipGetLastError();
}

hipError_t launch_cross_lines(const KParams& p, hipStream_t s) {
    const size_t lds = (size_t)p.kl_cap * 64 + (size_t)p.kl_cap * 16 + 520 * 4 + 64 * 4;
    hipLaunchKernelGGL(k_cross_lines, dim3(p.B), dim3(512), lds, s, p);
    return hipGetLastError();
}

}  // namespace gfpl
