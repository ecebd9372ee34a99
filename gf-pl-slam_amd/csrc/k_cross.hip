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
#include "gfpl_knn.hpp"

namespace gfpl {

// Exact spatial grid over the predicted projections of the previous points.
// Cells are CS px squares (CS a power of two >= gate+0.5, so x*inv_cs is exact);
// indices are clamped into the grid, which never separates two values whose
// cells differ by <= 1, so the 3x3 neighbourhood of a current point's cell is a
// superset of every q with |dx|,|dy| <= gate+0.5.  NaN projections (z = 0 or a
// NaN P) pass the reference's `norm() > 10` test, so they sit in a "wild"
// bucket every current point visits.  The visit order is irrelevant: the pick
// is the lexicographic minimum (dist, q), exactly the multimap resolution.
struct CrossGrid {
    int gx, gy, ncell;   // ncell = gx*gy; bucket ncell = wild
    double inv_cs;
};

__device__ __forceinline__ int grid_axis(double v, double inv_cs, int n) {
    double c = floor(v * inv_cs);
    c = c < 0.0 ? 0.0 : (c > (double)(n - 1) ? (double)(n - 1) : c);
    return (int)c;
}

// predictFramePose (src/stereoFrameHandler.cpp:153-157), lane per sequence: curr.Tfw =
// prev.Tfw * prev.DT and its inverse for projectPrev3DPoint.  (Inside k_cross_points the
// 4x4 products and the inverse set its register peak: 20 VGPR + 43 SGPR spills.)
__global__ void __launch_bounds__(64) k_predict_pose(KParams p) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= p.B) return;
    double T[16], A[16], Bm[16], Ti[16];
    for (int i = 0; i < 16; ++i) { A[i] = p.prev.pose.Tfw[16 * b + i]; Bm[i] = p.prev.pose.DT[16 * b + i]; }
    mat4_mul(A, Bm, T);
    mat4_inv(T, Ti);
    for (int i = 0; i < 16; ++i) {
        p.curr.pose.Tfw[16 * b + i] = T[i];
        p.scr.cross_tinv[16 * b + i] = Ti[i];
    }
}

// dynamic LDS: prevT[16] Tinv[16] f64 | (XL) spxy[cap] f64x2 | cnt[ncell+2] start[ncell+2] i32 |
//              sq[cap] i32 | spx[cap] spy[cap] f32 | lastT[cap] i32 | misc[64] i32
// XL: the exact projections of the bucketed points in LDS too (bucket order, beside their float
// copies), so a candidate that passes the float pre-filter reads them from LDS instead of an L2
// round trip ahead of its descriptor load; for capacities whose LDS then leaves two workgroups
// per CU (kp_cap <= 2048)
#ifndef GFPL_CP_WAVES
#define GFPL_CP_WAVES 8   // 2 workgroups / CU (84-B spill; 3.2 -> 2.6 ms measured)
#endif
#ifndef GFPL_CP_XL
#define GFPL_CP_XL 1
#endif
template <bool XL>
__global__ void __launch_bounds__(1024, GFPL_CP_WAVES) k_cross_points(KParams p, CrossGrid G) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int b = blockIdx.x;
    const int cap = p.kp_cap;
    const int NB = G.ncell + 1;   // buckets incl. wild
    double* prevT = (double*)smem;
    double* Tinv = prevT + 16;
    double2* spxy = reinterpret_cast<double2*>(Tinv + 16);   // (XL)
    int* cnt = (int*)(XL ? reinterpret_cast<double*>(spxy + cap) : Tinv + 16);
    int* start = cnt + NB + 1;
    int* sq = start + NB + 1;
    float* spx = (float*)(sq + cap);
    float* spy = spx + cap;
    int* lastT = (int*)(spy + cap);
    int* misc = lastT + cap;
    const int tid = threadIdx.x;
    const int Sp = p.prev.pt.n[b], Sc = p.curr.pt.n[b];
    if (tid < 16) {   // k_predict_pose wrote curr.Tfw and its inverse
        prevT[tid] = p.prev.pose.Tfw[16 * b + tid];
        Tinv[tid] = p.scr.cross_tinv[16 * b + tid];
    }
    for (int i = tid; i < NB; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    int total = 0;
    if (Sp > 0 && Sc > 0) {
        const DevPoints& P = p.prev.pt;
        const DevPoints& Cc = p.curr.pt;
        const size_t pb = (size_t)b * cap;
        double* proj = p.scr.proj + pb * 2;   // exact projections (L2-resident)
        // 1. projectPrev3DPoint (src/stereoFrame.cpp:1550-1570) + bucket histogram
        for (int q = tid; q < Sp; q += blockDim.x) {
            double v[4] = {P.P[3 * (pb + q)], P.P[3 * (pb + q) + 1], P.P[3 * (pb + q) + 2], 1.0};
            mat4_vec(prevT, v, v);
            mat4_vec(Tinv, v, v);
            double uv[2];
            projection(p.cam, v, uv);
            proj[2 * q] = uv[0];
            proj[2 * q + 1] = uv[1];
            int cell = G.ncell;
            if (uv[0] == uv[0] && uv[1] == uv[1])
                cell = grid_axis(uv[1], G.inv_cs, G.gy) * G.gx + grid_axis(uv[0], G.inv_cs, G.gx);
            lastT[q] = cell;
            atomicAdd(&cnt[cell], 1);
        }
        __syncthreads();
        // 2. bucket offsets (exclusive scan over NB counts, chunked by the block)
        int base = 0;
        for (int c0 = 0; c0 < NB; c0 += blockDim.x) {
            const int i = c0 + tid;
            const int v = i < NB ? cnt[i] : 0;
            int tot;
            const int r = base + block_exclusive_scan<1024>(v, misc, &tot);
            if (i < NB) start[i] = r;
            base += tot;
        }
        if (tid == 0) start[NB] = base;
        __syncthreads();
        for (int i = tid; i < NB; i += blockDim.x) cnt[i] = 0;
        __syncthreads();
        // 3. scatter (order inside a bucket is irrelevant, see above)
        for (int q = tid; q < Sp; q += blockDim.x) {
            const int cell = lastT[q];
            const int pos = start[cell] + atomicAdd(&cnt[cell], 1);
            sq[pos] = q;
            const double ux = proj[2 * q], uy = proj[2 * q + 1];
            spx[pos] = (float)ux;
            spy[pos] = (float)uy;
            if (XL) spxy[pos] = make_double2(ux, uy);
            lastT[q] = -1;
        }
        __syncthreads();
        const double gate = p.cfg.proj_gate_px;
        // float pre-filter margin: for |pl| < 1e6 and |proj - pl| <= gate+0.5 the float
        // difference is within 0.2 of the exact one, so gate+1.5 rejects no true candidate.
        const float fpre = (float)(gate + 1.5);
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
                auto consider_at = [&](int q, double ux, double uy) {
                    const double dx = ux - plx, dy = uy - ply;
                    if (sqrt(dx * dx + dy * dy) > gate) return;   // :536 (NaN passes, as in the reference)
                    uint32_t dq[8];
                    load_desc(PD + (size_t)q * 32, dq);
                    const int d = hamming8<1>(dq, dt);
                    if ((float)d <= radius && (d < bestd || (d == bestd && q < bestq))) { bestd = d; bestq = q; }
                };
                auto consider = [&](int q) { consider_at(q, proj[2 * q], proj[2 * q + 1]); };
                auto consider_k = [&](int k) {   // bucketed entry k
                    if (XL) {
                        const double2 u = spxy[k];
                        consider_at(sq[k], u.x, u.y);
                    } else {
                        consider(sq[k]);
                    }
                };
                const bool normal = fabs(plx) < 1e6 && fabs(ply) < 1e6;   // false for NaN too
                if (normal) {
                    const float fx = (float)plx, fy = (float)ply;
                    const int cx = grid_axis(plx, G.inv_cs, G.gx), cy = grid_axis(ply, G.inv_cs, G.gy);
                    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, G.gx - 1);
                    for (int yy = max(cy - 1, 0); yy <= min(cy + 1, G.gy - 1); ++yy) {
                        const int k1 = start[yy * G.gx + x1 + 1];
                        for (int k = start[yy * G.gx + x0]; k < k1; ++k) {
                            if (fabsf(spx[k] - fx) > fpre || fabsf(spy[k] - fy) > fpre) continue;
                            consider_k(k);
                        }
                    }
                    for (int k = start[G.ncell]; k < start[NB]; ++k) consider_k(k);   // wild bucket
                } else {
                    for (int q = 0; q < Sp; ++q) consider(q);   // exact slow path (NaN / huge pl)
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
        p.tr.n_inliers[b] = total + p.tr.n_matched_ls[b];   // counts = list sizes (:700-702)
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


// dynamic LDS: knn LUT | tb[cap*8] u32 (train rows: curr, knn_stage_views) |
//              i12 d0 d1 i21 [cap] | h12[260] h0[260] | misc[64]
#ifndef GFPL_CL_WAVES
#define GFPL_CL_WAVES 1
#endif
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK, GFPL_CL_WAVES) k_cross_lines(KParams p) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int b = blockIdx.x;
    const int cap = p.kl_cap;
    uint32_t* lut = (uint32_t*)smem;   // (first: a compile-time LDS address, folded into the reads' offsets)
    uint32_t* tb = lut + knn_lut_dwords<1>();
    int* i12 = (int*)(tb + cap * 8);
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
        const uint8_t* DP = P.desc + pb * 32;
        const uint8_t* DC = Cc.desc + pb * 32;
        knn_stage_views<1>(tb, cap, DC, Sc);
        for (int i = tid; i < 520; i += blockDim.x) h12[i] = 0;
        for (int j = tid; j < Sc; j += blockDim.x) i21[j] = -1;   // 21 keys (atomicMin)
        knn_lut_fill<1>(lut);
        __syncthreads();
        // 12: prev queries against curr trains, knn-2 on the matrix cores (gfpl_knn.hpp);
        // 21 (curr queries against prev trains, best index only) from the same distance tiles
        knn2_mfma<1, true, true>(tb, cap, Sc, DP, Sl, (uint32_t*)i12, (uint32_t*)d112, lut, (uint32_t*)i21);
        __syncthreads();
        for (int i = tid; i < Sl; i += blockDim.x) {
            const uint32_t k0 = (uint32_t)i12[i], k1 = (uint32_t)d112[i];
            const int d0 = (int)(k0 >> 16), d1 = (int)(k1 >> 16);
            i12[i] = (int)(k0 & 0xFFFFu); d012[i] = d0; d112[i] = d1;
            atomicAdd(&h12[d1 - d0], 1);
            atomicAdd(&h0[d0], 1);
        }
        for (int j = tid; j < Sc; j += blockDim.x) i21[j] = (int)((uint32_t)i21[j] & 0xFFFFu);
        __syncthreads();
        if (tid < 128) {   // (waves 0 and 1: the two medians side by side)
            if (tid < 64) {
                const int v = wave_hist_rank(h12, Sl / 2, 257);
                if (tid == 0) reinterpret_cast<double*>(misc + 16)[0] = (1.4826 * (double)(float)v) * p.cfg.desc_th_l;
            } else {
                const int k = min(p.cfg.max_line_match_num, Sl) - 1;
                const int v = wave_hist_rank(h0, k, 257);
                if (tid == 64) reinterpret_cast<double*>(misc + 16)[1] = (double)(float)v;
            }
        }
        __syncthreads();
        const double nn12 = reinterpret_cast<double*>(misc + 16)[0];
        const double budget = reinterpret_cast<double*>(misc + 16)[1];
        const int cap_m = p.cfg.max_line_match_num;
        int off = 0;
        for (int c0 = 0; c0 < Sl; c0 += BLOCK) {
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
            const int rank = off + block_exclusive_scan<BLOCK>(acc, misc, &tot);
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

CrossGrid cross_grid(const KParams& p) {
    const double pre = p.cfg.proj_gate_px + 0.5;
    int cs = 16;
    CrossGrid G;
    for (;;) {
        G.gx = (p.cam.width + cs - 1) / cs;
        G.gy = (p.cam.height + cs - 1) / cs;
        if ((double)cs >= pre && G.gx * G.gy <= 2048) break;
        cs *= 2;
    }
    G.ncell = G.gx * G.gy;
    G.inv_cs = 1.0 / cs;
    return G;
}

size_t cross_points_lds(const KParams& p, const CrossGrid& G, bool xl) {
    return 32 * 8 + (size_t)(G.ncell + 2) * 8 + (size_t)p.kp_cap * (xl ? 32 : 16) + 64 * 4;
}

hipError_t launch_cross_points(const KParams& p, hipStream_t s) {
    const CrossGrid G = cross_grid(p);
    hipLaunchKernelGGL(k_predict_pose, dim3((p.B + 63) / 64), dim3(64), 0, s, p);
    const size_t lxl = cross_points_lds(p, G, true);
    if (GFPL_CP_XL && p.kp_cap <= 2048 && lxl <= 80 * 1024) {
        static std::atomic<unsigned long long> attr{0};
        const hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(k_cross_points<true>), (int)lxl, &attr);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_cross_points<true>, dim3(p.B), dim3(1024), lxl, s, p, G);
    } else {
        hipLaunchKernelGGL(k_cross_points<false>, dim3(p.B), dim3(1024), cross_points_lds(p, G, false), s, p, G);
    }
    return hipGetLastError();
}

hipError_t launch_cross_lines(const KParams& p, hipStream_t s) {
    const size_t lds = (size_t)p.kl_cap * 32 + (size_t)p.kl_cap * 16 + 520 * 4 + 64 * 4 + 512 * 4;
    // large-capacity LDS layout (one workgroup per CU) and small batches: 16 waves
    if (p.kl_cap > 1024 || p.B <= sp_wide_max_b())
        hipLaunchKernelGGL(k_cross_lines<1024>, dim3(p.B), dim3(1024), lds, s, p);
    else
        hipLaunchKernelGGL(k_cross_lines<512>, dim3(p.B), dim3(512), lds, s, p);
    return hipGetLastError();
}

}  // namespace gfpl
