// k_kf.hip — keyframe consumers of the tracking kernels.
//
//  k_kf_gate : MapHandler::lookForCommonMatches, keyframe-pair stage
//              (src/mapHandler.cpp:199-470): after the two knn-2 launches
//              (k_knn2m, shared with gfpl_knn2_hamming), one workgroup applies
//              the mutual-best test, the ratio / lineDescriptorMAD test and the
//              chi-square reprojection gate of kf0's feature under DT, and
//              compacts the accepted (kf0, kf1) rows in kf0 order.
// Keyframe-rate work (one launch per keyframe pair): latency, not throughput.
#include "gfpl_kernels.hpp"

namespace gfpl {

struct Mat16 { double v[16]; };

template <int BLOCK>
__global__ void __launch_bounds__(BLOCK) k_kf_gate(KfGate g) {
    __shared__ int hist[257];
    __shared__ int scan[BLOCK / 64 + 1];
    __shared__ double th_s;
    const int tid = threadIdx.x;
    const int n0 = g.n0;
    // DT = inverse_se3(kf1->T_kf_w) * kf0->T_kf_w (src/mapHandler.cpp:196), per thread
    double Ti[16], DT[16];
    inverse_se3(g.T1, Ti);
    if (g.map) {
#pragma unroll
        for (int i = 0; i < 16; ++i) DT[i] = Ti[i];   // Twf (src/mapHandler.cpp:202)
    } else {
        mat4_mul(Ti, g.T0, DT);
    }
    double th = 0.0;
    if (g.lines) {
        // lineDescriptorMAD(lmatches_12).nn12 (src/stereoFrame.cpp:1287-1313, ledger U1):
        // the (d1 - d0) deviations are integers in [0, 256]; the element at sorted rank
        // n0 / 2 comes from a 257-bin histogram
        for (int i = tid; i < 257; i += BLOCK) hist[i] = 0;
        __syncthreads();
        for (int i = tid; i < n0; i += BLOCK) {
            const float v = fabsf((float)((double)(g.d12[2 * i + 1] - g.d12[2 * i]) - 0.0));
            atomicAdd(&hist[min((int)v, 256)], 1);
        }
        __syncthreads();
        if (tid == 0) {
            const int k = n0 / 2;
            int cum = 0, med = 256;
            for (int v = 0; v < 257; ++v) {
                cum += hist[v];
                if (cum > k) { med = v; break; }
            }
            th_s = (1.4826 * (double)(float)med) * g.desc_th_l;   // :366 nn12_mad * descThL
        }
        __syncthreads();
        th = th_s;
    }
    const double chi = sqrt(7.815);
    int off = 0;
    for (int c0 = 0; c0 < n0; c0 += BLOCK) {
        const int q = c0 + tid;
        int flag = 0, t = 0;
        if (q < n0) {
            t = g.i12[2 * q];
            const int rl = g.i21[2 * t];
            const int row = g.loc ? g.loc[q] : q;
            if (g.map) {
                // local-map stage (:571-595 points, :708-733 lines)
                if (!g.lines) {
                    const double dist_12 = (double)(g.d12[2 * q] / g.d12[2 * q + 1]);
                    if (q == rl && dist_12 <= g.max_ratio_12_p) {
                        double Pf[3], uv[2];
                        se3_apply(DT, g.P0 + (size_t)g.p_stride * row, Pf);
                        if (Pf[2] > 0.0) {
                            projection(g.cam, Pf, uv);
                            const double ex = uv[0] - g.pl1[2 * t], ey = uv[1] - g.pl1[2 * t + 1];
                            flag = sqrt(ex * ex + ey * ey) < g.epip_p;
                        }
                    }
                } else {
                    const double dist_12 = (double)(g.d12[2 * q + 1] - g.d12[2 * q]);
                    if (q == rl && dist_12 > th) {
                        double sc[3], ec[3], su[2], eu[2];
                        se3_apply(DT, g.P0 + (size_t)g.p_stride * row, sc);
                        projection(g.cam, sc, su);
                        se3_apply(DT, g.eP0 + (size_t)g.p_stride * row, ec);
                        projection(g.cam, ec, eu);
                        if (sc[2] > 0.0 && ec[2] > 0.0) {
                            const double* l = g.le1 + 3 * t;
                            const double e0 = (l[0] * su[0] + l[1] * su[1]) + l[2];
                            const double e1 = (l[0] * eu[0] + l[1] * eu[1]) + l[2];
                            flag = e0 < g.epip_l && e1 < g.epip_l;   // signed, as the reference
                        }
                    }
                }
            } else if (!g.lines) {
                // points (:243-262): mutual best and d0 / d1 <= maxRatio12P (float division)
                const double dist_12 = (double)(g.d12[2 * q] / g.d12[2 * q + 1]);
                if (q == rl && dist_12 <= g.max_ratio_12_p) {
                    double Pc[3], uv[2];
                    se3_apply(DT, g.P0 + 3 * q, Pc);
                    projection(g.cam, Pc, uv);
                    const double ex = uv[0] - g.pl1[2 * t], ey = uv[1] - g.pl1[2 * t + 1];
                    const double err = sqrt(ex * ex + ey * ey) * sqrt(g.sigma2_0[q]);
                    flag = err < chi;
                }
            } else {
                // lines (:369-392): mutual best and d1 - d0 > nn12 threshold
                const double dist_12 = (double)(g.d12[2 * q + 1] - g.d12[2 * q]);
                if (q == rl && dist_12 > th) {
                    double sc[3], ec[3], su[2], eu[2];
                    se3_apply(DT, g.P0 + 3 * q, sc);
                    projection(g.cam, sc, su);
                    se3_apply(DT, g.eP0 + 3 * q, ec);
                    projection(g.cam, ec, eu);
                    const double* l = g.le0 + 3 * q;
                    const double e0 = (l[0] * su[0] + l[1] * su[1]) + l[2];
                    const double e1 = (l[0] * eu[0] + l[1] * eu[1]) + l[2];
                    flag = sqrt(e0 * e0 + e1 * e1) * sqrt(g.sigma2_0[q]) < chi;
                }
            }
        }
        int tot;
        const int pos = off + block_exclusive_scan<BLOCK>(flag, scan, &tot);
        if (flag) { g.pairs[2 * pos] = g.loc ? g.loc[q] : q; g.pairs[2 * pos + 1] = t; }
        off += tot;
    }
    if (tid == 0) *g.count = off;
}

// map_local_points / map_local_lines selection (src/mapHandler.cpp:472-492, 611-635):
// rows whose projection under Twf = inverse_se3(T1) lies inside the image with z > 0
// (lines: both endpoints), compacted in map order with their descriptors.
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK) k_kf_map_filter(DevCam cam, Mat16 T1, const double* P, int n, int lines,
                                                         int32_t* loc, uint8_t* dout, const uint8_t* din, int* count) {
    __shared__ int scan[BLOCK / 64 + 1];
    double Twf[16];
    inverse_se3(T1.v, Twf);
    auto inside = [&](const double* X) {
        double Pf[3], pf[2];
        se3_apply(Twf, X, Pf);
        projection(cam, Pf, pf);
        return pf[0] > 0 && pf[0] < cam.width && pf[1] > 0 && pf[1] < cam.height && Pf[2] > 0.0;
    };
    int off = 0;
    for (int c0 = 0; c0 < n; c0 += BLOCK) {
        const int i = c0 + threadIdx.x;
        int flag = 0;
        if (i < n) flag = lines ? (inside(P + 6 * (size_t)i) && inside(P + 6 * (size_t)i + 3)) : inside(P + 3 * (size_t)i);
        int tot;
        const int pos = off + block_exclusive_scan<BLOCK>(flag, scan, &tot);
        if (flag) {
            loc[pos] = i;
            const uint4* s4 = reinterpret_cast<const uint4*>(din + 32 * (size_t)i);
            uint4* d4 = reinterpret_cast<uint4*>(dout + 32 * (size_t)pos);
            d4[0] = s4[0]; d4[1] = s4[1];
        }
        off += tot;
    }
    if (threadIdx.x == 0) *count = off;
}

hipError_t launch_kf_map_filter(const DevCam& cam, const double* T1, const double* P, int n, int lines,
                                int32_t* loc, uint8_t* desc_out, const uint8_t* desc_in, int* count, hipStream_t s) {
    Mat16 t;
    for (int i = 0; i < 16; ++i) t.v[i] = T1[i];
    hipLaunchKernelGGL(k_kf_map_filter<1024>, dim3(1), dim3(1024), 0, s, cam, t, P, n, lines, loc, desc_out, desc_in,
                       count);
    return hipGetLastError();
}

hipError_t launch_kf_gate(const KfGate& g, hipStream_t s) {
    hipLaunchKernelGGL(k_kf_gate<1024>, dim3(1), dim3(1024), 0, s, g);
    return hipGetLastError();
}

}  // namespace gfpl
