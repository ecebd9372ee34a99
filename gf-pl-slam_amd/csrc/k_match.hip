// k_match.hip — the descriptor matchers and match-list statistics StereoFrame exposes to its
// callers (MapHandler / KeyFrame), beside the knn-2 of k_stereo.hip:
//
//  k_radius_count / k_radius_rows : cv::BFMatcher::radiusMatch(NORM_HAMMING[2], maxDistance) as
//      StereoFrame::matchPointFeatures_radius / matchLineFeatures_radius call it
//      (src/stereoFrame.cpp:1243-1257): per query row, every train row with distance <= maxDistance
//      (ledger T1), sorted by distance — OpenCV's std::sort on DMatch::operator< leaves equal
//      distances in an unspecified order; here they stay in train order (pinned, ledger T2).
//      One wave per query; the rows are ragged: a count pass sizes them (host scan), the row pass
//      places each match by a counting sort over the <= 257 distances (LDS histogram, then the
//      distinct distances of each 64-row chunk resolved by ballots, in train order).
//  k_match_stats : pointDescriptorMAD / lineDescriptorMAD / *DescriptorBudgetThres
//      (src/stereoFrame.cpp:1259-1341): order statistics of a knn-2 list's distances by an MSB-first
//      radix select over order-preserving float keys (NaN above +inf: ledger U12), one workgroup.
// Keyframe-rate calls (latency, not throughput).
#include "gfpl_kernels.hpp"

namespace gfpl {

// ---------------------------------------------------------------- radius --
template <int CELL>
__global__ void __launch_bounds__(256) k_radius_count(const uint8_t* q, int nq, const uint8_t* t, int nt,
                                                      float radius, int32_t* cnt) {
    const int lane = threadIdx.x & 63;
    const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= nq) return;   // (wave-uniform)
    uint32_t a[8], b[8];
    load_desc(q + 32 * (size_t)qi, a);
    int c = 0;
    for (int j = lane; j < nt; j += 64) {
        load_desc(t + 32 * (size_t)j, b);
        c += ((float)hamming8<CELL>(a, b) <= radius) ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) cnt[qi] = c;
}

template <int CELL>
__global__ void __launch_bounds__(256) k_radius_rows(const uint8_t* q, int nq, const uint8_t* t, int nt, float radius,
                                                     const int32_t* row_off, int32_t* out_idx, float* out_dist) {
    __shared__ int hist[4][257 + 3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int qi = blockIdx.x * 4 + w;
    if (qi >= nq) return;   // (wave-uniform; the waves of a block share no LDS row)
    int* h = hist[w];
    for (int i = lane; i < 257; i += 64) h[i] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t a[8], b[8];
    load_desc(q + 32 * (size_t)qi, a);
    for (int j = lane; j < nt; j += 64) {
        load_desc(t + 32 * (size_t)j, b);
        const int d = hamming8<CELL>(a, b);
        if ((float)d <= radius) atomicAdd(&h[d], 1);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    // exclusive scan of the 257 bins: lane l owns bins [5l, 5l + 5) (lanes 0-51), a wave scan of the partials
    int own[5], tot = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int i = 5 * lane + k;
        own[k] = i < 257 ? h[i] : 0;
        tot += own[k];
    }
    int inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o);
        if (lane >= o) inc += v;
    }
    int run = inc - tot;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int i = 5 * lane + k;
        if (i < 257) h[i] = run;
        run += own[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    const int base = row_off[qi];
    // placement in train order: per 64-row chunk, one ballot per distinct distance present
    for (int j0 = 0; j0 < nt; j0 += 64) {   // (wave-uniform)
        const int j = j0 + lane;
        int d = -1;
        if (j < nt) {
            load_desc(t + 32 * (size_t)j, b);
            const int x = hamming8<CELL>(a, b);
            if ((float)x <= radius) d = x;
        }
        unsigned long long todo = __ballot(d >= 0);
        while (todo) {   // (wave-uniform)
            const int src = __ffsll((long long)todo) - 1;
            const int dv = __shfl(d, src);
            const unsigned long long grp = __ballot(d == dv);
            const int off = h[dv];
            if (d == dv) {
                const int pos = off + __popcll(grp & ((1ull << lane) - 1ull));
                out_idx[base + pos] = j;
                out_dist[base + pos] = (float)dv;
            }
            __builtin_amdgcn_wave_barrier();
            if (lane == src) h[dv] = off + __popcll(grp);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
            todo &= ~grp;
        }
    }
}

hipError_t launch_radius_count(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, float radius,
                               int32_t* cnt, hipStream_t s) {
    const dim3 g((nq + 3) / 4);
    if (cell == 2)
        hipLaunchKernelGGL(k_radius_count<2>, g, dim3(256), 0, s, q, nq, t, nt, radius, cnt);
    else
        hipLaunchKernelGGL(k_radius_count<1>, g, dim3(256), 0, s, q, nq, t, nt, radius, cnt);
    return hipGetLastError();
}

hipError_t launch_radius_rows(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, float radius,
                              const int32_t* row_off, int32_t* idx, float* dist, hipStream_t s) {
    const dim3 g((nq + 3) / 4);
    if (cell == 2)
        hipLaunchKernelGGL(k_radius_rows<2>, g, dim3(256), 0, s, q, nq, t, nt, radius, row_off, idx, dist);
    else
        hipLaunchKernelGGL(k_radius_rows<1>, g, dim3(256), 0, s, q, nq, t, nt, radius, row_off, idx, dist);
    return hipGetLastError();
}

// ----------------------------------------------------------------- stats --
// order-preserving key of a float (NaN above +inf, ledger U12), and back
__device__ __forceinline__ uint32_t fkey(float f) {
    if (f != f) return 0xFFFFFFFFu;
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fval(uint32_t k) {
    if (k == 0xFFFFFFFFu) return __builtin_nanf("");
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// the value of the kind-th statistic's element i (see k_match_stats)
__device__ __forceinline__ float stat_elem(int which, const float* d0, const float* d1, int i, double med) {
    if (which == 0) return d0[i];                                                   // NN distance
    if (which == 1) return fabsf((float)((double)d0[i] - 0.0));                     // |d0 - nn_dist_median| (U1)
    if (which == 2) return fabsf((float)((double)(d1[i] - d0[i]) - 0.0));           // line: |d1 - d0 - 0| (U1)
    if (which == 3) return d0[i] / d1[i];                                           // point: d0 / d1
    return fabsf((float)((double)(d0[i] / d1[i]) - med));                           // point: |d0/d1 - median|
}

// k-th smallest (0-based) of n values of statistic `which`: 4 passes of 8 bits, MSB first
__device__ float select_kth(int which, const float* d0, const float* d1, int n, int k, double med, int* hist,
                            uint32_t* sh) {
    const int tid = threadIdx.x;
    uint32_t prefix = 0, mask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
        hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < n; i += 256) {
            const uint32_t key = fkey(stat_elem(which, d0, d1, i, med));
            if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1);
        }
        __syncthreads();
        if (tid == 0) {
            int acc = 0, bin = 0;
            for (; bin < 256; ++bin) {
                if (acc + hist[bin] > k) break;
                acc += hist[bin];
            }
            sh[0] = (uint32_t)bin;
            sh[1] = (uint32_t)acc;
        }
        __syncthreads();
        prefix |= sh[0] << shift;
        mask |= 255u << shift;
        k -= (int)sh[1];
        __syncthreads();
    }
    return fval(prefix);
}

// out[0] nn_mad, out[1] nn12_mad, out[2] the budget threshold (kind 0 point, 1 line); n >= 1
__global__ void __launch_bounds__(256) k_match_stats(int kind, const float* d0, const float* d1, int n, int max_num,
                                                     double* out) {
    __shared__ int hist[256];
    __shared__ uint32_t sh[2];
    const int mid = n / 2;
    // nn_mad: sort by NN distance, the element at n / 2 of |d0 - 0| (the median first taken is overwritten)
    const float nn = select_kth(1, d0, d1, n, mid, 0.0, hist, sh);
    double nn12;
    if (kind == 1) {
        // lineDescriptorMAD: |d1 - d0 - nn_dist_median| (U1), element n / 2 ascending
        nn12 = 1.4826 * (double)select_kth(2, d0, d1, n, mid, 0.0, hist, sh);
    } else {
        // pointDescriptorMAD: the ratio at n / 2 of the DESCENDING ratio order (compare_descriptor_by_NN12_ratio)
        const double med = (double)select_kth(3, d0, d1, n, n - 1 - mid, 0.0, hist, sh);
        nn12 = 1.4826 * (double)select_kth(4, d0, d1, n, mid, med, hist, sh);
    }
    // *DescriptorBudgetThres: the element at min(max_num, n) - 1 of the NN distances, ascending
    const int bi = (max_num < n ? max_num : n) - 1;
    const float thr = select_kth(0, d0, d1, n, bi < 0 ? 0 : bi, 0.0, hist, sh);
    if (threadIdx.x == 0) {
        out[0] = 1.4826 * (double)nn;
        out[1] = nn12;
        out[2] = (double)thr;
    }
}

hipError_t launch_match_stats(int kind, const float* d0, const float* d1, int n, int max_num, double* out,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_match_stats, dim3(1), dim3(256), 0, s, kind, d0, d1, n, max_num, out);
    return hipGetLastError();
}

}  // namespace gfpl
