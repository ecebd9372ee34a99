// k_lsd.hip — LSD line detection on the GPU (detector part):
// line_descriptor::LSDDetectorC::detect(image, keylines, scale, numOctaves, opts)
// (3rdparty/line_descriptor/src/LSDDetector_custom.cpp:218-316) as
// StereoFrame::detectLineFeatures calls it (src/stereoFrame.cpp:1160-1186), over a batch of
// images resident in HBM, the arithmetic pinned as the CPU oracle's ledger S1-S7
// (oracle/gfpl_lsd_oracle.cpp).  Kernels, one launch each for the whole batch:
//  k_lsd_grad      per pixel (lsd.cpp ll_angle, S1): the 2x2 gradient, NOTDEF test, fastAtan2
//                  angle (degrees, float), cos / sin of float(angle) (S3), the image's max norm
//  k_lsd_keys      per pixel: the 64-bit sort element (norm bin << 32 | y << 16 | x), row-major
//  k_lsd_sort      one wave per image: libstdc++ std::sort's permutation (S2).  Introsort's
//                  Hoare partition is restated in parallel: the k-th left stopper swaps with
//                  the k-th right stopper while it lies left of it, so one ballot pass ranks
//                  the stoppers, a 64-ary search finds the crossing, and the swaps run in
//                  parallel; ranges <= 2048 elements finish in LDS; heapsort (depth limit) on
//                  one lane; the final insertion sort is per-leaf (ranges <= 16 never exchange
//                  elements with their neighbours), one leaf per lane
//  k_lsd_grow      one wave per image: the seed loop over the sorted pixels (64 candidates per
//                  ballot), region_grow (lanes 0-8 load a region point's 3x3 neighbours, the
//                  order-dependent angle update runs lane-uniform over them), region2rect /
//                  get_theta (list-ordered sums from lane values), refine and
//                  reduce_region_radius (its swap-with-last removal as a parallel hole/filler
//                  pairing); the used map is an LDS bitmap over the image's defined pixels
//                  (compact indices from k_lsd_grad) when they are at most a quarter of it
//  k_lsd_keylines  one wave per image: checkLineExtremes, the min-length filter (order-
//                  preserving), KeyLine angle / response, and the response std::sort + resize
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdio>

#include "gfpl_kernels.hpp"

namespace gfpl {

// ranges up to CAP elements are sorted in LDS: CAP 1024 (36.5 KB per two-wave workgroup, 4 images
// per CU) for batches up to 4 images per CU, CAP 512 (24 KB, 6 per CU) above (k_lsd_sort<CAP>)
#define LSD_RING 256               // region list entries mirrored in LDS
#define LSD_SMALL 64               // ranges up to this size: one lane runs libstdc++'s serial loop
                                   // (32 / 48 / 64 / 96: 22.2k / 23.5k / 23.7k / 23.1k images/s)
#ifndef GFPL_LSD_PRIO
#define GFPL_LSD_PRIO 1
#endif
#define LSD_CID_MAX 491520         // compact used-map bits at most (60 KB of LDS + the ring)

struct LsdDev {
    int W, H, NP;                  // NP = (W-1)(H-1) sorted pixels
    int n_bins, min_reg_size, seg_cap, kl_cap, n_features;
    double prec, rho, density_th, min_length;
    float4* cs_tab;                // [1021][1021] per (gx, gy) in +-510: float cos / sin of float(angle)
                                   // (a pixel joining a region) and of the double angle (a seed)
    float2* scs;                   // [n][W*H] a defined pixel's seed (cos, sin): cs_tab.zw
    float* ang;                    // [n][W*H] px.x alone (k_lsd_keys' neighbour reads)
    float4* px;                    // [n][W*H] per pixel: fastAtan2 degrees (-1 = NOTDEF), cos and
                                   // sin of float(angle), gx (low 16) | gy (high 16) as bits
    unsigned long long* maxg;      // [n] bits of the max norm of defined pixels
    uint64_t* keys;                // [n][NP]
    int* lpos;                     // [n][NP] partition scratch
    int* rpos;                     // [n][NP]
    uint32_t* reg;                 // [n][W*H] region list
    uint32_t* tmp;                 // [n][W*H] region scratch
    uint32_t* cid;                 // [n][W*H] a defined pixel's position in the sorted keys (k_lsd_sort):
                                   // its bit in the compact used map
    int* ndef;                     // [n] the sorted keys with a bin >= B0 (every defined pixel; k_lsd_sort)
    int cid_cap;                   // compact used-map bits (LDS): images with more defined
                                   // pixels grow with the HBM byte map
    uint8_t* used_g;               // [n][W*H] used map of the images above cid_cap
    float4* segs;                  // [n][seg_cap]
    int* nseg;                     // [n]
    float* kl_tmp;                 // [n][seg_cap][6]  filtered keylines (sx sy ex ey angle response)
    uint64_t* rkeys;               // [n][seg_cap] response sort elements
    int* rl;                       // [n][seg_cap]
    int* rr;                       // [n][seg_cap]
    int* err;                      // bit 0 segment overflow, bit 1 keyline overflow
};

namespace {

constexpr double kPi = 3.1415926535897932384626433832795;
constexpr double k32Pi = (3 * kPi) / 2;
constexpr double k2Pi = 2 * kPi;
constexpr double kDeg2Rad = kPi / 180;

__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// global-memory writes of one lane read by others of the same workgroup: a workgroup-scope
// fence (the workgroup's waves share the CU's write-through L1; an agent-scope fence would
// write back / invalidate the L2 every time)
__device__ __forceinline__ void mem_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
__device__ __forceinline__ int below(unsigned long long m) { return __popcll(m & ((1ull << lane_id()) - 1ull)); }
__device__ __forceinline__ double rl_d(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ float rl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int rl_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double wmax(double v) {
    for (int o = 32; o; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wmin(double v) {
    for (int o = 32; o; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

// O4: cv::fastAtan2 (degrees)
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI), p3 = -0.3258083974640975f * (float)(180 / M_PI),
                p5 = 0.1555786518463281f * (float)(180 / M_PI), p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = __fdiv_rn(ay, ax + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = __fdiv_rn(ax, ay + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// S4: fdlibm s_atan.c / e_atan2.c (finite arguments), + - * / only
__device__ double fd_atan(double x) {
    const double atanhi[] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                             1.57079632679489655800e+00};
    const double atanlo[] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                             6.12323399573676603587e-17};
    const double aT[] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                         -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                         6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                         -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    const int hx = __double2hiint(x);
    const int ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    if (ix < 0x3fdc0000) {
        if (ix < 0x3e200000) return x;
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
            else { id = 3; x = -1.0 / x; }
        }
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}
__device__ double fd_atan2(double y, double x) {
    const double pi_o_2 = 1.5707963267948965580e+00, pi = 3.1415926535897931160e+00,
                 pi_lo = 1.2246467991473531772e-16, tiny = 1.0e-300;
    const int hx = __double2hiint(x), hy = __double2hiint(y);
    const int ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const unsigned lx = (unsigned)__double2loint(x), ly = (unsigned)__double2loint(y);
    if ((((unsigned)hx - 0x3ff00000u) | lx) == 0) return fd_atan(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (((unsigned)iy | ly) == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (((unsigned)ix | lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0;
    else z = fd_atan(fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

__device__ __forceinline__ double angle_diff_signed(double a, double b) {
    double diff = a - b;
    while (diff <= -kPi) diff += k2Pi;
    while (diff > kPi) diff -= k2Pi;
    return diff;
}

// ------------------------------------------------------------- std::sort (S2) --
// comp(a, b) = key(a) > key(b): the descending order of the high 32 bits
__device__ __forceinline__ uint32_t skey(uint64_t e) { return (uint32_t)(e >> 32); }

template <bool LDS>
__device__ __forceinline__ void ssync() {
    if (LDS) lds_sync();
    else mem_sync();
}

// libstdc++ __adjust_heap / __push_heap (one lane)
__device__ void adjust_heap(uint64_t* a, int hole, int len, uint64_t value) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (skey(a[second]) > skey(a[second - 1])) second--;
        a[hole] = a[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[hole] = a[second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && skey(a[parent]) > skey(value)) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = value;
}
// __partial_sort(first, last, last) = __make_heap + __sort_heap
__device__ void heap_sort(uint64_t* a, int len) {
    if (len >= 2) {
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap(a, parent, len, a[parent]);
            if (parent == 0) break;
        }
    }
    while (len > 1) {
        --len;
        const uint64_t v = a[len];
        a[len] = a[0];
        adjust_heap(a, 0, len, v);
    }
}

// __unguarded_partition_pivot(a + f, a + l) by the wave; returns the cut
template <bool LDS, typename IT, int CH = (LDS ? 4 : 16), int SW = (LDS ? 4 : 8)>
__device__ int partition_pivot(uint64_t* a, int f, int l, IT* Lp, IT* Rp, uint32_t* pko = nullptr) {
    const int lane = lane_id();
    const int mid = f + (l - f) / 2;
    // __move_median_to_first(f, f + 1, mid, l - 1)
    const uint32_t ka = skey(a[f + 1]), kb = skey(a[mid]), kc = skey(a[l - 1]);
    int sel;
    if (ka > kb) sel = kb > kc ? mid : (ka > kc ? l - 1 : f + 1);
    else sel = ka > kc ? f + 1 : (kb > kc ? l - 1 : mid);
    const uint64_t pv = a[sel], old = a[f];
    ssync<LDS>();
    if (lane == 0) {
        a[sel] = old;
        a[f] = pv;
    }
    ssync<LDS>();
    const uint32_t pk = skey(pv);
    if (pko) *pko = pk;
    // __unguarded_partition(f + 1, l, f): the stoppers of both scans, ranked
    int cl = 0, cr = 0;   // CH: chunks' loads in flight
    for (int base = f + 1; base < l; base += 64 * CH) {
        uint32_t k4[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int pos = base + 64 * c + lane;
            k4[c] = pos < l ? skey(a[pos]) : 0;
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int pos = base + 64 * c + lane;
            const bool v = pos < l;
            const bool isl = v && k4[c] <= pk, isr = v && k4[c] >= pk;
            const unsigned long long ml = __ballot(isl), mr = __ballot(isr);
            if (isl) Lp[cl + below(ml)] = (IT)pos;
            if (isr) Rp[cr + below(mr)] = (IT)pos;
            cl += __popcll(ml);
            cr += __popcll(mr);
        }
    }
    ssync<LDS>();
    // K = #k with L[k] < R[k] (L ascending, R[k] = Rp[cr - 1 - k] descending): 64-ary search
    int lo = 0, hi = min(cl, cr);
    while (hi > lo) {
        const int step = (hi - lo + 63) >> 6;
        const int k = lo + lane * step;
        const bool inr = k < hi;
        const bool p = inr && Lp[k] < Rp[cr - 1 - k];
        const int t = __popcll(__ballot(p)), nv = __popcll(__ballot(inr));
        if (step == 1 || t == 0) {
            lo += t * step;   // t == 0: K = lo
            break;
        }
        const int nlo = lo + (t - 1) * step + 1;
        hi = t < nv ? lo + t * step : hi;
        lo = nlo;
    }
    const int K = lo;
    for (int base = 0; base < K; base += 64 * SW) {
        int pl[SW], pr[SW];
        uint64_t x[SW], y[SW];
#pragma unroll
        for (int c = 0; c < SW; ++c) {
            const int k = base + 64 * c + lane;
            if (k < K) {
                pl[c] = Lp[k];
                pr[c] = Rp[cr - 1 - k];
            }
        }
#pragma unroll
        for (int c = 0; c < SW; ++c)
            if (base + 64 * c + lane < K) {
                x[c] = a[pl[c]];
                y[c] = a[pr[c]];
            }
#pragma unroll
        for (int c = 0; c < SW; ++c)
            if (base + 64 * c + lane < K) {
                a[pl[c]] = y[c];
                a[pr[c]] = x[c];
            }
    }
    const int cL = K < cl ? Lp[K] : INT_MAX;
    const int cR = K >= 1 ? Rp[cr - K] : INT_MAX;
    ssync<LDS>();
    return min(cL, cR);
}

template <int CAP>
struct SortLds {
    uint64_t buf[CAP];
    uint16_t lp[CAP], rp[CAP];
    int stk[3 * 64];
    int small[3 * 64];
    int lstk[64 * 3 * 3];   // per-lane stacks of lane_introsort (depth <= 3, see there)
};

// libstdc++'s __introsort_loop + final insertion sort of one range [f, l) of an LDS array by
// one lane (ranges <= LSD_SMALL; the lanes of a wave sort disjoint ranges).  The larger part
// of each partition is pushed and the smaller one continued (ranges are independent, so the
// order they are finished in does not change the result): a range stacked at depth i is at most
// 128 / 2^(i-1) elements and only ranges > 16 are partitioned, so the stack stays <= 3 deep.
__device__ void lane_introsort(uint64_t* a, int f, int l, int d, int* st) {
    const int F0 = f, L0 = l;
    int sp = 0;
    for (;;) {
        while (l - f > 16) {
            if (d == 0) {
                heap_sort(a + f, l - f);
                break;
            }
            --d;
            const int mid = f + (l - f) / 2;
            const uint32_t ka = skey(a[f + 1]), kb = skey(a[mid]), kc = skey(a[l - 1]);
            int sel;
            if (ka > kb) sel = kb > kc ? mid : (ka > kc ? l - 1 : f + 1);
            else sel = ka > kc ? f + 1 : (kb > kc ? l - 1 : mid);
            const uint64_t pv = a[sel];
            a[sel] = a[f];
            a[f] = pv;
            const uint32_t pk = skey(pv);
            int first = f + 1, last = l;
            for (;;) {
                while (skey(a[first]) > pk) ++first;
                --last;
                while (pk > skey(a[last])) --last;
                if (!(first < last)) break;
                const uint64_t t = a[first];
                a[first] = a[last];
                a[last] = t;
                ++first;
            }
            const int cut = first;
            // push the larger part (if it needs work), continue with the smaller one: every
            // stacked range is at least twice the current one: from <= 64 elements (LSD_SMALL) the stack
            // holds <= 3 ranges (64 -> 32 -> 16 stops)
            if (cut - f >= l - cut) {
                if (cut - f > 16) { st[3 * sp] = f; st[3 * sp + 1] = cut; st[3 * sp + 2] = d; ++sp; }
                f = cut;
            } else {
                if (l - cut > 16) { st[3 * sp] = cut; st[3 * sp + 1] = l; st[3 * sp + 2] = d; ++sp; }
                l = cut;
            }
        }
        if (sp == 0) break;
        --sp;
        f = st[3 * sp]; l = st[3 * sp + 1]; d = st[3 * sp + 2];
    }
    for (int i = F0 + 1; i < L0; ++i) {   // stable: equals the final insertion sort here
        const uint64_t v = a[i];
        int j = i;
        while (j > F0 && skey(v) > skey(a[j - 1])) {
            a[j] = a[j - 1];
            --j;
        }
        a[j] = v;
    }
}

template <int CAP>
__device__ void flush_small(uint64_t* a, SortLds<CAP>& S, int& ns) {
    const int lane = lane_id();
    if (ns == 0) return;
    lds_sync();
    if (lane < ns) lane_introsort(a, S.small[3 * lane], S.small[3 * lane + 1], S.small[3 * lane + 2], S.lstk + 9 * lane);
    lds_sync();
    ns = 0;
}

// the final insertion sort, one leaf (<= 16 elements, disjoint) per lane
template <bool LDS>
__device__ void flush_leaves(uint64_t* a, int* leaf, int& nleaf) {
    const int lane = lane_id();
    if (nleaf == 0) return;
    ssync<LDS>();
    if (lane < nleaf) {
        const int f = leaf[2 * lane], n = leaf[2 * lane + 1];
        for (int i = 1; i < n; ++i) {
            const uint64_t v = a[f + i];
            int j = i;
            while (j > 0 && skey(v) > skey(a[f + j - 1])) {
                a[f + j] = a[f + j - 1];
                --j;
            }
            a[f + j] = v;
        }
    }
    ssync<LDS>();
    nleaf = 0;
}

template <bool LDS>
__device__ void add_leaf(uint64_t* a, int* leaf, int& nleaf, int f, int l) {
    if (l - f < 2) return;
    if (lane_id() == 0) {
        leaf[2 * nleaf] = f;
        leaf[2 * nleaf + 1] = l - f;
    }
    lds_sync();
    if (++nleaf == 64) flush_leaves<LDS>(a, leaf, nleaf);
}

// __introsort_loop over [0, n) of an LDS array with the given depth budget, then the
// final insertion sort of its leaves.  B0 > 0: a right part whose pivot key is below B0 holds
// only keys below B0 and is left unsorted (see mw_sort)
template <int CAP>
__device__ void introsort_lds(uint64_t* a, int n, int depth, SortLds<CAP>& S, uint32_t B0 = 0) {
    const int lane = lane_id();
    int* stk = S.stk;
    int ns = 0;
    if (lane == 0) {
        stk[0] = 0;
        stk[1] = n;
        stk[2] = depth;
    }
    lds_sync();
    int sp = 1;
    while (sp > 0) {
        --sp;
        int f = stk[3 * sp], l = stk[3 * sp + 1], d = stk[3 * sp + 2];
        bool done = false;
        while (l - f > LSD_SMALL) {
            if (d == 0) {
                if (lane == 0) heap_sort(a + f, l - f);
                lds_sync();
                done = true;
                break;
            }
            --d;
            uint32_t pk;
            const int cut = partition_pivot<true>(a, f, l, S.lp, S.rp, &pk);
            if (pk >= B0) {
                if (lane == 0) {
                    stk[3 * sp] = cut;
                    stk[3 * sp + 1] = l;
                    stk[3 * sp + 2] = d;
                }
                lds_sync();
                ++sp;
            }
            l = cut;
        }
        if (!done && l - f > 1) {
            if (lane == 0) {
                S.small[3 * ns] = f;
                S.small[3 * ns + 1] = l;
                S.small[3 * ns + 2] = d;
            }
            lds_sync();
            if (++ns == 64) flush_small(a, S, ns);
        }
    }
    flush_small(a, S, ns);
}

}  // namespace

// the global-memory sort keeps its stack and leaves in the lower half of SortLds' small
// arrays while a nested LDS sort runs: give the nested call its own copies
template <int CAP>
struct SortLdsPair {
    SortLds<CAP> inner;
    int stk[3 * 64];
    int leaf[2 * 64];
};

namespace {
// std::sort of a[0, n) by descending key (S2), the wave of the calling workgroup
template <int CAP>
__device__ void wave_sort(uint64_t* a, int n, int* Lp, int* Rp, SortLdsPair<CAP>& P) {
    if (n < 2) return;
    const int depth = 2 * (31 - __clz(n));
    if (n <= CAP) {
        const int lane = lane_id();
#pragma unroll 8
        for (int i = lane; i < n; i += 64) P.inner.buf[i] = a[i];
        lds_sync();
        introsort_lds(P.inner.buf, n, depth, P.inner);
        for (int i = lane; i < n; i += 64) a[i] = P.inner.buf[i];
        mem_sync();
        return;
    }
    // outer loop in global memory with its own stack / leaf arrays
    SortLds<CAP>& S = P.inner;
    const int lane = lane_id();
    int* stk = P.stk;
    int* leaf = P.leaf;
    int nleaf = 0;
    if (lane == 0) {
        stk[0] = 0;
        stk[1] = n;
        stk[2] = depth;
    }
    lds_sync();
    int sp = 1;
    while (sp > 0) {
        --sp;
        int f = stk[3 * sp], l = stk[3 * sp + 1], d = stk[3 * sp + 2];
        bool done = false;
        while (l - f > 16) {
            if (l - f <= CAP) {
                const int m = l - f;
#pragma unroll 8
                for (int i = lane; i < m; i += 64) S.buf[i] = a[f + i];
                lds_sync();
                introsort_lds(S.buf, m, d, S);
                for (int i = lane; i < m; i += 64) a[f + i] = S.buf[i];
                mem_sync();
                done = true;
                break;
            }
            if (d == 0) {
                if (lane == 0) heap_sort(a + f, l - f);
                mem_sync();
                done = true;
                break;
            }
            --d;
            const int cut = partition_pivot<false>(a, f, l, Lp, Rp);
            if (lane == 0) {
                stk[3 * sp] = cut;
                stk[3 * sp + 1] = l;
                stk[3 * sp + 2] = d;
            }
            lds_sync();
            ++sp;
            l = cut;
        }
        if (!done) add_leaf<false>(a, leaf, nleaf, f, l);
    }
    flush_leaves<false>(a, leaf, nleaf);
}

// ---- std::sort of one image's pixels by the NW waves of a workgroup (k_lsd_sort) ----
// Introsort's recursion tree has independent subtrees: whichever wave partitions or finishes a
// range, every element ends where libstdc++ puts it.  The waves share the pending ranges through
// a LIFO queue in LDS (a lock word; the queue only holds range bounds, the elements stay in HBM):
// a wave pops a range and walks its introsort_loop spine — while it is > CAP it partitions it in
// HBM (its stoppers go to Lp / Rp at the range's own offset, so concurrent partitions never share
// scratch) and pushes the right part; a range <= CAP is sorted in the wave's own LDS buffer; a
// spent depth budget heap-sorts; leaves (<= 16) are collected for the per-leaf insertion sort.
#ifndef LSD_SORT_WAVES
#define LSD_SORT_WAVES 2
#endif
#ifndef LSD_SORT_CAP
#define LSD_SORT_CAP 1024    // 2 waves x ~17 KB + the queue: four images' workgroups per CU
#endif
#define LSD_QCAP 192         // shared queue entries (a full queue spills to the wave's own stack)
// __unguarded_partition_pivot(a + f, a + l) of a range in HBM by one wave, as Hoare's two scans
// in rounds of up to BT stopper pairs: the left scan gathers the next BT left stoppers (key <=
// pivot) in position order, the right scan the next BT right stoppers (key >= pivot) from the
// right, both staged (position and element) in the wave's LDS sort buffer; the pairs with the
// left stopper still left of its right partner swap (they are a prefix), and a full round moves
// both scans past the swapped positions, which the next round never reads — every scan reads
// elements as the serial algorithm leaves them, and no stopper list goes to HBM.  The cut is
// partition_pivot's: min(next left stopper, last swapped right stopper).
template <int CAP>
__device__ int partition_hoare(uint64_t* a, int f, int l, SortLds<CAP>& S, uint32_t& pko) {
    constexpr int BT = CAP / 2, CH = 16;
    const int lane = lane_id();
    const int mid = f + (l - f) / 2;
    const uint32_t ka = skey(a[f + 1]), kb = skey(a[mid]), kc = skey(a[l - 1]);
    int sel;
    if (ka > kb) sel = kb > kc ? mid : (ka > kc ? l - 1 : f + 1);
    else sel = ka > kc ? f + 1 : (kb > kc ? l - 1 : mid);
    const uint64_t pv = a[sel], old = a[f];
    mem_sync();
    if (lane == 0) {
        a[sel] = old;
        a[f] = pv;
    }
    mem_sync();
    const uint32_t pk = skey(pv);
    pko = pk;
    uint64_t* LV = S.buf;
    uint64_t* RV = S.buf + BT;
    uint32_t* LP = reinterpret_cast<uint32_t*>(S.lp);   // lp | rp: 4 CAP bytes = 2 BT positions
    uint32_t* RP = LP + BT;
    int lnext = f + 1, rnext = l - 1;   // next positions the scans read
    int lbound = l, rbound = f;         // the left scan stays below lbound, the right one above rbound
    for (;;) {
        int nL = 0, nR = 0;
        // both scans advance together: each step issues CH chunks per side before ranking either
        for (int pl = lnext, pr = rnext;;) {
            const bool gl = nL < BT && pl < lbound, gr = nR < BT && pr > rbound;   // (uniform)
            if (!gl && !gr) break;
            uint64_t vl[CH], vr[CH];
            if (gl) {
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    const int pos = pl + 64 * c + lane;
                    vl[c] = pos < lbound ? a[pos] : 0;
                }
            }
            if (gr) {
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    const int pos = pr - 64 * c - lane;
                    vr[c] = pos > rbound ? a[pos] : 0;
                }
            }
            if (gl) {
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    const int pos = pl + 64 * c + lane;
                    const bool st = pos < lbound && skey(vl[c]) <= pk;
                    const unsigned long long m = __ballot(st);
                    const int r = nL + below(m);
                    if (st && r < BT) { LP[r] = (uint32_t)pos; LV[r] = vl[c]; }
                    nL += __popcll(m);
                }
                pl += 64 * CH;
            }
            if (gr) {
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    const int pos = pr - 64 * c - lane;
                    const bool st = pos > rbound && skey(vr[c]) >= pk;
                    const unsigned long long m = __ballot(st);
                    const int r = nR + below(m);
                    if (st && r < BT) { RP[r] = (uint32_t)pos; RV[r] = vr[c]; }
                    nR += __popcll(m);
                }
                pr -= 64 * CH;
            }
        }
        nL = min(nL, BT);
        nR = min(nR, BT);
        lds_sync();
        const int np = min(nL, nR);
        int kb = 0;   // pairs with L[k] < R[k]: a prefix of the round's ranks
        for (int k0 = 0; k0 < np; k0 += 64) {
            const int k = k0 + lane;
            kb += __popcll(__ballot(k < np && LP[k] < RP[k]));
        }
        for (int k = lane; k < kb; k += 64) {
            a[LP[k]] = RV[k];
            a[RP[k]] = LV[k];
        }
        if (kb == BT) {   // (both scans gathered BT stoppers, every pair swapped)
            rbound = (int)LP[BT - 1];
            lbound = (int)RP[BT - 1];
            lnext = rbound + 1;
            rnext = lbound - 1;
            lds_sync();
            continue;
        }
        // the scans have crossed: L[K] is the next left stopper if this round gathered it (else
        // the left scan reached lbound: L[K] lies beyond the last swapped right stopper and is
        // not the min)
        const int cL = kb < nL ? (int)LP[kb] : INT_MAX;
        const int cR = kb >= 1 ? (int)RP[kb - 1] : (lbound < l ? lbound : INT_MAX);
        mem_sync();
        return min(cL, cR);
    }
}

template <int CAP, int NW>
struct SortLdsMW {
    SortLds<CAP> w[NW];
    int leaf[NW][2 * 64];
    int own[NW][3 * 40];     // per-wave overflow stack (depth budget <= 2 log2 n <= 40)
    int lock, qn, busy;
    int q[3 * LSD_QCAP];
};

__device__ __forceinline__ void q_lock(int* lk) {
    int e = 0;
    while (!__hip_atomic_compare_exchange_strong(lk, &e, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
        e = 0;
        __builtin_amdgcn_s_sleep(1);
    }
}
__device__ __forceinline__ void q_unlock(int* lk) {
    __hip_atomic_store(lk, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// the queue counters are read outside the lock too: relaxed atomics (written under the lock)
__device__ __forceinline__ int q_get(int* v) { return __hip_atomic_load(v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void q_set(int* v, int x) { __hip_atomic_store(v, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// B0 > 0 (k_lsd_sort): only the order of the keys >= B0 is read (the seed scan stops at the
// first key below B0: an undefined pixel), so a right part [cut, l) whose pivot key is below B0
// — all of its keys are <= the pivot's — is not sorted further.  Every other range is
// partitioned exactly as libstdc++ does, and the skipped ranges lie after every key >= B0, so
// the keys >= B0 end in std::sort's permutation.  B0 = 0 sorts everything (the test hook).
template <int CAP, int NW>
__device__ __forceinline__ void mw_sort(uint64_t* a, int n, int* Lp, int* Rp, SortLdsMW<CAP, NW>& M,
                                        uint32_t B0 = 0) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        M.lock = 0;
        M.busy = 0;
        M.qn = n > 1 ? 1 : 0;
        M.q[0] = 0;
        M.q[1] = n;
        M.q[2] = n > 1 ? 2 * (31 - __clz(n)) : 0;
    }
    __syncthreads();
    SortLds<CAP>& S = M.w[w];
    int* leaf = M.leaf[w];
    int* own = M.own[w];
    int nleaf = 0, nown = 0;
    int held = 0;   // this wave counts in M.busy (a popped range or its spilled parts are pending)
    for (;;) {
        int f, l, d;
        if (nown > 0) {
            --nown;
            f = own[3 * nown]; l = own[3 * nown + 1]; d = own[3 * nown + 2];
        } else {
            int st = 0;   // 1: a range, 2: every range is done, 0: wait for a push
            int qf = 0, ql = 0, qd = 0;
            // an idle wave peeks at the counters and takes the lock only when there is a range
            // to pop or every wave may be done (idle waves polling under the lock starved the
            // working waves' pushes)
            if (lane == 0 && (held || q_get(&M.qn) > 0 || q_get(&M.busy) == 0)) {
                q_lock(&M.lock);
                int busy = q_get(&M.busy) - held;
                const int qn = q_get(&M.qn);
                if (qn > 0) {
                    const int k = qn - 1;
                    qf = M.q[3 * k]; ql = M.q[3 * k + 1]; qd = M.q[3 * k + 2];
                    q_set(&M.qn, k);
                    ++busy;
                    st = 1;
                } else if (busy == 0) {
                    st = 2;
                }
                q_set(&M.busy, busy);
                q_unlock(&M.lock);
            }
            st = __builtin_amdgcn_readfirstlane(st);
            held = st == 1;
            if (st == 2) break;
            if (st == 0) {
                __builtin_amdgcn_s_sleep(8);
                continue;
            }
            f = __builtin_amdgcn_readfirstlane(qf);
            l = __builtin_amdgcn_readfirstlane(ql);
            d = __builtin_amdgcn_readfirstlane(qd);
            mem_sync();   // acquire: the elements as the partitioning wave left them
        }
        for (;;) {    // one introsort_loop spine
            const int m = l - f;
            if (m <= 16) {
                add_leaf<false>(a, leaf, nleaf, f, l);
                break;
            }
            if (m <= CAP) {
#pragma unroll 4
                for (int i = lane; i < m; i += 64) S.buf[i] = a[f + i];
                lds_sync();
                introsort_lds(S.buf, m, d, S, B0);
                for (int i = lane; i < m; i += 64) a[f + i] = S.buf[i];
                mem_sync();
                break;
            }
            if (d == 0) {
                if (lane == 0) heap_sort(a + f, m);
                mem_sync();
                break;
            }
            --d;
            // (partition_pivot ends with a fence: its swaps are visible to the wave that pops [cut, l))
            uint32_t pk;
            const int cut = partition_hoare(a, f, l, S, pk);
            if (pk < B0) {
                // [cut, l): keys below B0 only, left unsorted
            } else if (l - cut > 16) {
                int pushed = 0;
                if (lane == 0) {
                    q_lock(&M.lock);
                    const int k = q_get(&M.qn);
                    if (k < LSD_QCAP) {
                        M.q[3 * k] = cut; M.q[3 * k + 1] = l; M.q[3 * k + 2] = d;
                        q_set(&M.qn, k + 1);
                        pushed = 1;
                    }
                    q_unlock(&M.lock);
                }
                if (!__builtin_amdgcn_readfirstlane(pushed)) {   // queue full: keep it on the own stack
                    own[3 * nown] = cut; own[3 * nown + 1] = l; own[3 * nown + 2] = d;
                    ++nown;
                }
            } else {
                add_leaf<false>(a, leaf, nleaf, cut, l);
            }
            l = cut;
        }
    }
    flush_leaves<false>(a, leaf, nleaf);
}
}  // namespace

// ------------------------------------------------------------------ ll_angle --
#define LSD_GRAD_ROWS 64   // rows per workgroup (16 passes of 4): one max-norm atomic per 4096 px
__global__ void __launch_bounds__(256) k_lsd_grad(LsdDev o, const uint8_t* images) {
    __shared__ unsigned long long wmaxv[4];
    const int img = blockIdx.z;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int W = o.W, H = o.H;
    const uint8_t* I = images + (size_t)img * W * H;
    unsigned long long b = 0;   // bits of the max norm of defined pixels (norm >= 0 orders like its bits)
    for (int r = 0; r < LSD_GRAD_ROWS; r += 4) {
        const int y = blockIdx.y * LSD_GRAD_ROWS + r + (threadIdx.x >> 6);
        if (x >= W || y >= H) continue;
        const size_t p = (size_t)img * W * H + (size_t)y * W + x;
        float a = -1.0f;
        uint32_t g = 0;
        float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
        if (x < W - 1 && y < H - 1) {
            const int DA = (int)I[(size_t)(y + 1) * W + x + 1] - (int)I[(size_t)y * W + x];
            const int BC = (int)I[(size_t)y * W + x + 1] - (int)I[(size_t)(y + 1) * W + x];
            const int gx = DA + BC, gy = DA - BC;
            g = (uint32_t)(uint16_t)(int16_t)gx | ((uint32_t)(uint16_t)(int16_t)gy << 16);
            const double norm = sqrt((double)(gx * gx + gy * gy) / 4.0);
            if (norm > o.rho) {
                a = fast_atan2((float)gx, (float)-gy);
                cs = o.cs_tab[(gx + 510) * 1021 + (gy + 510)];   // S3, tabulated per (gx, gy)
                const unsigned long long nb = (unsigned long long)__double_as_longlong(norm);
                b = nb > b ? nb : b;
            }
        }
        o.px[p] = make_float4(a, cs.x, cs.y, __uint_as_float(g));
        o.ang[p] = a;
        if (a >= 0.0f) o.scs[p] = make_float2(cs.z, cs.w);
    }
    for (int off = 32; off; off >>= 1) {
        const unsigned long long t = __shfl_xor(b, off);
        b = t > b ? t : b;
    }
    if ((threadIdx.x & 63) == 0) wmaxv[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wmaxv[0];
        for (int w = 1; w < 4; ++w) m = wmaxv[w] > m ? wmaxv[w] : m;
        if (m) atomicMax(&o.maxg[img], m);
    }
}

// S3 for every gradient an 8-bit image can give: the cos / sin of float(angle) depend on
// (gx, gy) only, so the f64 fdlibm evaluations run once per detector, not per pixel
__global__ void __launch_bounds__(256) k_lsd_cs_table(float4* tab) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 1021 * 1021) return;
    const int gx = i / 1021 - 510, gy = i % 1021 - 510;
    const float a = fast_atan2((float)gx, (float)-gy);
    const double ad = (double)a * kDeg2Rad;
    const double af = (double)(float)ad;   // float(angle)
    // region_grow's seed sums: cos / sin of the double angle itself (no float rounding)
    tab[i] = make_float4((float)det_cos(af), (float)det_sin(af), (float)det_cos(ad), (float)det_sin(ad));
}

// one wave per 64 pixels of a row (4 rows per workgroup, no index division); the gradient
// is recomputed from the image bytes (S1: the same integers, hence the same norm and bin as
// k_lsd_grad) instead of read back from the 16-B records, and the angle comes from `ang`
__global__ void __launch_bounds__(256) k_lsd_keys(LsdDev o, const uint8_t* images) {
    const int img = blockIdx.z;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int W = o.W, H = o.H, W1 = W - 1;
    if (x >= W1 || y >= H - 1) return;
    const uint8_t* I = images + (size_t)img * W * H + (size_t)y * W + x;
    const int DA = (int)I[W + 1] - (int)I[0];
    const int BC = (int)I[1] - (int)I[W];
    const int gx = DA + BC, gy = DA - BC;
    const double mg = __longlong_as_double((long long)o.maxg[img]);
    const double bin_coef = (mg > 0) ? (double)(o.n_bins - 1) / mg : 0;
    const double norm = sqrt((double)(gx * gx + gy * gy) / 4.0);
    const int bin = (int)(norm * bin_coef);
    const float* A = o.ang + (size_t)img * W * H;
    const float ac = A[(size_t)y * W + x];
    // bit 31 (above y): a defined pixel none of whose 8 neighbours is defined and aligned with
    // its angle — region_grow from it as a seed stops at the seed (isAligned against the seed's
    // own angle, lsd.cpp), so k_lsd_grow only marks it used (a one-pixel region never reaches
    // min_reg_size >= 2).  The sort compares bin only (skey), the payload bits ride along.
    // The 8 tests run unconditionally (clamped reads, selects): no per-neighbour branches.
    // Each test is taken in float degrees first (|ac - at| wrapped past 270 against the
    // threshold prec in degrees, both within 1e-4 degrees of the double quantities); only a
    // lane with a difference within 1e-3 degrees of the threshold repeats its tests in double
    // as isAligned does.  The 8 tests run unconditionally (clamped reads, selects).
    uint32_t iso = 0;
    if (__any(ac >= 0.0f) && o.min_reg_size > 1) {
        const float pdeg = (float)(o.prec / kDeg2Rad);
        float at[8];
        bool ok[8];
#pragma unroll
        for (int t = 0, k = 0; t < 9; ++t) {
            if (t == 4) continue;
            const int xx = x + t % 3 - 1, yy = y + t / 3 - 1;
            ok[k] = xx >= 0 && yy >= 0 && xx < W && yy < H;
            at[k] = A[(size_t)min(max(yy, 0), H - 1) * W + min(max(xx, 0), W - 1)];
            ++k;
        }
        // (the float wrap at 270 may differ from the double one at 3 pi / 2 only where both
        // 270 and 90 degrees are unaligned: thresholds of 80 degrees and more take the double tests)
        const bool fast = pdeg < 80.0f;
        bool any = false, amb = false;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool v = ok[k] && at[k] >= 0.0f;
            float d = fabsf(ac - at[k]);
            d = d > 270.0f ? fabsf(d - 360.0f) : d;
            any = any || (fast && v && d < pdeg - 1e-3f);
            amb = amb || (v && (!fast || fabsf(d - pdeg) <= 1e-3f));
        }
        if (__any(amb && !any && ac >= 0.0f)) {
            if (amb && !any) {
                const double ra = (double)ac * kDeg2Rad;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    double nt = ra - (double)at[k] * kDeg2Rad;
                    if (nt < 0) nt = -nt;
                    double nw = nt - k2Pi;
                    if (nw < 0) nw = -nw;
                    nt = (nt > k32Pi) ? nw : nt;
                    any = any || (ok[k] && at[k] >= 0.0f && nt <= o.prec);
                }
            }
        }
        iso = (ac >= 0.0f && !any) ? 1u : 0u;
    }
    o.keys[(size_t)img * o.NP + (size_t)y * W1 + x] =
        ((uint64_t)(uint32_t)bin << 32) | (iso << 31) | ((uint32_t)y << 16) | (uint32_t)x;
}

// CAP: LSD_SORT_CAP (36.5 KB per workgroup, four images per CU) for batches up to four images per
// CU; half of it (24 KB, six per CU) for larger batches, whose images would otherwise run in two
// rounds of four per CU (the ranges between the capacities partition in HBM instead of LDS)
template <int CAP>
__global__ void __launch_bounds__(64 * LSD_SORT_WAVES) __attribute__((amdgpu_waves_per_eu(LSD_SORT_WAVES))) k_lsd_sort(LsdDev o) {
    __shared__ SortLdsMW<CAP, LSD_SORT_WAVES> S;
    const size_t img = blockIdx.x;
    // B0 as lsd_image computes it (the bins of k_lsd_keys)
    const double mg = __longlong_as_double((long long)o.maxg[img]);
    const double bin_coef = (mg > 0) ? (double)(o.n_bins - 1) / mg : 0;
    const uint32_t B0 = (uint32_t)(int)(o.rho * bin_coef);
    mw_sort(o.keys + img * o.NP, o.NP, o.lpos + img * o.NP, o.rpos + img * o.NP, S, B0);
    // the compact indices of the used map (k_lsd_grow_lds): a pixel's position in the sorted
    // prefix of keys >= B0 — every defined pixel is there (norm > rho gives a bin >= B0), the
    // sort leaves that prefix first and in order, and everything after it is below B0
    __shared__ int pfx;
    __syncthreads();
    const uint64_t* a = o.keys + img * o.NP;
    if (threadIdx.x == 0) {
        int lo = 0, hi = o.NP;   // the first position with a bin below B0
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((uint32_t)(a[mid] >> 32) >= B0) lo = mid + 1;
            else hi = mid;
        }
        pfx = lo;
        o.ndef[img] = lo;
    }
    __syncthreads();
    uint32_t* cid = o.cid + img * (size_t)o.W * o.H;
    for (int i = threadIdx.x; i < pfx; i += blockDim.x) {
        const uint64_t e = a[i];
        cid[(int)((e >> 16) & 0x7fff) * o.W + (int)(e & 0xffff)] = (uint32_t)i;
    }
}

// ---------------------------------------------------------------- the regions --
namespace {

// The used map of one image: LU — an LDS bitmap over the image's defined pixels, indexed by
// their compact index c (only defined pixels are ever used: seeds and aligned neighbours), so
// a VGA image needs ~3 KB instead of a 38 KB bitmap over every pixel; !LU — an HBM byte map
// by pixel (images with more than cid_cap defined pixels)
template <bool LU>
struct Used {
    uint32_t* bits;   // LDS bitmap (LU)
    uint8_t* g;       // global byte map (!LU)
    int W;
    __device__ __forceinline__ bool get(int x, int y, uint32_t c) const {
        if (LU) return (bits[c >> 5] >> (c & 31)) & 1u;
        return g[y * W + x] != 0;
    }
    __device__ __forceinline__ void set1(int x, int y, uint32_t c) const {   // one lane
        if (LU) atomicOr(&bits[c >> 5], 1u << (c & 31));
        else g[y * W + x] = 1;
    }
    __device__ __forceinline__ void clr(int x, int y, uint32_t c) const {    // any lanes
        if (LU) atomicAnd(&bits[c >> 5], ~(1u << (c & 31)));
        else g[y * W + x] = 0;
    }
    __device__ __forceinline__ void sync() const {
        if (LU) lds_sync();
        else mem_sync();
    }
};

struct Rect { double x1, y1, x2, y2, width; };

struct Img {
    const float4* px;
    const uint32_t* cid;
    uint32_t* reg;
    uint32_t* tmp;
    uint32_t* ring;   // LDS
    int W, H;
};

__device__ __forceinline__ double modgrad(const Img& I, int x, int y) {
    const uint32_t g = __float_as_uint(I.px[y * I.W + x].w);
    const int gx = (int16_t)(g & 0xffff), gy = (int16_t)(g >> 16);
    return sqrt((double)(gx * gx + gy * gy) / 4.0);
}

// region_grow (lsd.cpp): returns the region size; the points in push order are in the LDS
// ring and, once the region nears LSD_RING points (in_hbm), in the HBM list as well: a region
// that stays small never stores to HBM (a store would hold up the next wait for a load, the
// prefetch of the next seed's neighbourhood included); ring_to_hbm() completes the list for
// the callers that read it (region2rect / refine), which fence before reading.
// has_pre: lanes 0-24 of `pre` hold the records of the seed's 5x5 neighbourhood (lane
// 5 (dy + 2) + dx + 2) and lane 25 of `pcs` its seed (cos, sin): the first two batches (the
// seed and the pixels it adds) need no HBM round trip.  (seed_deg: the seed's angle record)
// (scid: the seed's compact index; pre_c: lanes 0-24's compact indices with `pre`)
template <bool LU>
__device__ int region_grow(const Img& I, const Used<LU>& U, int sx, int sy, uint32_t scid, float seed_deg,
                           double prec, double& reg_angle, bool& in_hbm, bool has_pre = false,
                           float4 pre = float4{}, float2 pcs = float2{}, uint32_t pre_c = 0) {
    const int lane = lane_id();
    int n = 0;
    reg_angle = (double)seed_deg * kDeg2Rad;
    float sumdx, sumdy;   // S3
    if (has_pre) {
        sumdx = rl_f(pcs.x, 25);
        sumdy = rl_f(pcs.y, 25);
    } else {
        sumdx = (float)det_cos(reg_angle);
        sumdy = (float)det_sin(reg_angle);
    }
    const uint32_t s = ((uint32_t)sy << 16) | (uint32_t)sx;
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    lds_u32* ring = (lds_u32*)(uintptr_t)(uint32_t)(uintptr_t)I.ring;
    if (lane == 0) {
        ring[0] = s;
        U.set1(sx, sy, scid);
    }
    n = 1;
    bool glob = false;   // (uniform) new points go to the HBM list too
    U.sync();
    lds_sync();
    // the region list is expanded in batches of up to 7 points: lanes 9g..9g+8 load point
    // i+g's 3x3 neighbour records in one round trip, then the points are processed in list
    // order, each reading the used map as the earlier points of the batch left it
    const int g = lane / 9, t9 = lane - 9 * g;
    const int dxl = t9 % 3 - 1, dyl = t9 / 3 - 1;
    for (int i = 0; i < n;) {
        const int nb = min(7, n - i);
        int rx = 0, ry = 0, xx = 0, yy = 0;
        bool ok = false;
        uint32_t r = 0;
        if (n - i > LSD_RING) {   // (uniform) the oldest points have left the ring
            mem_sync();
            if (g < nb) {
                const int idx = i + g;
                r = n - idx > LSD_RING ? I.reg[idx] : (uint32_t)ring[idx & (LSD_RING - 1)];
            }
        } else if (g < nb) {
            r = i == 0 ? s : (uint32_t)ring[(i + g) & (LSD_RING - 1)];   // (the first batch is the seed)
        }
        if (g < nb) {
            rx = (int)(r & 0xffff);
            ry = (int)(r >> 16);
            xx = rx + dxl;
            yy = ry + dyl;
            ok = xx >= 0 && yy >= 0 && xx < I.W && yy < I.H;
        }
        float4 q = make_float4(-1.0f, 0.f, 0.f, 0.f);
        uint32_t cq = 0;
        bool inwin = false;
        if (has_pre) {   // (uniform)
            const int ox = xx - sx + 2, oy = yy - sy + 2;
            inwin = ok && ox >= 0 && ox < 5 && oy >= 0 && oy < 5;
            const int src = inwin ? 5 * oy + ox : 0;
            const float4 w = make_float4(__shfl(pre.x, src), __shfl(pre.y, src), __shfl(pre.z, src), __shfl(pre.w, src));
            const uint32_t wc = LU ? (uint32_t)__shfl((int)pre_c, src) : 0u;
            if (inwin) {
                q = w;
                cq = wc;
            }
        }
        if (ok && !inwin) {
            q = I.px[yy * I.W + xx];
            if (LU) cq = I.cid[yy * I.W + xx];
        }
        if (!(q.x >= 0.0f)) cq = 0;   // (an undefined pixel has no index)
        for (int k = 0; k < nb; ++k) {
            if (!glob && n > LSD_RING - 16) {   // <= 9 points join per step: the ring has not wrapped
                for (int e = lane; e < n; e += 64) I.reg[e] = ring[e];
                glob = true;
            }
            const bool av = g == k && ok && q.x >= 0.0f && !U.get(xx, yy, cq);
            unsigned long long m = __ballot(av) >> (9 * k);
            if (!m) continue;
            const int b = 9 * k;
            const int prx = rl_i(rx, b), pry = rl_i(ry, b);
            // isAligned (lsd.cpp) of every pending neighbour against the current reg_angle at
            // once (lane b + t: neighbour t): the first aligned one is the next the serial
            // loop adds, those before it failed against the same angle; the angle then
            // changes and the neighbours after it are tested again (the used map of this
            // point's neighbours does not change meanwhile: they are distinct pixels)
            const double ad = (double)q.x * kDeg2Rad;
            const bool mine = lane >= b && lane < b + 9;
            while (m) {
                double nt = reg_angle - ad;
                if (nt < 0) nt = -nt;
                if (nt > k32Pi) {
                    nt -= k2Pi;
                    if (nt < 0) nt = -nt;
                }
                const unsigned long long ma = (__ballot(mine && nt <= prec) >> b) & m;
                if (!ma) break;
                const int t = __ffsll((long long)ma) - 1;
                m &= ~((2ull << t) - 1ull);
                const int px = prx + t % 3 - 1, py = pry + t / 3 - 1;
                const uint32_t e = ((uint32_t)py << 16) | (uint32_t)px;
                const uint32_t pc = LU ? (uint32_t)rl_i((int)cq, b + t) : 0u;
                if (lane == 0) {
                    U.set1(px, py, pc);
                    if (glob) I.reg[n] = e;
                    ring[n & (LSD_RING - 1)] = e;
                }
                ++n;
                sumdx += rl_f(q.y, b + t);
                sumdy += rl_f(q.z, b + t);
                reg_angle = (double)fast_atan2(sumdy, sumdx) * kDeg2Rad;
            }
            lds_sync();
            if (!LU) mem_sync();
        }
        i += nb;
    }
    in_hbm = glob;
    return n;
}

// the region list of a region_grow that stayed in the ring, copied to HBM (caller fences)
__device__ __forceinline__ void ring_to_hbm(const Img& I, int n, bool in_hbm) {
    if (in_hbm) return;
    for (int e = lane_id(); e < n; e += 64) I.reg[e] = I.ring[e];
}

// region2rect + get_theta (lsd.cpp), sums in list order
__device__ void region2rect(const Img& I, int n, double reg_angle, double prec, Rect& rec) {
    const int lane = lane_id();
    double X = 0, Y = 0, S = 0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        double px = 0, py = 0, w = 0;
        if (i < n) {
            const uint32_t r = I.reg[i];
            const int x = (int)(r & 0xffff), y = (int)(r >> 16);
            w = modgrad(I, x, y);
            px = (double)x * w;
            py = (double)y * w;
        }
        const int m = min(64, n - b);
        for (int t = 0; t < m; ++t) {
            X += rl_d(px, t);
            Y += rl_d(py, t);
            S += rl_d(w, t);
        }
    }
    const double x = X / S, y = Y / S;
    double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        double txx = 0, tyy = 0, txy = 0;
        if (i < n) {
            const uint32_t r = I.reg[i];
            const int rx = (int)(r & 0xffff), ry = (int)(r >> 16);
            const double w = modgrad(I, rx, ry);
            const double dx = (double)rx - x, dy = (double)ry - y;
            txx = dy * dy * w;
            tyy = dx * dx * w;
            txy = dx * dy * w;
        }
        const int m = min(64, n - b);
        for (int t = 0; t < m; ++t) {
            Ixx += rl_d(txx, t);
            Iyy += rl_d(tyy, t);
            Ixy -= rl_d(txy, t);
        }
    }
    const double lambda = 0.5 * (Ixx + Iyy - sqrt((Ixx - Iyy) * (Ixx - Iyy) + 4.0 * Ixy * Ixy));
    double theta = (fabs(Ixx) > fabs(Iyy)) ? (double)fast_atan2((float)(lambda - Ixx), (float)Ixy)
                                           : (double)fast_atan2((float)Ixy, (float)(lambda - Iyy));
    theta *= kDeg2Rad;
    if (fabs(angle_diff_signed(theta, reg_angle)) > prec) theta += kPi;
    const double dx = det_cos(theta), dy = det_sin(theta);
    double lmax = 0, lmin = 0, wmx = 0, wmn = 0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        if (i < n) {
            const uint32_t r = I.reg[i];
            const double rdx = (double)(int)(r & 0xffff) - x, rdy = (double)(int)(r >> 16) - y;
            const double l = rdx * dx + rdy * dy;
            const double w = -rdx * dy + rdy * dx;
            lmax = fmax(lmax, l);
            lmin = fmin(lmin, l);
            wmx = fmax(wmx, w);
            wmn = fmin(wmn, w);
        }
    }
    lmax = wmax(lmax);
    lmin = wmin(lmin);
    wmx = wmax(wmx);
    wmn = wmin(wmn);
    rec.x1 = x + lmin * dx;
    rec.y1 = y + lmin * dy;
    rec.x2 = x + lmax * dx;
    rec.y2 = y + lmax * dy;
    rec.width = wmx - wmn;
    if (rec.width < 1.0) rec.width = 1.0;
}

__device__ __forceinline__ double rdist(const Rect& r) {
    return sqrt((r.x2 - r.x1) * (r.x2 - r.x1) + (r.y2 - r.y1) * (r.y2 - r.y1));
}

// reduce_region_radius (lsd.cpp): each pass's swap-with-last removal = holes (far points
// below the new size, ascending) filled by the kept points above it, descending
template <bool LU>
__device__ bool reduce_region_radius(const Img& I, const Used<LU>& U, int& n, double reg_angle, double prec,
                                     Rect& rec, double density, double density_th) {
    const int lane = lane_id();
    const uint32_t r0 = I.reg[0];
    const double xc = (double)(int)(r0 & 0xffff), yc = (double)(int)(r0 >> 16);
    const double rad1 = (rec.x1 - xc) * (rec.x1 - xc) + (rec.y1 - yc) * (rec.y1 - yc);
    const double rad2 = (rec.x2 - xc) * (rec.x2 - xc) + (rec.y2 - yc) * (rec.y2 - yc);
    double rad_sq = rad1 > rad2 ? rad1 : rad2;
    while (density < density_th) {
        rad_sq *= 0.75 * 0.75;
        // kept count
        int nk = 0;
        for (int b = 0; b < n; b += 64) {
            const int i = b + lane;
            bool far = false;
            if (i < n) {
                const uint32_t r = I.reg[i];
                const double px = (double)(int)(r & 0xffff), py = (double)(int)(r >> 16);
                far = (px - xc) * (px - xc) + (py - yc) * (py - yc) > rad_sq;
                if (far) {
                    const int x = (int)(r & 0xffff), y = (int)(r >> 16);
                    U.clr(x, y, LU ? I.cid[y * I.W + x] : 0u);
                }
            }
            nk += __popcll(__ballot(i < n && !far));
        }
        // fillers: kept points at positions >= nk, rank from the end -> tmp
        int cf = 0;
        for (int b = nk; b < n; b += 64) {
            const int i = b + lane;
            bool keep = false;
            uint32_t r = 0;
            if (i < n) {
                r = I.reg[i];
                const double px = (double)(int)(r & 0xffff), py = (double)(int)(r >> 16);
                keep = !((px - xc) * (px - xc) + (py - yc) * (py - yc) > rad_sq);
            }
            const unsigned long long m = __ballot(keep);
            if (keep) I.tmp[cf + below(m)] = r;
            cf += __popcll(m);
        }
        mem_sync();
        // holes: far points at positions < nk, ascending; hole k takes filler cf - 1 - k
        int ch = 0;
        for (int b = 0; b < nk; b += 64) {
            const int i = b + lane;
            bool far = false;
            if (i < nk) {
                const uint32_t r = I.reg[i];
                const double px = (double)(int)(r & 0xffff), py = (double)(int)(r >> 16);
                far = (px - xc) * (px - xc) + (py - yc) * (py - yc) > rad_sq;
            }
            const unsigned long long m = __ballot(far);
            if (far) I.reg[i] = I.tmp[cf - 1 - (ch + below(m))];
            ch += __popcll(m);
        }
        n = nk;
        mem_sync();
        U.sync();
        if (n < 2) return false;
        region2rect(I, n, reg_angle, prec, rec);
        density = (double)n / (rdist(rec) * rec.width);
    }
    return true;
}

// refine (lsd.cpp, LSD_REFINE_STD)
template <bool LU>
__device__ bool refine(const Img& I, const Used<LU>& U, int& n, double reg_angle, double prec, Rect& rec,
                       double density_th) {
    const int lane = lane_id();
    double density = (double)n / (rdist(rec) * rec.width);
    if (density >= density_th) return true;
    const uint32_t r0 = I.reg[0];
    const int sx = (int)(r0 & 0xffff), sy = (int)(r0 >> 16);
    const double xc = (double)sx, yc = (double)sy;
    const double ang_c = (double)I.px[sy * I.W + sx].x * kDeg2Rad;
    double sum = 0, s_sum = 0;
    int cnt = 0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        double ad = 0;
        bool in = false;
        if (i < n) {
            const uint32_t r = I.reg[i];
            const int x = (int)(r & 0xffff), y = (int)(r >> 16);
            U.clr(x, y, LU ? I.cid[y * I.W + x] : 0u);
            in = sqrt(((double)x - xc) * ((double)x - xc) + ((double)y - yc) * ((double)y - yc)) < rec.width;
            if (in) ad = angle_diff_signed((double)I.px[y * I.W + x].x * kDeg2Rad, ang_c);
        }
        const unsigned long long m = __ballot(in);
        const int c = min(64, n - b);
        for (int t = 0; t < c; ++t) {
            if (!((m >> t) & 1ull)) continue;
            const double v = rl_d(ad, t);
            sum += v;
            s_sum += v * v;
        }
        cnt += __popcll(m);
    }
    U.sync();
    const double mean_angle = sum / (double)cnt;
    const double tau = 2.0 * sqrt((s_sum - 2.0 * mean_angle * sum) / (double)cnt + mean_angle * mean_angle);
    bool in_hbm;
    n = region_grow<LU>(I, U, sx, sy, LU ? I.cid[sy * I.W + sx] : 0u, I.px[sy * I.W + sx].x, tau, reg_angle,
                        in_hbm);
    ring_to_hbm(I, n, in_hbm);
    mem_sync();   // the region list (HBM) is read by every lane next
    if (n < 2) return false;
    region2rect(I, n, reg_angle, prec, rec);
    density = (double)n / (rdist(rec) * rec.width);
    if (density < density_th) return reduce_region_radius<LU>(I, U, n, reg_angle, prec, rec, density, density_th);
    return true;
}

template <bool LU>
__device__ void lsd_image(const LsdDev& o, int img, uint32_t* bits, uint32_t* ring) {
    const int lane = lane_id();
    const size_t off = (size_t)img * o.W * o.H;
    Img I{o.px + off, o.cid + off, o.reg + off, o.tmp + off, ring, o.W, o.H};
    Used<LU> U{bits, o.used_g + off, o.W};
    const uint32_t* cidp = o.cid + off;
    if (LU) {
        const int nw = (o.ndef[img] + 31) >> 5;
        for (int i = lane; i < nw; i += 64) bits[i] = 0;
        lds_sync();
    } else {
        for (int i = lane; i < o.W * o.H; i += 64) U.g[i] = 0;
        mem_sync();
    }
    const uint64_t* keys = o.keys + (size_t)img * o.NP;
    const float* pxf = (const float*)I.px;
    int nseg = 0;
    // software pipeline: chunk c+2's keys and chunk c+1's angles load while chunk c is processed
    uint64_t e1 = lane < o.NP ? keys[lane] : 0;
    float a1 = lane < o.NP ? pxf[4 * ((int)((e1 >> 16) & 0x7fff) * o.W + (int)(e1 & 0xffff))] : -1.0f;
    uint32_t c1 = (LU && lane < o.NP) ? cidp[(int)((e1 >> 16) & 0x7fff) * o.W + (int)(e1 & 0xffff)] : 0u;
    // (a candidate's angle record comes with the scan: a region's first round trip is its
    // seed's neighbourhood)
    uint64_t e2 = 64 + lane < o.NP ? keys[64 + lane] : 0;
    // the keys descend by norm bin and a bin below B0 = (int)(rho * bin_coef) means norm < rho
    // (rounding is monotone), i.e. an undefined pixel, which is never a seed: the scan stops at
    // the first chunk whose leading key is below B0 (the 93% undefined tail is not walked)
    const double mg = __longlong_as_double((long long)o.maxg[img]);
    const double bin_coef = (mg > 0) ? (double)(o.n_bins - 1) / mg : 0;
    const uint32_t B0 = (uint32_t)(int)(o.rho * bin_coef);
#if GFPL_LSD_PRIO
    const int nscan = max(1, o.ndef[img]);   // the seeds scanned: every defined pixel
#endif
    for (int base = 0; base < o.NP; base += 64) {
#if GFPL_LSD_PRIO
        {   // issue priority by progress through the seeds (3 .. 0): the waves of a SIMD keep pace
            const int q = (4 * base) / nscan;
            if (q <= 0) __builtin_amdgcn_s_setprio(3);
            else if (q == 1) __builtin_amdgcn_s_setprio(2);
            else if (q == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
#endif
        const uint64_t e = e1;
        if ((uint32_t)(__builtin_amdgcn_readfirstlane((uint32_t)(e >> 32))) < B0) break;
        int px = (int)(e & 0xffff), py = (int)((e >> 16) & 0x7fff);
        const bool iso = (e >> 31) & 1u;   // (k_lsd_keys)
        const float a0 = a1;
        const uint32_t c0 = a0 >= 0.0f ? c1 : 0u;   // (an undefined pixel has no index)
        e1 = e2;
        a1 = base + 64 + lane < o.NP ? pxf[4 * ((int)((e1 >> 16) & 0x7fff) * o.W + (int)(e1 & 0xffff))] : -1.0f;
        if (LU) c1 = base + 64 + lane < o.NP ? cidp[(int)((e1 >> 16) & 0x7fff) * o.W + (int)(e1 & 0xffff)] : 0u;
        e2 = base + 128 + lane < o.NP ? keys[base + 128 + lane] : 0;
        bool cand = a0 >= 0.0f;
        int pre_j = -1;   // the candidate whose 5x5 records and seed (cos, sin) `pre` holds
        float4 pre = make_float4(-1.0f, 0.f, 0.f, 0.f);
        float2 pcs = make_float2(0.f, 0.f);
        uint32_t pre_c = 0;
        for (;;) {
            const unsigned long long m = __ballot(cand && !U.get(px, py, c0));
            if (!m) break;
            // isolated seeds ahead of the next one that grows become used, in one step
            const unsigned long long mg = m & __ballot(!iso);
            const unsigned long long mi = mg ? m & ((mg & (0ull - mg)) - 1ull) : m;
            if (mi) {
                if ((mi >> lane) & 1ull) {
                    U.set1(px, py, c0);
                    cand = false;
                }
                U.sync();
            }
            if (!mg) break;
            const int j = __ffsll((long long)mg) - 1;
            if (lane <= j) cand = false;
            const int sx = rl_i(px, j), sy = rl_i(py, j);
            // the next candidate's neighbourhood loads while this region grows (records are
            // static; whether it is still a seed is decided from the used map later)
            const bool has_pre = pre_j == j;
            const float4 cur = pre;
            const float2 cur_cs = pcs;
            const uint32_t cur_c = pre_c;
            const unsigned long long m2 = mg & ~((2ull << j) - 1ull);
            pre_j = m2 ? __ffsll((long long)m2) - 1 : -1;
            pre = make_float4(-1.0f, 0.f, 0.f, 0.f);
            if (pre_j >= 0) {   // (separate registers: no wait for one load before the other)
                const int cx = rl_i(px, pre_j), cy = rl_i(py, pre_j);
                const int xx = cx + lane % 5 - 2, yy = cy + lane / 5 - 2;
                if (lane < 25 && xx >= 0 && yy >= 0 && xx < o.W && yy < o.H) {
                    pre = I.px[yy * o.W + xx];
                    if (LU) pre_c = cidp[yy * o.W + xx];
                }
                if (lane == 25) pcs = o.scs[off + (size_t)cy * o.W + cx];
            }
            double reg_angle;
            bool in_hbm;
            int n = region_grow<LU>(I, U, sx, sy, LU ? (uint32_t)rl_i((int)c0, j) : 0u, rl_f(a0, j), o.prec, reg_angle,
                                    in_hbm, has_pre, cur, cur_cs, cur_c);
            if (n < o.min_reg_size) continue;
            ring_to_hbm(I, n, in_hbm);
            mem_sync();   // the region list (HBM) is read by every lane next
            Rect rec;
            region2rect(I, n, reg_angle, o.prec, rec);
            if (!refine<LU>(I, U, n, reg_angle, o.prec, rec, o.density_th)) continue;
            if (lane == 0) {
                if (nseg < o.seg_cap)
                    o.segs[(size_t)img * o.seg_cap + nseg] =
                        make_float4((float)(rec.x1 + 0.5), (float)(rec.y1 + 0.5), (float)(rec.x2 + 0.5),
                                    (float)(rec.y2 + 0.5));
                else
                    atomicOr(o.err, 1);
            }
            ++nseg;
        }
    }
    if (lane == 0) o.nseg[img] = min(nseg, o.seg_cap);
}

}  // namespace

// one wave per image, both launched over the batch: the compact LDS bitmap (cid_cap bits
// after the ring) for the images with at most cid_cap defined pixels, the HBM byte map for the
// others (separate kernels: one holding both paths took 184 VGPRs and a private segment)
__global__ void __launch_bounds__(64) k_lsd_grow_lds(LsdDev o) {
    extern __shared__ uint32_t lds[];
    if (o.ndef[blockIdx.x] > o.cid_cap) return;
    lsd_image<true>(o, blockIdx.x, lds + LSD_RING, lds);
}
__global__ void __launch_bounds__(64) k_lsd_grow_glb(LsdDev o) {
    __shared__ uint32_t ring[LSD_RING];
    if (o.ndef[blockIdx.x] <= o.cid_cap) return;
    lsd_image<false>(o, blockIdx.x, nullptr, ring);
}

// std::sort of one device array (test hook of the S2 restatement)
__global__ void __launch_bounds__(64 * LSD_SORT_WAVES) __attribute__((amdgpu_waves_per_eu(LSD_SORT_WAVES))) k_lsd_sort_one(uint64_t* a, int n, int* lp, int* rp) {
    __shared__ SortLdsMW<LSD_SORT_CAP, LSD_SORT_WAVES> S;
    mw_sort(a, n, lp, rp, S);
}

// ------------------------------------------------------------------ keylines --
// LSDDetector_custom.cpp:266-306 and src/stereoFrame.cpp:1177-1185
__global__ void __launch_bounds__(64) k_lsd_keylines(LsdDev o, gfpl_keyline* kl_out, int* n_kl, float* rsp_out) {
    __shared__ SortLdsPair<1024> S;
    const int img = blockIdx.x, lane = lane_id();
    const int ns = o.nseg[img];
    const float fw = (float)o.W, fh = (float)o.H;
    const float mx = (float)max(o.W, o.H);
    float* kt = o.kl_tmp + (size_t)img * o.seg_cap * 6;
    int m = 0;
    for (int b = 0; b < ns; b += 64) {
        const int i = b + lane;
        bool keep = false;
        float e0 = 0, e1 = 0, e2 = 0, e3 = 0, ang = 0, rsp = 0;
        if (i < ns) {
            const float4 s = o.segs[(size_t)img * o.seg_cap + i];
            e0 = s.x; e1 = s.y; e2 = s.z; e3 = s.w;
            // checkLineExtremes (:78-103)
            if (e0 < 0) e0 = 0;
            if (e0 >= fw) e0 = fw - 1.0f;
            if (e2 < 0) e2 = 0;
            if (e2 >= fw) e2 = fw - 1.0f;
            if (e1 < 0) e1 = 0;
            if (e1 >= fh) e1 = fh - 1.0f;
            if (e3 < 0) e3 = 0;
            if (e3 >= fh) e3 = fh - 1.0f;
            const float d0 = e0 - e2, d1 = e1 - e3;
            const double length = (double)(float)sqrt((double)d0 * (double)d0 + (double)d1 * (double)d1);
            keep = length > o.min_length;
            ang = (float)fd_atan2((double)(e3 - e1), (double)(e2 - e0));   // S4
            rsp = __fdiv_rn((float)length, mx);
        }
        const unsigned long long mk = __ballot(keep);
        if (keep) {
            float* d = kt + 6 * (m + below(mk));
            d[0] = e0; d[1] = e1; d[2] = e2; d[3] = e3; d[4] = ang; d[5] = rsp;
        }
        m += __popcll(mk);
    }
    mem_sync();
    const bool cut = m > o.n_features && o.n_features != 0;
    const int nout = cut ? o.n_features : m;
    if (nout > o.kl_cap) {
        if (lane == 0) {
            atomicOr(o.err, 2);
            n_kl[img] = 0;
        }
        return;
    }
    uint64_t* rk = o.rkeys + (size_t)img * o.seg_cap;
    if (cut) {
        for (int i = lane; i < m; i += 64)
            rk[i] = ((uint64_t)__float_as_uint(kt[6 * i + 5]) << 32) | (uint32_t)i;
        mem_sync();
        wave_sort(rk, m, o.rl + (size_t)img * o.seg_cap, o.rr + (size_t)img * o.seg_cap, S);   // S7
    }
    for (int k = lane; k < nout; k += 64) {
        const int i = cut ? (int)(uint32_t)rk[k] : k;
        const float* d = kt + 6 * i;
        gfpl_keyline q;
        q.sx = d[0]; q.sy = d[1]; q.ex = d[2]; q.ey = d[3]; q.angle = d[4]; q.octave = 0;
        kl_out[(size_t)img * o.kl_cap + k] = q;
        if (rsp_out) rsp_out[(size_t)img * o.kl_cap + k] = d[5];
    }
    if (lane == 0) n_kl[img] = nout;
}

}  // namespace gfpl

// ======================================================================= ABI ==
using namespace gfpl;

struct gfpl_lsd {
    int device = 0;
    hipStream_t stream = nullptr;
    gfpl_ctx* ctx = nullptr;   // counted in while this object lives
    AsyncStatus st;
    int max_images = 0;
    int n_cu = 256;            // compute units of the device (the sort's capacity choice)
    size_t lds_bytes = 0;
    LsdDev d{};
    void* base = nullptr;
};

extern "C" int gfpl_lsd_create(gfpl_ctx* ctx, const gfpl_lsd_params* prm, int width, int height, int max_images,
                               int kl_cap, int seg_cap, gfpl_lsd** out) {
    if (!ctx || !prm || !out || max_images < 1 || kl_cap < 1 || seg_cap < 1 || width < 8 || height < 8 ||
        width > 2048 || height > 2048 || prm->n_bins < 1 || prm->n_features < 0)
        return GFPL_E_INVALID;
    if (prm->refine != 1 || prm->scale != 1.0) return GFPL_E_UNSUPPORTED;
    const int dev = gfpl_ctx_device(ctx);
    if (hipSetDevice(dev) != hipSuccess) return GFPL_E_HIP;
    gfpl_lsd* o = new gfpl_lsd();
    o->device = dev;
    o->stream = (hipStream_t)gfpl_ctx_stream(ctx);
    o->max_images = max_images;
    {
        int cu = 0;
        if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cu > 0) o->n_cu = cu;
    }
    LsdDev& d = o->d;
    d.W = width;
    d.H = height;
    d.NP = (width - 1) * (height - 1);
    d.n_bins = prm->n_bins;
    d.seg_cap = seg_cap;
    d.kl_cap = kl_cap;
    d.n_features = prm->n_features;
    d.density_th = prm->density_th;
    d.min_length = prm->min_length;
    {   // flsd's constants (S5), host libm as the oracle computes them
        const double pi = 3.1415926535897932384626433832795;
        d.prec = pi * prm->ang_th / 180;
        const double p = prm->ang_th / 180;
        d.rho = prm->quant / std::sin(d.prec);
        const double log_nt = 5 * (std::log10((double)width) + std::log10((double)height)) / 2 + std::log10(11.0);
        d.min_reg_size = (int)(size_t)(-log_nt / std::log10(p));
    }
    const size_t px = (size_t)width * height, M = (size_t)max_images, NP = (size_t)d.NP, SC = (size_t)seg_cap;
    // the compact used map covers a quarter of the pixels defined (VGA: 9.6 KB; the scenes
    // measured define 5-8%), so 15 images share a CU's LDS instead of 4 with a full-image bitmap
    d.cid_cap = (int)std::min<size_t>(((px + 3) / 4 + 31) & ~(size_t)31, LSD_CID_MAX);
    o->lds_bytes = (size_t)d.cid_cap / 8 + 4 * LSD_RING;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t b_tab = al(16 * 1021 * 1021), b_px = al(16 * M * px), b_scs = al(8 * M * px), b_ang = al(4 * M * px), b_max = al(8 * M),
                 b_keys = al(8 * M * NP), b_pos = al(4 * M * NP), b_reg = al(4 * M * px),
                 b_used = al(M * px), b_segs = al(16 * M * SC), b_nseg = al(4 * M),
                 b_klt = al(24 * M * SC), b_rk = al(8 * M * SC), b_rl = al(4 * M * SC);
    const size_t total = b_tab + b_px + b_scs + b_ang + b_max + b_keys + 2 * b_pos + 3 * b_reg + b_used + b_segs + 2 * b_nseg +
                         b_klt + b_rk + 2 * b_rl + 256;
    if (hipMalloc(&o->base, total) != hipSuccess) { delete o; return GFPL_E_HIP; }
    char* p = (char*)o->base;
    d.cs_tab = (float4*)p; p += b_tab;
    d.px = (float4*)p; p += b_px;
    d.scs = (float2*)p; p += b_scs;
    d.ang = (float*)p; p += b_ang;
    d.maxg = (unsigned long long*)p; p += b_max;
    d.keys = (uint64_t*)p; p += b_keys;
    d.lpos = (int*)p; p += b_pos;
    d.rpos = (int*)p; p += b_pos;
    d.reg = (uint32_t*)p; p += b_reg;
    d.tmp = (uint32_t*)p; p += b_reg;
    d.cid = (uint32_t*)p; p += b_reg;
    d.used_g = (uint8_t*)p; p += b_used;
    d.segs = (float4*)p; p += b_segs;
    d.nseg = (int*)p; p += b_nseg;
    d.ndef = (int*)p; p += b_nseg;
    d.kl_tmp = (float*)p; p += b_klt;
    d.rkeys = (uint64_t*)p; p += b_rk;
    d.rl = (int*)p; p += b_rl;
    d.rr = (int*)p; p += b_rl;
    d.err = (int*)p;
    if (hipFuncSetAttribute((const void*)k_lsd_grow_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)o->lds_bytes) != hipSuccess) {
        (void)hipFree(o->base);
        delete o;
        return GFPL_E_HIP;
    }
    hipLaunchKernelGGL(k_lsd_cs_table, dim3((1021 * 1021 + 255) / 256), dim3(256), 0, o->stream, d.cs_tab);
    if (hipGetLastError() != hipSuccess || o->st.init(d.err, o->stream) != hipSuccess) {
        o->st.destroy();
        (void)hipFree(o->base);
        delete o;
        return GFPL_E_HIP;
    }
    o->ctx = ctx;
    gfpl_ctx_attach(ctx);
    *out = o;
    return GFPL_OK;
}

extern "C" int gfpl_lsd_sort_desc(gfpl_lsd* o, uint64_t* a, int n) {
    if (!o || !a || n < 0 || n > o->d.NP) return GFPL_E_INVALID;
    if (hipSetDevice(o->device) != hipSuccess) return GFPL_E_HIP;
    hipLaunchKernelGGL(k_lsd_sort_one, dim3(1), dim3(64 * LSD_SORT_WAVES), 0, o->stream, a, n, o->d.lpos, o->d.rpos);
    if (hipGetLastError() != hipSuccess) return GFPL_E_HIP;
    return hipStreamSynchronize(o->stream) == hipSuccess ? GFPL_OK : GFPL_E_HIP;
}

extern "C" int gfpl_lsd_destroy(gfpl_lsd* o) {
    if (!o) return GFPL_E_INVALID;
    (void)hipStreamSynchronize(o->stream);
    o->st.destroy();
    if (o->base) (void)hipFree(o->base);
    gfpl_ctx_detach(o->ctx);
    delete o;
    return GFPL_OK;
}

extern "C" int gfpl_lsd_detect_async(gfpl_lsd* o, const uint8_t* images, int n, gfpl_keyline* keylines, int* n_kl,
                                     float* response) {
    if (!o || !images || n < 1 || n > o->max_images || !keylines || !n_kl) return GFPL_E_INVALID;
    if (hipSetDevice(o->device) != hipSuccess) return GFPL_E_HIP;
    const LsdDev& d = o->d;
    hipStream_t s = o->stream;
    if (hipMemsetAsync(d.maxg, 0, 8 * (size_t)n, s) != hipSuccess ||
        hipMemsetAsync(d.ndef, 0, 4 * (size_t)n, s) != hipSuccess)
        return GFPL_E_HIP;
    hipLaunchKernelGGL(k_lsd_grad, dim3((d.W + 63) / 64, (d.H + LSD_GRAD_ROWS - 1) / LSD_GRAD_ROWS, n), dim3(256), 0, s,
                       d, images);
    hipLaunchKernelGGL(k_lsd_keys, dim3((d.W - 1 + 63) / 64, (d.H - 1 + 3) / 4, n), dim3(256), 0, s, d, images);
    // (a third tier, CAP / 4 at 128 VGPRs so eight images share a CU, measured 56.9k vs 64.8k
    // images/s at 3072: its 12 VGPR spills and the smaller LDS ranges cost more than the
    // residency gained; profiles/r04_y)
    if (n <= 4 * o->n_cu)
        hipLaunchKernelGGL((k_lsd_sort<LSD_SORT_CAP>), dim3(n), dim3(64 * LSD_SORT_WAVES), 0, s, d);
    else
        hipLaunchKernelGGL((k_lsd_sort<LSD_SORT_CAP / 2>), dim3(n), dim3(64 * LSD_SORT_WAVES), 0, s, d);
    hipLaunchKernelGGL(k_lsd_grow_glb, dim3(n), dim3(64), 0, s, d);
    hipLaunchKernelGGL(k_lsd_grow_lds, dim3(n), dim3(64), o->lds_bytes, s, d);
    hipLaunchKernelGGL(k_lsd_keylines, dim3(n), dim3(64), 0, s, d, keylines, n_kl, response);
    if (hipGetLastError() != hipSuccess) return GFPL_E_HIP;
    return o->st.enqueue(s) == hipSuccess ? GFPL_OK : GFPL_E_HIP;
}

extern "C" int gfpl_lsd_status(gfpl_lsd* o) {
    if (!o) return GFPL_E_INVALID;
    int bits = 0;
    if (o->st.wait(o->stream, &bits) != hipSuccess) return GFPL_E_HIP;
    return bits ? GFPL_E_CAPACITY : GFPL_OK;
}

extern "C" int gfpl_lsd_detect(gfpl_lsd* o, const uint8_t* images, int n, gfpl_keyline* keylines, int* n_kl,
                               float* response) {
    const int e = gfpl_lsd_detect_async(o, images, n, keylines, n_kl, response);
    if (e) return e;
    return gfpl_lsd_status(o);
}
