// k_orb.hip — ORB extraction on the GPU: ORB_SLAM2::ORBextractor::
// operator() (src/ORBextractor.cc:1043-1105) over a batch of grey images resident in HBM,
// with the arithmetic of the OpenCV calls it makes pinned as in the CPU oracle (ledger
// O1-O7, oracle/gfpl_orb_oracle.cpp).  Kernels, per launch over all images:
//  k_orb_copy0    level 0 of the pyramid = the image (the pyramid is the caller's array
//                 when it asks for one, so the levels never need a second copy)
//  k_orb_resize   level l from level l-1: cv::resize INTER_LINEAR fixed point (O1)
//                 (ComputePyramid :1107-1132), coefficient tables built on the host
//  k_orb_blur     GaussianBlur 7x7 sigma 2 REFLECT_101 fixed point (O2) of every level,
//                 one 64x32 tile per workgroup through LDS (rows pass, then columns)
//  k_orb_cellfast one wave per 30-px cell of ComputeKeyPointsOctTree (:765-853), all
//                 levels and images in one launch: FAST_t + cornerScore (O3) on the cell's
//                 ROI in LDS, non-max suppression, the minThFAST retry for empty cells,
//                 the keys in cv::FAST's row-major order into the cell's slot
//  k_orb_gather   one workgroup per (image, level): the cells' keys concatenated in cell
//                 order = vToDistributeKeys
//  k_orb_octree   one wave per (image, level): DistributeOctTree (:539-763) with the
//                 node list in LDS (the reference's list order, O6 for ties), the list
//                 bookkeeping in wave-uniform registers and every DivideNode a
//                 wave-parallel stable 4-way partition of the node's keys
//  k_orb_describe two kept keypoints per wave: IC_Angle (:77-104, O4), rBRIEF on the
//                 blurred level (:108-148, O5), the level scale (:1094-1101), output in
//                 the reference's order (level by level, node-list order)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "gfpl_kernels.hpp"
#include "gfpl_orb_pattern.h"

namespace gfpl {

__constant__ int c_orb_pattern[1024];

// everything the ORB kernels read, passed by value (device pointers)
struct OrbLevel {
    int w, h;                        // level image size (ComputePyramid :1111-1112)
    long long off;                   // offset of the level in an image's pyramid
    int minBX, minBY, maxBX, maxBY;  // ComputeKeyPointsOctTree borders (:773-776)
    int nCols, nRows, wCell, hCell;  // its 30-px cells (:781-787)
    int N;                           // mnFeaturesPerLevel (:435-446)
    int nIni;                        // DistributeOctTree initial nodes (:543)
    float hX;                        // their width (:545)
    float scale;                     // mvScaleFactor
};
struct OrbDev {
    int W, H, nlevels, ini_th, min_th;
    int key_cap, sel_cap, node_cap;
    int key_lds;      // levels with up to key_lds keys keep them in the octree's LDS
    long long pyr_stride;            // bytes between the pyramids of two images
    long long blur_stride;           // ... between their blurred copies
    OrbLevel lv[GFPL_MAX_LEVELS];
    const int* xofs[GFPL_MAX_LEVELS];
    const int16_t* alpha[GFPL_MAX_LEVELS];
    const int* yofs[GFPL_MAX_LEVELS];
    const int16_t* beta[GFPL_MAX_LEVELS];
    int xmax[GFPL_MAX_LEVELS];
    int blur_k[7];
    int umax[16];
    uint8_t* pyr;     // [n][pyr_stride] level images (the caller's pyramid array when it asks for one)
    uint8_t* blur;    // [n][blur_stride] their Gaussian blur
    int ncell;        // 30-px cells of all levels of one image
    int cbase[GFPL_MAX_LEVELS + 1];   // first cell of each level
    int ccap;         // key slots per cell (strict 3x3 maxima: <= ceil(w/2) ceil(h/2))
    int patch_cap;    // pixels of one cell's ROI (LDS per wave: ROI and scores u8, candidates u16)
    int cell_waves;   // cells (waves) per k_orb_cellfast workgroup
    uint32_t* ckeys;  // [n][ncell][ccap] the keys of each cell in FAST's row-major order
    int* ccnt;        // [n][ncell]
    uint32_t* keys;   // [n][nlevels][key_cap] vToDistributeKeys (packed)
    uint32_t* tmp;    // [n][nlevels][key_cap] partition scratch
    int* nkeys;       // [n][nlevels]
    uint32_t* sel;    // [n][nlevels][sel_cap] kept keys in node-list order
    int* nsel;        // [n][nlevels]
    int* err;         // bit 0: key capacity, bit 1: node capacity, bit 2: output capacity
};


namespace {

constexpr int kCircleX[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
constexpr int kCircleY[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

// LDS written by some lanes of a wave, then read by others (the wave's DS operations
// complete in order; the clobber keeps the compiler from moving accesses across)
__device__ __forceinline__ void wave_sync_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
#define ORB_MAX_CELLS 4096

__device__ __forceinline__ uint8_t sat_u8(int v) { return (uint8_t)min(max(v, 0), 255); }

// packed key: x (11 bits) | y (11 bits) << 11 | score (8 bits) << 22, coordinates
// relative to (minBorderX, minBorderY) as the reference's vToDistributeKeys
__device__ __forceinline__ uint32_t key_pack(int x, int y, int s) {
    return (uint32_t)x | ((uint32_t)y << 11) | ((uint32_t)s << 22);
}
__device__ __forceinline__ int key_x(uint32_t k) { return (int)(k & 0x7FFu); }
__device__ __forceinline__ int key_y(uint32_t k) { return (int)((k >> 11) & 0x7FFu); }
__device__ __forceinline__ int key_s(uint32_t k) { return (int)(k >> 22); }

}  // namespace

// ------------------------------------------------------------------ pyramid --
__global__ void k_orb_copy0(OrbDev o, const uint8_t* images, int n) {
    const size_t npx = (size_t)o.W * o.H;
    const int img = blockIdx.y;
    const uint8_t* src = images + img * npx;
    uint8_t* dst = o.pyr + img * o.pyr_stride;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {   // 16-B rows of the image, then the tail
        const size_t nv = npx / 16;
        for (size_t i = t0; i < nv; i += nt) reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
        for (size_t i = nv * 16 + t0; i < npx; i += nt) dst[i] = src[i];
    } else {
        for (size_t i = t0; i < npx; i += nt) dst[i] = src[i];
    }
}

// O1: dst(x, y) = ((h(y0, x) b0 + h(y1, x) b1 + 2^21) >> 22), h = exact 11-bit horizontal blend
// RESIZE_ROWS output rows per workgroup, in three phases through LDS:
//  1. the source rows they read (yofs of the first row .. of the last + 1) with aligned dword
//     loads (a row's bytes start at its address & 3 in its LDS row);
//  2. per 4-px column unit, the x tables loaded once, every output row's 4 px from the LDS
//     source bytes into an LDS output row as one dword;
//  3. each output row stored as dwords at 4-B aligned addresses (two LDS dwords funnel-shifted
//     by the row's misalignment), its unaligned head / tail bytes one by one.
// (One pixel per thread from global bytes: 171 us per level at 256 VGA images; this layout with
// 16 / 8 / 4 / 2 rows per workgroup: 95, 63, 62, 74 us — 16 rows left too few waves resident.)
#define RESIZE_ROWS 8
#define RESIZE_T 128
__device__ __forceinline__ uint32_t resize_lds_px(const uint8_t* L0, const uint8_t* L1, int sx, uint32_t al, bool blend,
                                                  int b0, int b1) {
    const int a0 = (int16_t)(al & 0xFFFFu), a1 = (int16_t)(al >> 16);
    const int h0 = blend ? L0[sx] * a0 + L0[sx + 1] * a1 : L0[sx] * 2048;
    const int h1 = blend ? L1[sx] * a0 + L1[sx + 1] * a1 : L1[sx] * 2048;
    return sat_u8((h0 * b0 + h1 * b1 + (1 << 21)) >> 22);
}
__global__ void __launch_bounds__(RESIZE_T) k_orb_resize(OrbDev o, int l) {
    extern __shared__ uint32_t rz_lds[];
    const OrbLevel& d = o.lv[l];
    const OrbLevel& s = o.lv[l - 1];
    const int img = blockIdx.y;
    const uint8_t* S = o.pyr + img * o.pyr_stride + s.off;
    uint8_t* Dl = o.pyr + img * o.pyr_stride + d.off;
    const int* yofs = o.yofs[l];
    const int16_t* beta = o.beta[l];
    const int y0 = blockIdx.x * RESIZE_ROWS;
    const int nr = min(RESIZE_ROWS, d.h - y0);
    const int r_lo = min(max(yofs[y0], 0), s.h - 1);
    const int r_hi = min(max(yofs[y0 + nr - 1] + 1, 0), s.h - 1);
    const int sdw = (s.w + 6) >> 2;   // dwords per source row (any alignment)
    const int odw = (d.w >> 2) + 2;   // dwords per output row (+1 for the funnel shift)
    uint32_t* src = rz_lds;
    uint32_t* out = rz_lds + (r_hi - r_lo + 1) * sdw;
    // 1. source rows
    const int nsrc = (r_hi - r_lo + 1) * sdw;
    for (int i0 = 0; i0 < nsrc; i0 += 8 * RESIZE_T) {   // eight loads per thread in flight
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * RESIZE_T + threadIdx.x;
            if (i < nsrc) {
                const int j = i / sdw, m = i - j * sdw;
                const uintptr_t row = (uintptr_t)(S + (size_t)(r_lo + j) * s.w);
                v[u] = reinterpret_cast<const uint32_t*>(row & ~(uintptr_t)3)[m];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * RESIZE_T + threadIdx.x;
            if (i < nsrc) src[i] = v[u];
        }
    }
    __syncthreads();
    // 2. 4-px units
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(src);
    const uint32_t sh0 = (uint32_t)((uintptr_t)(S + (size_t)r_lo * s.w) & 3u);
    const uint32_t wmod = (uint32_t)s.w & 3u;
    const int* xofs = o.xofs[l];
    const uint32_t* al = reinterpret_cast<const uint32_t*>(o.alpha[l]);   // (alpha0, alpha1) int16 pairs
    const int xmax = o.xmax[l];
    const int nu = (d.w + 3) >> 2;
    for (int k = threadIdx.x; k < nu; k += RESIZE_T) {
        int sx[4];
        uint32_t a4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int x = min(4 * k + i, d.w - 1);   // a short last unit repeats its last pixel
            sx[i] = xofs[x];
            a4[i] = al[x];
        }
#pragma unroll 2
        for (int r = 0; r < nr; ++r) {
            const int sy = yofs[y0 + r];
            const int j0 = min(max(sy, 0), s.h - 1) - r_lo, j1 = min(max(sy + 1, 0), s.h - 1) - r_lo;
            // byte offset of source row j in LDS: its row * 4 sdw + the row address & 3
            const uint8_t* L0 = sb + j0 * 4 * sdw + ((sh0 + (uint32_t)j0 * wmod) & 3u);
            const uint8_t* L1 = sb + j1 * 4 * sdw + ((sh0 + (uint32_t)j1 * wmod) & 3u);
            const int b0 = beta[2 * (y0 + r)], b1 = beta[2 * (y0 + r) + 1];
            uint32_t q[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = resize_lds_px(L0, L1, sx[i], a4[i], 4 * k + i < xmax, b0, b1);
            // packed with v_perm: the shift-or form was selected as v_ashr_pk_u8_i32, whose
            // result's upper half then leaked into bytes 2-3 (measured wrong on gfx950)
            const uint32_t lo = __builtin_amdgcn_perm(q[1], q[0], 0x0C0C0400u);
            const uint32_t hi = __builtin_amdgcn_perm(q[3], q[2], 0x0C0C0400u);
            out[r * odw + k] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
        }
    }
    __syncthreads();
    // 3. aligned stores
    const uint8_t* ob = reinterpret_cast<const uint8_t*>(out);
    const int U = (d.w >> 2) + 2;   // units of a row: head bytes (k = -1), dwords, tail bytes
    for (int i = threadIdx.x; i < nr * U; i += RESIZE_T) {
        const int r = i / U, k = i - r * U - 1;
        uint8_t* D = Dl + (size_t)(y0 + r) * d.w;
        const int lead = (int)((4u - ((uint32_t)(uintptr_t)D & 3u)) & 3u);
        const int nd = (d.w - lead) >> 2;
        if (k > nd) continue;
        if (k < 0 || k == nd) {
            const int xa = k < 0 ? 0 : lead + 4 * nd, xb = k < 0 ? lead : d.w;
            for (int x = xa; x < xb; ++x) D[x] = ob[4 * r * odw + x];
        } else {
            const uint32_t* orow = out + r * odw;
            const int x = lead + 4 * k;   // bytes x .. x + 3 of the output row
            *reinterpret_cast<uint32_t*>(D + x) =
                __builtin_amdgcn_alignbyte(orow[(x >> 2) + 1], orow[x >> 2], (uint32_t)(x & 3));
        }
    }
}

// O2: 7x7 Gaussian, 8-bit integer taps, rows exact, columns (s + 2^15) >> 16.  One 64x32
// tile per workgroup: the (32+6)x(64+6) source bytes (REFLECT_101 at the level's edges:
// levels are >= 38 px, so one reflection suffices), the row pass into LDS, then every
// thread slides the column pass down 8 rows of one column.
#define BLUR_TW 64
#define BLUR_TH 32
__device__ __forceinline__ int refl1(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }
__global__ void __launch_bounds__(256) k_orb_blur(OrbDev o) {
    __shared__ int tile[BLUR_TH + 6][BLUR_TW + 8];   // (dword cells: byte LDS traffic measured slower)
    __shared__ int rows[BLUR_TH + 6][BLUR_TW + 1];
    const int l = blockIdx.z % o.nlevels, img = blockIdx.z / o.nlevels;
    const OrbLevel& L = o.lv[l];
    const int x0 = blockIdx.x * BLUR_TW, y0 = blockIdx.y * BLUR_TH;
    if (x0 >= L.w || y0 >= L.h) return;
    const uint8_t* S = o.pyr + img * o.pyr_stride + L.off;
    const int tx = threadIdx.x & 63, ty0 = threadIdx.x >> 6;
    if (x0 >= 3 && x0 + BLUR_TW + 2 < L.w && y0 >= 3 && y0 + BLUR_TH + 2 < L.h) {
        // interior tile: each source row's 70 bytes as 19 aligned dwords (byte loads bound
        // the border path's memory pipeline), three loads per thread in flight
        constexpr int NDW = 19, NLD = (BLUR_TH + 6) * NDW;
        uint32_t v[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int i = threadIdx.x + 256 * u;
            if (i < NLD) {
                const int r = i / NDW, m = i - r * NDW;
                const uintptr_t a = (uintptr_t)(S + (size_t)(y0 - 3 + r) * L.w + (x0 - 3));
                v[u] = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3)[m];
            }
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int i = threadIdx.x + 256 * u;
            if (i < NLD) {
                const int r = i / NDW, m = i - r * NDW;
                const int sh = (int)((uintptr_t)(S + (size_t)(y0 - 3 + r) * L.w + (x0 - 3)) & 3u);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int c = 4 * m + k - sh;
                    if (c >= 0 && c < BLUR_TW + 6) tile[r][c] = (int)((v[u] >> (8 * k)) & 0xFFu);
                }
            }
        }
    } else {   // 10 rows x (1 or 2) columns per thread, loads in flight before the LDS stores
        const int sx0 = refl1(min(x0 + tx - 3, L.w + 2), L.w);
        const int sx1 = refl1(min(x0 + tx + 61, L.w + 2), L.w);
        uint8_t a[10], b[10];
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int r = ty0 + 4 * q;
            const size_t row = (size_t)refl1(min(y0 + min(r, BLUR_TH + 5) - 3, L.h + 2), L.h) * L.w;
            a[q] = S[row + sx0];
            b[q] = tx < 6 ? S[row + sx1] : 0;
        }
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int r = ty0 + 4 * q;
            if (r < BLUR_TH + 6) {
                tile[r][tx] = a[q];
                if (tx < 6) tile[r][tx + 64] = b[q];
            }
        }
    }
    __syncthreads();
    const int k0 = o.blur_k[0], k1 = o.blur_k[1], k2 = o.blur_k[2], k3 = o.blur_k[3];
    for (int r = ty0; r < BLUR_TH + 6; r += 4) {
        const int* T = &tile[r][tx];
        rows[r][tx] = k0 * (T[0] + T[6]) + k1 * (T[1] + T[5]) + k2 * (T[2] + T[4]) + k3 * T[3];
    }
    __syncthreads();
    uint8_t* D = o.blur + img * o.blur_stride + L.off;
    const int x = x0 + tx;
    if (x >= L.w) return;
    const int r0 = ty0 * 8;
    int w[14];
#pragma unroll
    for (int t = 0; t < 14; ++t) w[t] = rows[r0 + t][tx];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int y = y0 + r0 + q;
        if (y < L.h) {
            const int a = k3 * w[q + 3] + k2 * (w[q + 2] + w[q + 4]) + k1 * (w[q + 1] + w[q + 5]) + k0 * (w[q] + w[q + 6]);
            D[(size_t)y * L.w + x] = sat_u8((a + (1 << 15)) >> 16);
        }
    }
}

// ---------------------------------------------------------------------- FAST --
// O3: FAST_t<16> segment test (>= 9 contiguous circle pixels darker than v - t or
// brighter than v + t) and cornerScore<16>; 0 = no corner (scores are >= t - 1 > 0)
__device__ __forceinline__ int fast_score(const int* d, int threshold) {
    int a0 = threshold;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(d[k + 1], d[k + 2]);
        a = min(a, d[k + 3]);
        if (a <= a0) continue;
        a = min(a, d[k + 4]);
        a = min(a, d[k + 5]);
        a = min(a, d[k + 6]);
        a = min(a, d[k + 7]);
        a = min(a, d[k + 8]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + 9]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int b = max(d[k + 1], d[k + 2]);
        b = max(b, d[k + 3]);
        b = max(b, d[k + 4]);
        if (b >= b0) continue;
        b = max(b, d[k + 5]);
        b = max(b, d[k + 6]);
        b = max(b, d[k + 7]);
        b = max(b, d[k + 8]);
        b0 = min(b0, max(b, d[k]));
        b0 = min(b0, max(b, d[k + 9]));
    }
    return -b0 - 1;
}
__device__ __forceinline__ bool fast_test(const int* d, int t) {
    // d[k] = v - p_k: darker means d > t, brighter means d < -t
    uint32_t dark = 0, bright = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        dark |= (uint32_t)(d[k] > t) << k;
        bright |= (uint32_t)(d[k] < -t) << k;
    }
    auto arc9 = [](uint32_t m) {
        uint32_t w = m | (m << 16);   // wrap
        uint32_t r = w;
#pragma unroll
        for (int i = 1; i < 9; ++i) r &= w >> i;
        return (r & 0xFFFFu) != 0;
    };
    return arc9(dark) || arc9(bright);
}

// ---------------------------------------------------------------- cells --
// One wave per 30-px cell of ComputeKeyPointsOctTree (:765-853), all cells of all levels
// of all images in one launch: the cell's ROI [iniX, maxX) x [iniY, maxY) into LDS, the
// FAST_t segment test + cornerScore on its detectable area [3, w - 3) x [3, h - 3) (O3),
// strict 3x3 non-max suppression with 0 outside that area, the surviving keys compacted
// in row-major order (cv::FAST's output order) into the cell's slot; the minThFAST pass
// only for cells the iniThFAST pass left empty (:803-808).
// Pass A: OpenCV's FAST_t prefilter on the four opposite pairs (0,8) (2,10) (4,12) (6,14)
// (every 9-arc holds one pixel of each pair: a necessary condition), zero scores, the
// candidates' indices compacted into LDS; pass B: the segment test + cornerScore on the
// candidates only, 64 at a time.
__device__ __forceinline__ void cell_fast(const uint8_t* P, int pw, uint8_t* Sc, uint16_t* cand, int dw, int dh,
                                          int th, int lane) {
    const float rdw = 1.0f / (float)dw;
    int nc = 0;
    for (int b = 0; b < dw * dh; b += 64) {
        const int i = b + lane;
        bool pass = false;
        if (i < dw * dh) {
            const int y = (int)(((float)i + 0.5f) * rdw), x = i - y * dw;
            const uint8_t* c = P + (y + 3) * pw + (x + 3);
            const int v = c[0];
            int dk = 1, br = 1;
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const int d0 = v - (int)c[kCircleY[k] * pw + kCircleX[k]];
                const int d1 = v - (int)c[kCircleY[k + 8] * pw + kCircleX[k + 8]];
                dk &= (d0 > th) | (d1 > th);
                br &= (d0 < -th) | (d1 < -th);
            }
            pass = (dk | br) != 0;
            Sc[i] = 0;
        }
        const unsigned long long m = __ballot(pass);
        if (pass) cand[nc + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)i;
        nc += __popcll(m);
    }
    wave_sync_lds();
    for (int b = 0; b < nc; b += 64) {
        if (b + lane < nc) {
            const int i = cand[b + lane];
            const int y = (int)(((float)i + 0.5f) * rdw), x = i - y * dw;
            const uint8_t* c = P + (y + 3) * pw + (x + 3);
            const int v = c[0];
            int d[25];
#pragma unroll
            for (int k = 0; k < 16; ++k) d[k] = v - (int)c[kCircleY[k] * pw + kCircleX[k]];
#pragma unroll
            for (int k = 16; k < 25; ++k) d[k] = d[k - 16];
            if (fast_test(d, th)) Sc[i] = (uint8_t)fast_score(d, th);
        }
    }
}

// strict 3x3 maxima of the score map (0 outside it), compacted in row-major order;
// returns their count (keys beyond cap are counted, not written)
__device__ __forceinline__ int cell_nms(const uint8_t* Sc, int dw, int dh, uint32_t* K, int cap, int kx0, int ky0,
                                        int lane) {
    int pos = 0;
    for (int b = 0; b < dw * dh; b += 64) {
        const int idx = b + lane;
        int keep = 0, x = 0, y = 0;
        if (idx < dw * dh) {
            y = idx / dw;
            x = idx - y * dw;
            keep = Sc[idx];
            if (keep) {
#pragma unroll
                for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                    for (int dx = -1; dx <= 1; ++dx) {
                        if (!dx && !dy) continue;
                        const int xx = x + dx, yy = y + dy;
                        const int nb = (xx >= 0 && xx < dw && yy >= 0 && yy < dh) ? Sc[yy * dw + xx] : 0;
                        if (!(keep > nb)) keep = 0;
                    }
            }
        }
        const unsigned long long m = __ballot(keep != 0);
        if (keep) {
            const int rank = pos + __popcll(m & ((1ull << lane) - 1ull));
            if (rank < cap) K[rank] = key_pack(kx0 + x, ky0 + y, keep);
        }
        pos += __popcll(m);
    }
    return pos;
}

#define CELL_LD 24
__global__ void __launch_bounds__(256) k_orb_cellfast(OrbDev o) {
    extern __shared__ __align__(16) unsigned char csm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = blockIdx.x * (blockDim.x >> 6) + wave, img = blockIdx.y;
    if (c >= o.ncell) return;
    // byte cells (dword cells triple the LDS and halve the occupancy: measured 1.9x slower)
    uint8_t* P = csm + wave * 4 * o.patch_cap;
    uint8_t* Sc = P + o.patch_cap;
    uint16_t* cand = reinterpret_cast<uint16_t*>(Sc + o.patch_cap);
    int l = 0;
    while (c >= o.cbase[l + 1]) ++l;
    const OrbLevel& L = o.lv[l];
    const int ci = c - o.cbase[l];
    const int i = ci / L.nCols, j = ci - (ci / L.nCols) * L.nCols;
    int* cnt_out = o.ccnt + (size_t)img * o.ncell + c;
    const int iniY = L.minBY + i * L.hCell, iniX = L.minBX + j * L.wCell;
    if (!(iniY < L.maxBY - 3 && iniX < L.maxBX - 6)) {
        if (lane == 0) *cnt_out = 0;
        return;
    }
    const int maxY = min(iniY + L.hCell + 6, L.maxBY), maxX = min(iniX + L.wCell + 6, L.maxBX);
    const int pw = maxX - iniX, ph = maxY - iniY, dw = pw - 6, dh = ph - 6;
    if (dw <= 0 || dh <= 0) {
        if (lane == 0) *cnt_out = 0;
        return;
    }
    const uint8_t* S = o.pyr + img * o.pyr_stride + L.off + (size_t)iniY * L.w + iniX;
    // the ROI in batches of CELL_LD bytes per lane, all loads in flight before the stores
    // (row = floor((idx + 0.5) / pw) is exact in float for ROIs below 2^12 bytes)
    const float rpw = 1.0f / (float)pw;
    for (int b = 0; b < pw * ph; b += 64 * CELL_LD) {
        uint8_t v[CELL_LD];
#pragma unroll
        for (int q = 0; q < CELL_LD; ++q) {
            const int idx = b + q * 64 + lane;
            const int r = (int)(((float)idx + 0.5f) * rpw), x = idx - r * pw;
            v[q] = idx < pw * ph ? S[(size_t)r * L.w + x] : 0;
        }
#pragma unroll
        for (int q = 0; q < CELL_LD; ++q) {
            const int idx = b + q * 64 + lane;
            if (idx < pw * ph) P[idx] = v[q];
        }
    }
    wave_sync_lds();
    uint32_t* K = o.ckeys + ((size_t)img * o.ncell + c) * o.ccap;
    cell_fast(P, pw, Sc, cand, dw, dh, o.ini_th, lane);
    wave_sync_lds();
    int pos = cell_nms(Sc, dw, dh, K, o.ccap, iniX + 3 - L.minBX, iniY + 3 - L.minBY, lane);
    if (pos == 0) {   // vKeysCell.empty(): FAST again at minThFAST (:803-808)
        cell_fast(P, pw, Sc, cand, dw, dh, o.min_th, lane);
        wave_sync_lds();
        pos = cell_nms(Sc, dw, dh, K, o.ccap, iniX + 3 - L.minBX, iniY + 3 - L.minBY, lane);
    }
    if (lane == 0) {
        if (pos > o.ccap) atomicOr(o.err, 1);
        *cnt_out = min(pos, o.ccap);
    }
}

// one workgroup per (image, level): the cells' keys concatenated in cell order (cell row,
// cell column) = vToDistributeKeys (:810-816)
#define GATHER_T 256
__global__ void __launch_bounds__(GATHER_T) k_orb_gather(OrbDev o) {
    __shared__ int off[ORB_MAX_CELLS + 1];
    __shared__ int wsum[GATHER_T / 64];
    const int l = blockIdx.x % o.nlevels, img = blockIdx.x / o.nlevels;
    const int c0 = o.cbase[l], nc = o.cbase[l + 1] - c0;
    const int* cnt = o.ccnt + (size_t)img * o.ncell + c0;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    // exclusive scan: GATHER_T contiguous chunks
    const int per = (nc + GATHER_T - 1) / GATHER_T;
    int acc = 0;
    for (int q = 0; q < per; ++q) {
        const int c = t * per + q;
        if (c < nc) acc += cnt[c];
    }
    int incl = acc;
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const int v = __shfl_up(incl, sh, 64);
        if (lane >= sh) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += wsum[w];
    int run = base + incl - acc;
    for (int q = 0; q < per; ++q) {
        const int c = t * per + q;
        if (c < nc) { off[c] = run; run += cnt[c]; }
    }
    if (t == GATHER_T - 1) off[nc] = run;
    __syncthreads();
    const int total = off[nc];
    uint32_t* K = o.keys + ((size_t)img * o.nlevels + l) * o.key_cap;
    const uint32_t* CK = o.ckeys + ((size_t)img * o.ncell + c0) * o.ccap;
    for (int c = wave; c < nc; c += GATHER_T / 64) {
        const int n = cnt[c], b = off[c];
        for (int k = lane; k < n; k += 64)
            if (b + k < o.key_cap) K[b + k] = CK[(size_t)c * o.ccap + k];
    }
    if (t == 0) {
        o.nkeys[img * o.nlevels + l] = min(total, o.key_cap);
        if (total > o.key_cap) atomicOr(o.err, 1);
    }
}

// ------------------------------------------------------------------- octree --
// DistributeOctTree (:539-763) — one wave per (image, level).  Nodes live in LDS as
// rectangles (x0, y0, x1, y1) over a contiguous range of the level's key array; the
// reference's std::list order is a doubly linked list (push_front, erase); DivideNode
// (:481-537) is a stable partition of the node's range by the wave (one ballot per
// group), through the per-level scratch array, children laid out n1 | n2 | n3 | n4.
struct ONode {
    int16_t x0, y0, x1, y1;
    int32_t off, len;
    int32_t id;            // creation order (O6)
    int16_t prev, next;    // (bNoMore is len == 1: it is only ever set from the key count)
};
// vSizeAndPointerToNode entry: size << 40 | creation id << 16 | node, so the u64 order is
// the (size, node) order of the reference's sort with O6 for ties
typedef uint64_t OExp;
__device__ __forceinline__ OExp oexp(int size, int id, int node) {
    return ((uint64_t)(uint32_t)size << 40) | ((uint64_t)(uint32_t)id << 16) | (uint32_t)node;
}
#define ORB_MAX_INI 16
#define DIV_REG 4   // nodes of up to 64 * DIV_REG keys are divided from registers

__device__ __forceinline__ void wave_fence_global() { __threadfence_block(); }


// stable partition of K[off, off + len) into G groups (grp(key) in [0, G)), through T
template <int G, typename F>
__device__ __forceinline__ void wave_partition(uint32_t* K, uint32_t* T, int off, int len, F grp, int* cnt) {
    const int lane = threadIdx.x & 63;
    int c[G];
#pragma unroll
    for (int q = 0; q < G; ++q) c[q] = 0;
    for (int b = 0; b < len; b += 64) {
        const int i = b + lane;
        const int g = i < len ? grp(K[off + i]) : -1;
#pragma unroll
        for (int q = 0; q < G; ++q) c[q] += __popcll(__ballot(g == q));
    }
    int run[G];
    int acc = 0;
#pragma unroll
    for (int q = 0; q < G; ++q) { run[q] = acc; acc += c[q]; }
    for (int b = 0; b < len; b += 64) {
        const int i = b + lane;
        const uint32_t k = i < len ? K[off + i] : 0u;
        const int g = i < len ? grp(k) : -1;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const unsigned long long m = __ballot(g == q);
            if (g == q) T[off + run[q] + __popcll(m & ((1ull << lane) - 1ull))] = k;
            run[q] += __popcll(m);
        }
    }
    __threadfence_block();
    for (int i = lane; i < len; i += 64) K[off + i] = T[off + i];
    __threadfence_block();
#pragma unroll
    for (int q = 0; q < G; ++q) cnt[q] = c[q];
}

__host__ __device__ __forceinline__ size_t orb_octree_node_lds(int node_cap) {
    return (size_t)node_cap * (sizeof(ONode) + 2 * sizeof(OExp) + 2);
}

// The list bookkeeping runs on wave-uniform registers (head, size, ids, allocation) with
// lane 0 storing the node records, so a DivideNode costs a few LDS round trips.  The
// nodes a main-loop pass divides are, in list order, the previous pass's children with
// more than one key in reverse creation order (every child is pushed to the front), i.e.
// vSizeAndPointerToNode of that pass read backwards; the first pass divides the initial
// nodes in column order.
__global__ void __launch_bounds__(64) k_orb_octree(OrbDev o) {
    extern __shared__ __align__(16) unsigned char osm[];
    const int cap = o.node_cap;
    ONode* nd = reinterpret_cast<ONode*>(osm);
    OExp* exA = reinterpret_cast<OExp*>(nd + cap);
    OExp* exB = exA + cap;
    int16_t* freel = reinterpret_cast<int16_t*>(exB + cap);
    const int lane = threadIdx.x;
    const int l = blockIdx.x % o.nlevels, img = blockIdx.x / o.nlevels;
    const OrbLevel& L = o.lv[l];
    const size_t kb = ((size_t)img * o.nlevels + l) * o.key_cap;
    uint32_t* K = o.keys + kb;   // generic pointer: global, or the LDS copy below
    uint32_t* T = o.tmp + kb;
    const int nk = o.nkeys[img * o.nlevels + l];
    const int N = L.N;
    uint32_t* out = o.sel + ((size_t)img * o.nlevels + l) * o.sel_cap;
    if (nk == 0) {
        if (lane == 0) o.nsel[img * o.nlevels + l] = 0;
        return;
    }
    if (nk <= o.key_lds) {   // every divide then reads and writes LDS instead of HBM
        uint32_t* KL = reinterpret_cast<uint32_t*>(osm + ((orb_octree_node_lds(cap) + 15) & ~(size_t)15));
        for (int i = lane; i < nk; i += 64) KL[i] = K[i];
        K = KL;
    }
    // wave-uniform list state
    int head = -1, lsize = 0, next_id = 0, nfree = 0, nalloc = 0;
    OExp* cur = exA;   // vSizeAndPointerToNode of the running pass / round
    OExp* prv = exB;   // ... of the previous one
    int ncur = 0;
    bool overflow = false;
    auto alloc = [&]() -> int {
        if (nfree > 0) return freel[--nfree];
        if (nalloc < cap) return nalloc++;
        overflow = true;
        return -1;
    };
    auto push_front = [&](int c) {
        if (lane == 0) {
            nd[c].prev = -1;
            nd[c].next = (int16_t)head;
            if (head >= 0) nd[head].prev = (int16_t)c;
        }
        head = c;
        ++lsize;
    };
    // DivideNode (:481-537) of node i and the list surgery of :621-660 / :700-730: the
    // non-empty children pushed to the front in n1..n4 order, those with > 1 keys recorded,
    // the parent erased.  Returns the number recorded.
    auto divide = [&](int i) -> int {
        wave_sync_lds();
        const ONode nv = nd[i];
        const int x0 = nv.x0, y0 = nv.y0, x1 = nv.x1, y1 = nv.y1, off = nv.off, len = nv.len;
        int pv = nv.prev;
        const int nx = nv.next;
        const int halfX = (int)ceilf((float)(x1 - x0) / 2), halfY = (int)ceilf((float)(y1 - y0) / 2);
        const int mx = x0 + halfX, my = y0 + halfY;
        int cnt[4];
        auto quad = [&](uint32_t k) {
            const float x = (float)key_x(k), y = (float)key_y(k);
            return x < (float)mx ? (y < (float)my ? 0 : 2) : (y < (float)my ? 1 : 3);
        };
        if (len <= 64 * DIV_REG) {
            // the node's keys in registers: one read, one scatter in place (stores reach
            // memory before the pass ends: wave_fence_global at the end of every pass)
            uint32_t kr[DIV_REG];
            int g[DIV_REG];
#pragma unroll
            for (int q = 0; q < 4; ++q) cnt[q] = 0;
#pragma unroll
            for (int r = 0; r < DIV_REG; ++r) {
                if (r * 64 < len) {
                    const int idx = r * 64 + lane;
                    kr[r] = idx < len ? K[off + idx] : 0u;
                    g[r] = idx < len ? quad(kr[r]) : -1;
#pragma unroll
                    for (int q = 0; q < 4; ++q) cnt[q] += __popcll(__ballot(g[r] == q));
                }
            }
            int run[4] = {off, off + cnt[0], off + cnt[0] + cnt[1], off + cnt[0] + cnt[1] + cnt[2]};
#pragma unroll
            for (int r = 0; r < DIV_REG; ++r) {
                if (r * 64 < len) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const unsigned long long m = __ballot(g[r] == q);
                        if (g[r] == q) K[run[q] + __popcll(m & ((1ull << lane) - 1ull))] = kr[r];
                        run[q] += __popcll(m);
                    }
                }
            }
        } else {
            wave_partition<4>(K, T, off, len, quad, cnt);
        }
        const int cx0[4] = {x0, mx, x0, mx}, cy0[4] = {y0, y0, my, my};
        const int cx1[4] = {mx, x1, mx, x1}, cy1[4] = {my, my, y1, y1};
        int o2 = off, rec = 0, first = -1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (cnt[q] > 0) {
                const int c = alloc();
                if (c >= 0) {
                    const int id = next_id++;
                    if (lane == 0) {
                        nd[c].x0 = (int16_t)cx0[q]; nd[c].y0 = (int16_t)cy0[q];
                        nd[c].x1 = (int16_t)cx1[q]; nd[c].y1 = (int16_t)cy1[q];
                        nd[c].off = o2; nd[c].len = cnt[q]; nd[c].id = id;
                    }
                    push_front(c);
                    if (first < 0) first = c;
                    if (cnt[q] > 1) {
                        if (lane == 0) cur[ncur] = oexp(cnt[q], id, c);
                        ++ncur;
                        ++rec;
                    }
                }
            }
            o2 += cnt[q];
        }
        // erase the parent: a parent at the head has the first child pushed as prev now
        if (pv < 0 && first >= 0) pv = first;
        if (lane == 0) {
            if (pv >= 0) nd[pv].next = (int16_t)nx;
            if (nx >= 0) nd[nx].prev = (int16_t)pv;
            freel[nfree] = (int16_t)i;
        }
        if (pv < 0) head = nx;
        ++nfree;
        --lsize;
        return rec;
    };
    // ---- initial nodes (:542-585): nIni columns of width hX over the keys' x
    const int nIni = L.nIni;
    {
        const float hX = L.hX;
        // stable partition by column, one pass over the keys per column (nIni is 1-4 for
        // camera aspect ratios; a loop keeps the code small), through T
        int cnt[ORB_MAX_INI], offs[ORB_MAX_INI];
        int run = 0;
#pragma unroll 1
        for (int q = 0; q < nIni; ++q) {
            const int r0 = run;
            for (int b = 0; b < nk; b += 64) {
                const int i = b + lane;
                const uint32_t k = i < nk ? K[i] : 0u;
                const bool in = i < nk && (int)__fdiv_rn((float)key_x(k), hX) == q;
                const unsigned long long m = __ballot(in);
                if (in) T[run + __popcll(m & ((1ull << lane) - 1ull))] = k;
                run += __popcll(m);
            }
            // (registers indexed by the loop counter: written through a select chain)
#pragma unroll
            for (int u = 0; u < ORB_MAX_INI; ++u)
                if (u == q) { offs[u] = r0; cnt[u] = run - r0; }
        }
#pragma unroll
        for (int u = 0; u < ORB_MAX_INI; ++u)
            if (u >= nIni) { offs[u] = run; cnt[u] = 0; }
        wave_fence_global();
        for (int i = lane; i < nk; i += 64) K[i] = T[i];
        wave_fence_global();
        const int H = L.maxBY - L.minBY;
        next_id = nIni;   // the reference creates all nIni nodes, then erases the empty ones
        // push_back in column order = push_front from the last column
#pragma unroll
        for (int q = ORB_MAX_INI - 1; q >= 0; --q) {
            int c = -1;
            if (q < nIni && cnt[q] > 0) {
                c = alloc();
                if (c >= 0) {
                    if (lane == 0) {
                        nd[c].x0 = (int16_t)(int)(hX * (float)q); nd[c].y0 = 0;
                        nd[c].x1 = (int16_t)(int)(hX * (float)(q + 1)); nd[c].y1 = (int16_t)H;
                        nd[c].off = offs[q]; nd[c].len = cnt[q]; nd[c].id = q;
                    }
                    push_front(c);
                }
            }
            // the first pass's work list: the initial nodes with > 1 keys, read from the back
            if (q < nIni && c >= 0 && cnt[q] > 1) {
                if (lane == 0) cur[ncur] = (OExp)c;
                ++ncur;
            }
        }
    }
    wave_sync_lds();
    // ---- the subdivision loop (:594-739), one call site of divide (code size): phase 0 =
    // the first pass, 1 = a later pass of the main loop, 2 = a round of the sorted expansion
    // (:699-737).  Each pass / round reads its work list `prv` from the back and records
    // this pass's children in `cur`.
    bool finish = false;
    int phase = 0;
    while (!finish) {
        const int prevSize = lsize;
        const int ntodo = ncur;
        if (phase < 2) {
            OExp* t = prv; prv = cur; cur = t;
        } else {
            // vPrevSizeAndPointerToNode = vSizeAndPointerToNode sorted by (size, node) (O6):
            // rank sort (the entries are distinct) from cur into prv
            wave_sync_lds();
            for (int e = lane; e < ntodo; e += 64) {
                const OExp v = cur[e];
                int rank = 0;
                for (int j = 0; j < ntodo; ++j) rank += cur[j] < v;
                prv[rank] = v;
            }
        }
        wave_sync_lds();
        ncur = 0;
        int nToExpand = 0;
        for (int j = ntodo - 1; j >= 0; --j) {
            nToExpand += divide((int)(prv[j] & 0xFFFFu));
            if (phase == 2 && lsize >= N) break;
        }
        wave_fence_global();
        if (overflow) break;
        if (lsize >= N || lsize == prevSize) finish = true;
        else if (phase < 2) phase = (lsize + nToExpand * 3 > N) ? 2 : 1;
    }
    wave_sync_lds();
    // ---- the best key of every node, in list order (:741-760): first strict maximum.
    // The list order into LDS (prv is free now), then a lane per node for nodes of up to
    // 16 keys and the whole wave for the larger ones
    int16_t* ordl = reinterpret_cast<int16_t*>(prv);
    if (lane == 0) {
        int k = 0;
        for (int it = head; it >= 0; it = nd[it].next) ordl[k++] = (int16_t)it;
    }
    wave_sync_lds();
    const int n_out = lsize;
    for (int base = 0; base < n_out; base += 64) {
        const int idx = base + lane;
        const int node = idx < n_out ? ordl[idx] : -1;
        const int off = node >= 0 ? nd[node].off : 0, len = node >= 0 ? nd[node].len : 0;
        uint32_t bk = len > 0 ? K[off] : 0u;
        if (len <= 16) {
            for (int q = 1; q < len; ++q) {
                const uint32_t k = K[off + q];
                if (key_s(k) > key_s(bk)) bk = k;
            }
        }
        unsigned long long big = __ballot(len > 16);
        while (big) {
            const int src = __ffsll((long long)big) - 1;
            big &= big - 1;
            const int boff = __shfl(off, src), blen = __shfl(len, src);
            int bs = -1, bi = 0x7FFFFFFF;
            for (int b = 0; b < blen; b += 64) {
                const int i = b + lane;
                int sc = i < blen ? key_s(K[boff + i]) : -1;
                int mi = i < blen ? i : 0x7FFFFFFF;
#pragma unroll
                for (int sh = 32; sh > 0; sh >>= 1) {
                    const int os = __shfl_xor(sc, sh, 64), oi = __shfl_xor(mi, sh, 64);
                    if (os > sc || (os == sc && oi < mi)) { sc = os; mi = oi; }
                }
                if (sc > bs) { bs = sc; bi = mi; }   // strictly larger: the earlier block keeps ties
            }
            if (lane == src) bk = K[boff + bi];
        }
        if (idx < n_out && idx < o.sel_cap) out[idx] = bk;
    }
    if (lane == 0) {
        if (overflow) atomicOr(o.err, 2);
        if (n_out > o.sel_cap) atomicOr(o.err, 4);
        o.nsel[img * o.nlevels + l] = overflow ? 0 : min(n_out, o.sel_cap);
    }
}

// ----------------------------------------------------------------- describe --
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

// two kept keypoints per wave (one per 32-lane half, 8 per workgroup): IC_Angle's integer
// moments over the 31-px disc split across the half's lanes (u = lane - 15, rows v = 0..15)
// and reduced (exact in any order); bit 32w + lane of the descriptor (pattern points 2b,
// 2b + 1) on lane `lane` of the half, one ballot per 32 bits of each keypoint
__device__ __forceinline__ int half_sum(int v) {
#pragma unroll
    for (int sh = 16; sh > 0; sh >>= 1) v += __shfl_xor(v, sh, 64);
    return v;
}

__global__ void __launch_bounds__(256) k_orb_describe(OrbDev o, int n, gfpl_keypoint* kps, uint8_t* desc, int* n_kp,
                                                      float* angle_out, float* resp_out, int kp_cap) {
    const int img = blockIdx.y, lane = threadIdx.x & 63, hl = lane & 31, half = lane >> 5;
    const int t = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + half;
    int tot = 0;
    for (int l = 0; l < o.nlevels; ++l) tot += o.nsel[img * o.nlevels + l];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        n_kp[img] = min(tot, kp_cap);
        if (tot > kp_cap) atomicOr(o.err, 4);
    }
    const int nt = min(tot, kp_cap);
    if ((t & ~1) >= nt) return;   // both halves idle (the wave is uniform here)
    const bool valid = t < nt;
    int l = 0, r = valid ? t : 0;
    while (r >= o.nsel[img * o.nlevels + l]) { r -= o.nsel[img * o.nlevels + l]; ++l; }
    const OrbLevel& L = o.lv[l];
    const uint32_t k = o.sel[((size_t)img * o.nlevels + l) * o.sel_cap + r];
    const int x = key_x(k) + L.minBX, y = key_y(k) + L.minBY;   // level coordinates (:843-844)
    // IC_Angle (:77-104)
    const uint8_t* center = o.pyr + img * o.pyr_stride + L.off + (size_t)y * L.w + x;
    const int u = hl - 15;
    int m_01 = 0, m_10 = 0;
    if (u <= 15) {
        m_10 = u * center[u];
#pragma unroll
        for (int v = 1; v <= 15; ++v) {
            if (u >= -o.umax[v] && u <= o.umax[v]) {
                const int vp = center[u + v * L.w], vm = center[u - v * L.w];
                m_01 += v * (vp - vm);
                m_10 += u * (vp + vm);
            }
        }
    }
    m_01 = half_sum(m_01);
    m_10 = half_sum(m_10);
    const float ang = fast_atan2((float)m_01, (float)m_10);
    // computeOrbDescriptor (:108-148) on the blurred level, O5
    const float factorPI = (float)(M_PI / 180.f);
    const float a_ = ang * factorPI;
    const float ca = (float)det_cos((double)a_), sa = (float)det_sin((double)a_);
    const uint8_t* B = o.blur + img * o.blur_stride + L.off + (size_t)y * L.w + x;
    const size_t q = (size_t)img * kp_cap + t;
    uint32_t* dd = reinterpret_cast<uint32_t*>(desc + 32 * q);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const int bit = 32 * w + hl;
        const int px0 = c_orb_pattern[4 * bit], py0 = c_orb_pattern[4 * bit + 1];
        const int px1 = c_orb_pattern[4 * bit + 2], py1 = c_orb_pattern[4 * bit + 3];
        const int t0 = B[__float2int_rn(px0 * sa + py0 * ca) * L.w + __float2int_rn(px0 * ca - py0 * sa)];
        const int t1 = B[__float2int_rn(px1 * sa + py1 * ca) * L.w + __float2int_rn(px1 * ca - py1 * sa)];
        const unsigned long long m = __ballot(t0 < t1);
        if (valid && hl == w) dd[w] = (uint32_t)(m >> (32 * half));
    }
    if (valid && hl == 0) {
        // keypoint coordinates scaled to level 0 (:1094-1101)
        float fx = (float)x, fy = (float)y;
        if (l != 0) { fx = fx * L.scale; fy = fy * L.scale; }
        kps[q] = gfpl_keypoint{fx, fy, l};
        if (angle_out) angle_out[q] = ang;
        if (resp_out) resp_out[q] = (float)key_s(k);
    }
}

}  // namespace gfpl

// ======================================================================= ABI ==
using namespace gfpl;

struct gfpl_orb {
    int device = 0;
    hipStream_t stream = nullptr;
    gfpl_ctx* ctx = nullptr;  // its camera checks the pyramid layout the tracker will read
    AsyncStatus st;
    gfpl_orb_params prm{};
    int max_images = 0, kp_cap = 0;
    OrbDev d{};
    void* base = nullptr;         // one allocation for everything
    long long pyr_bytes = 0;      // used bytes of one pyramid
    int resize_lds[GFPL_MAX_LEVELS] = {};   // k_orb_resize's LDS bytes per level
};

namespace {

#define ORB_HIPCHK(x)                                                                  \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "gfpl_orb: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return GFPL_E_HIP;                                                         \
        }                                                                              \
    } while (0)

size_t orb_octree_lds(int node_cap, int key_lds) {
    return ((orb_octree_node_lds(node_cap) + 15) & ~(size_t)15) + 4 * (size_t)key_lds;
}

inline int cv_round_f(float v) { return (int)std::nearbyintf(v); }
inline int cv_round_d(double v) { return (int)std::nearbyint(v); }
inline int16_t sat_short(float v) { return (int16_t)std::min(std::max(cv_round_f(v), -32768), 32767); }

// O1 resize tables of levels 1.. of d's pyramid geometry (d.lv[l].w / h, d.nlevels): per level
// the x offsets / weights and y offsets / weights, d.xmax, and k_orb_resize's LDS bytes
void resize_tables(OrbDev& d, std::vector<int>& xofs_h, std::vector<int16_t>& alpha_h, std::vector<int>& yofs_h,
                   std::vector<int16_t>& beta_h, long long* xoff, long long* yoff, int* resize_lds) {
    for (int l = 1; l < d.nlevels; ++l) {
        const OrbLevel& s = d.lv[l - 1];
        const OrbLevel& t = d.lv[l];
        const double scale_x = 1. / ((double)t.w / s.w), scale_y = 1. / ((double)t.h / s.h);
        xoff[l] = (long long)xofs_h.size();
        int xmax = t.w;
        for (int dx = 0; dx < t.w; ++dx) {
            float fx = (float)((dx + 0.5) * scale_x - 0.5);
            int sx = (int)std::floor(fx);
            fx -= sx;
            if (sx < 0) { fx = 0; sx = 0; }
            if (sx + 1 >= s.w) {
                xmax = std::min(xmax, dx);
                if (sx >= s.w - 1) { fx = 0; sx = s.w - 1; }
            }
            xofs_h.push_back(sx);
            alpha_h.push_back(sat_short((1.f - fx) * 2048));
            alpha_h.push_back(sat_short(fx * 2048));
        }
        d.xmax[l] = xmax;
        yoff[l] = (long long)yofs_h.size();
        for (int dy = 0; dy < t.h; ++dy) {
            float fy = (float)((dy + 0.5) * scale_y - 0.5);
            const int sy = (int)std::floor(fy);
            fy -= sy;
            yofs_h.push_back(sy);
            beta_h.push_back(sat_short((1.f - fy) * 2048));
            beta_h.push_back(sat_short(fy * 2048));
        }
        // k_orb_resize's LDS: the most source rows a RESIZE_ROWS band reads + its output rows
        int rows = 1;
        for (int y0 = 0; y0 < t.h; y0 += RESIZE_ROWS) {
            const int y1 = std::min(y0 + RESIZE_ROWS, t.h) - 1;
            const int lo = std::min(std::max(yofs_h[yoff[l] + y0], 0), s.h - 1);
            const int hi = std::min(std::max(yofs_h[yoff[l] + y1] + 1, 0), s.h - 1);
            rows = std::max(rows, hi - lo + 1);
        }
        resize_lds[l] = 4 * (rows * ((s.w + 6) >> 2) + RESIZE_ROWS * ((t.w >> 2) + 2));
    }
}

}  // namespace

extern "C" int gfpl_orb_create(gfpl_ctx* ctx, int width, int height, const gfpl_orb_params* prm, int max_images,
                               int kp_cap, gfpl_orb** out) {
    if (!ctx || !prm || !out || max_images < 1 || kp_cap < 1) return GFPL_E_INVALID;
    if (prm->nlevels < 1 || prm->nlevels > GFPL_MAX_LEVELS || !(prm->scale_factor > 1.0f) || prm->nfeatures < 1)
        return GFPL_E_INVALID;
    if (width < 64 || height < 64 || width > 2047 || height > 2047) return GFPL_E_INVALID;
    const int dev = gfpl_ctx_device(ctx);
    ORB_HIPCHK(hipSetDevice(dev));
    gfpl_orb* o = new gfpl_orb();
    o->device = dev;
    o->stream = (hipStream_t)gfpl_ctx_stream(ctx);
    o->ctx = ctx;
    o->prm = *prm;
    o->max_images = max_images;
    o->kp_cap = kp_cap;
    OrbDev& d = o->d;
    d.W = width;
    d.H = height;
    d.nlevels = prm->nlevels;
    d.ini_th = std::min(std::max(prm->ini_th_fast, 0), 255);
    d.min_th = std::min(std::max(prm->min_th_fast, 0), 255);
    // ORBextractor::ORBextractor (:410-470)
    float sc[GFPL_MAX_LEVELS], isc[GFPL_MAX_LEVELS];
    sc[0] = 1.0f;
    for (int i = 1; i < d.nlevels; ++i) sc[i] = sc[i - 1] * prm->scale_factor;
    for (int i = 0; i < d.nlevels; ++i) isc[i] = 1.0f / sc[i];
    int nPer[GFPL_MAX_LEVELS];
    {
        const float factor = 1.0f / prm->scale_factor;
        float nDesired = prm->nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)d.nlevels));
        int sum = 0;
        for (int l = 0; l < d.nlevels - 1; ++l) {
            nPer[l] = cv_round_f(nDesired);
            sum += nPer[l];
            nDesired *= factor;
        }
        nPer[d.nlevels - 1] = std::max(prm->nfeatures - sum, 0);
    }
    {
        int umax[16];
        const int vmax = (int)std::floor(15 * std::sqrt(2.f) / 2 + 1), vmin = (int)std::ceil(15 * std::sqrt(2.f) / 2);
        for (int v = 0; v <= vmax; ++v) umax[v] = cv_round_d(std::sqrt(225.0 - v * v));
        for (int v = 15, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
        for (int v = 0; v < 16; ++v) d.umax[v] = umax[v];
    }
    {   // O2 taps
        float cf[7];
        double sum = 0;
        for (int i = 0; i < 7; ++i) {
            const double x = i - 3.0;
            cf[i] = (float)std::exp(-0.125 * x * x);
            sum += cf[i];
        }
        sum = 1. / sum;
        for (int i = 0; i < 7; ++i) d.blur_k[i] = cv_round_f((float)(cf[i] * sum) * 256.0f);
    }
    long long off = 0;
    int max_cells = 0, max_n = 0;
    for (int l = 0; l < d.nlevels; ++l) {
        OrbLevel& L = d.lv[l];
        L.w = cv_round_f((float)width * isc[l]);
        L.h = cv_round_f((float)height * isc[l]);
        L.off = off;
        off += (long long)L.w * L.h;
        L.minBX = 19 - 3;
        L.minBY = L.minBX;
        L.maxBX = L.w - 19 + 3;
        L.maxBY = L.h - 19 + 3;
        const float wf = (float)(L.maxBX - L.minBX), hf = (float)(L.maxBY - L.minBY);
        L.nCols = (int)(wf / 30.f);
        L.nRows = (int)(hf / 30.f);
        if (L.nCols < 1 || L.nRows < 1) { delete o; return GFPL_E_INVALID; }
        L.wCell = (int)std::ceil(wf / L.nCols);
        L.hCell = (int)std::ceil(hf / L.nRows);
        L.N = nPer[l];
        L.nIni = (int)std::round(wf / (float)(L.maxBY - L.minBY));
        if (L.nIni < 1 || L.nIni > ORB_MAX_INI) { delete o; return GFPL_E_UNSUPPORTED; }
        L.hX = wf / L.nIni;
        L.scale = sc[l];
        max_cells = std::max(max_cells, L.nRows * L.nCols);
        max_n = std::max(max_n, L.N);
    }
    if (max_cells > ORB_MAX_CELLS) { delete o; return GFPL_E_UNSUPPORTED; }
    {
        int ncell = 0, maxw = 0, maxh = 0;
        for (int l = 0; l < d.nlevels; ++l) {
            d.cbase[l] = ncell;
            ncell += d.lv[l].nRows * d.lv[l].nCols;
            maxw = std::max(maxw, d.lv[l].wCell);
            maxh = std::max(maxh, d.lv[l].hCell);
        }
        d.cbase[d.nlevels] = ncell;
        d.ncell = ncell;
        d.ccap = ((maxw + 1) / 2) * ((maxh + 1) / 2);
        d.patch_cap = ((maxw + 6) * (maxh + 6) + 15) & ~15;
        // waves (cells) per workgroup: up to 4 within 150 KB of LDS
        d.cell_waves = (int)std::min<long long>(4, (150 * 1024) / (4LL * d.patch_cap));
        if (d.cell_waves < 1 || (maxw + 6) * (maxh + 6) >= 4096) { delete o; return GFPL_E_UNSUPPORTED; }
    }
    d.node_cap = max_n + 4 * ORB_MAX_INI + 16;   // list size <= max(N, 4 nIni) + 3, + 4 children in flight
    // keys in LDS up to a 40 KB workgroup (four single-wave octree workgroups per CU)
    d.key_lds = std::max(0, (int)((40 * 1024 - (long long)orb_octree_lds(d.node_cap, 0)) / 4) & ~63);
    if (orb_octree_lds(d.node_cap, d.key_lds) > 160 * 1024 - 64) { delete o; return GFPL_E_UNSUPPORTED; }
    if (hipFuncSetAttribute((const void*)k_orb_cellfast, hipFuncAttributeMaxDynamicSharedMemorySize,
                            4 * d.patch_cap * d.cell_waves) !=
        hipSuccess) { delete o; return GFPL_E_HIP; }
    if (hipFuncSetAttribute((const void*)k_orb_octree, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)orb_octree_lds(d.node_cap, d.key_lds)) != hipSuccess) { delete o; return GFPL_E_HIP; }
    o->pyr_bytes = off;
    d.pyr_stride = (off + 255) & ~255LL;
    d.blur_stride = d.pyr_stride;
    // FAST keys per level: the reference keeps them all; strict 3x3 maxima are never
    // 8-adjacent, so a level holds at most ~1/4 of its cells' pixels
    d.key_cap = (int)std::min<long long>((long long)width * height / 4 + 4LL * (width + height) + 1024, 1 << 22);
    d.sel_cap = max_n + 4 * ORB_MAX_INI + 8;   // DistributeOctTree keeps <= max(N, 4 nIni) + 3 nodes
    // resize tables (O1), one set per level
    std::vector<int> xofs_h, yofs_h;
    std::vector<int16_t> alpha_h, beta_h;
    long long xoff[GFPL_MAX_LEVELS] = {}, yoff[GFPL_MAX_LEVELS] = {};
    resize_tables(d, xofs_h, alpha_h, yofs_h, beta_h, xoff, yoff, o->resize_lds);
    int rz_max = 0;
    for (int l = 1; l < d.nlevels; ++l) rz_max = std::max(rz_max, o->resize_lds[l]);
    if (rz_max > 160 * 1024 - 64) { delete o; return GFPL_E_UNSUPPORTED; }
    if (rz_max > 0 && hipFuncSetAttribute((const void*)k_orb_resize, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          rz_max) != hipSuccess) { delete o; return GFPL_E_HIP; }
    // one allocation: tables | pyr | blur | ckeys | ccnt | keys | tmp | nkeys | nsel | sel | err
    const long long M = max_images;
    auto al = [](long long v) { return (v + 255) & ~255LL; };
    const long long b_x = al(4 * (long long)xofs_h.size() + 4), b_a = al(2 * (long long)alpha_h.size() + 4);
    const long long b_y = al(4 * (long long)yofs_h.size() + 4), b_b = al(2 * (long long)beta_h.size() + 4);
    const long long b_img = al(M * d.pyr_stride);
    const long long b_keys = al(4 * M * d.nlevels * (long long)d.key_cap);
    const long long b_n = al(4 * M * d.nlevels);
    const long long b_sel = al(4 * M * d.nlevels * (long long)d.sel_cap);
    const long long b_ck = al(4 * M * d.ncell * (long long)d.ccap), b_cc = al(4 * M * d.ncell);
    const long long total = b_x + b_a + b_y + b_b + 2 * b_img + 2 * b_keys + 2 * b_n + b_sel + b_ck + b_cc + 256;
    if (hipMalloc(&o->base, (size_t)total) != hipSuccess) { delete o; return GFPL_E_HIP; }
    char* p = (char*)o->base;
    int* xo = (int*)p; p += b_x;
    int16_t* ap = (int16_t*)p; p += b_a;
    int* yo = (int*)p; p += b_y;
    int16_t* bp = (int16_t*)p; p += b_b;
    d.pyr = (uint8_t*)p; p += b_img;
    d.blur = (uint8_t*)p; p += b_img;
    d.ckeys = (uint32_t*)p; p += b_ck;
    d.ccnt = (int*)p; p += b_cc;
    d.keys = (uint32_t*)p; p += b_keys;
    d.tmp = (uint32_t*)p; p += b_keys;
    d.nkeys = (int*)p; p += b_n;
    d.nsel = (int*)p; p += b_n;
    d.sel = (uint32_t*)p; p += b_sel;
    d.err = (int*)p;
    for (int l = 1; l < d.nlevels; ++l) {
        d.xofs[l] = xo + xoff[l];
        d.alpha[l] = ap + 2 * xoff[l];
        d.yofs[l] = yo + yoff[l];
        d.beta[l] = bp + 2 * yoff[l];
    }
    bool ok = true;
    if (!xofs_h.empty()) {
        ok = ok && hipMemcpy(xo, xofs_h.data(), 4 * xofs_h.size(), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && hipMemcpy(ap, alpha_h.data(), 2 * alpha_h.size(), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && hipMemcpy(yo, yofs_h.data(), 4 * yofs_h.size(), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && hipMemcpy(bp, beta_h.data(), 2 * beta_h.size(), hipMemcpyHostToDevice) == hipSuccess;
    }
    ok = ok && hipMemcpyToSymbol(HIP_SYMBOL(c_orb_pattern), kOrbPattern, sizeof(kOrbPattern)) == hipSuccess;
    if (!ok || o->st.init(d.err, o->stream) != hipSuccess) { o->st.destroy(); (void)hipFree(o->base); delete o; return GFPL_E_HIP; }
    gfpl_ctx_attach(ctx);
    *out = o;
    return GFPL_OK;
}

extern "C" int gfpl_orb_destroy(gfpl_orb* o) {
    if (!o) return GFPL_E_INVALID;
    (void)hipStreamSynchronize(o->stream);
    o->st.destroy();
    if (o->base) (void)hipFree(o->base);
    gfpl_ctx_detach(o->ctx);
    delete o;
    return GFPL_OK;
}

// ---- pyramid builder (levels 1.. of packed right pyramids from their level 0; used by
// gfpl_upload_frames_l0_async): the O1 tables of the camera's geometry, k_orb_resize per level
namespace gfpl {
struct PyrBuild {
    OrbDev d{};
    void* tables = nullptr;
    int resize_lds[GFPL_MAX_LEVELS] = {};
};
int pyrbuild_create(const gfpl_camera* cam, PyrBuild** out) {
    if (!cam || !out || cam->n_levels < 1 || cam->n_levels > GFPL_MAX_LEVELS) return GFPL_E_INVALID;
    PyrBuild* pb = new PyrBuild();
    OrbDev& d = pb->d;
    d.W = cam->width;
    d.H = cam->height;
    d.nlevels = cam->n_levels;
    for (int l = 0; l < d.nlevels; ++l) {
        d.lv[l].w = cam->lvl_cols[l];
        d.lv[l].h = cam->lvl_rows[l];
        d.lv[l].off = cam->lvl_offset[l];
    }
    std::vector<int> xofs_h, yofs_h;
    std::vector<int16_t> alpha_h, beta_h;
    long long xoff[GFPL_MAX_LEVELS] = {}, yoff[GFPL_MAX_LEVELS] = {};
    resize_tables(d, xofs_h, alpha_h, yofs_h, beta_h, xoff, yoff, pb->resize_lds);
    int rz_max = 0;
    for (int l = 1; l < d.nlevels; ++l) rz_max = std::max(rz_max, pb->resize_lds[l]);
    if (rz_max > 160 * 1024 - 64) { delete pb; return GFPL_E_UNSUPPORTED; }
    if (rz_max > 0 && hipFuncSetAttribute((const void*)k_orb_resize, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          rz_max) != hipSuccess) { delete pb; return GFPL_E_HIP; }
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t bx = al(4 * xofs_h.size() + 4), ba = al(2 * alpha_h.size() + 4), by = al(4 * yofs_h.size() + 4),
                 bb = al(2 * beta_h.size() + 4);
    if (hipMalloc(&pb->tables, bx + ba + by + bb) != hipSuccess) { delete pb; return GFPL_E_HIP; }
    char* q = (char*)pb->tables;
    int* xo = (int*)q;
    int16_t* ap = (int16_t*)(q + bx);
    int* yo = (int*)(q + bx + ba);
    int16_t* bp = (int16_t*)(q + bx + ba + by);
    bool ok = true;
    if (!xofs_h.empty()) {
        ok = ok && hipMemcpy(xo, xofs_h.data(), 4 * xofs_h.size(), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && hipMemcpy(ap, alpha_h.data(), 2 * alpha_h.size(), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && hipMemcpy(yo, yofs_h.data(), 4 * yofs_h.size(), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && hipMemcpy(bp, beta_h.data(), 2 * beta_h.size(), hipMemcpyHostToDevice) == hipSuccess;
    }
    if (!ok) { (void)hipFree(pb->tables); delete pb; return GFPL_E_HIP; }
    for (int l = 1; l < d.nlevels; ++l) {
        d.xofs[l] = xo + xoff[l];
        d.alpha[l] = ap + 2 * xoff[l];
        d.yofs[l] = yo + yoff[l];
        d.beta[l] = bp + 2 * yoff[l];
    }
    *out = pb;
    return GFPL_OK;
}
hipError_t pyrbuild_run(PyrBuild* pb, uint8_t* pyr, long long stride, int n, hipStream_t s) {
    OrbDev d = pb->d;
    d.pyr = pyr;
    d.pyr_stride = stride;
    for (int l = 1; l < d.nlevels; ++l)
        hipLaunchKernelGGL(k_orb_resize, dim3((d.lv[l].h + RESIZE_ROWS - 1) / RESIZE_ROWS, n), dim3(RESIZE_T),
                           pb->resize_lds[l], s, d, l);
    return hipGetLastError();
}
void pyrbuild_destroy(PyrBuild* pb) {
    if (!pb) return;
    if (pb->tables) (void)hipFree(pb->tables);
    delete pb;
}
}  // namespace gfpl

extern "C" int gfpl_orb_pyramid_bytes(const gfpl_orb* o, int64_t* bytes) {
    if (!o || !bytes) return GFPL_E_INVALID;
    *bytes = o->pyr_bytes;
    return GFPL_OK;
}

extern "C" int gfpl_orb_extract_async(gfpl_orb* o, const uint8_t* images, int n, gfpl_keypoint* kps, uint8_t* desc,
                                      int* n_kp, float* angle, float* response, uint8_t* pyramid, int64_t pyr_stride) {
    if (!o || !images || n < 1 || n > o->max_images || !kps || !desc || !n_kp) return GFPL_E_INVALID;
    if (pyramid && pyr_stride < o->pyr_bytes) return GFPL_E_INVALID;
    if (pyramid) {
        // a pyramid written at the stride of the context camera's pyramids, for images of its
        // size, is the tracker's input (gfpl_frames.pyr_r): its level geometry must be the
        // camera's, else the sub-pixel SAD would read other pixels than the reference's
        const gfpl_camera* cam = gfpl_ctx_camera(o->ctx);
        if (cam && cam->width == o->d.W && cam->height == o->d.H && pyr_stride == cam->pyr_bytes) {
            if (cam->n_levels != o->d.nlevels) return GFPL_E_INVALID;
            for (int l = 0; l < o->d.nlevels; ++l)
                if (cam->lvl_cols[l] != o->d.lv[l].w || cam->lvl_rows[l] != o->d.lv[l].h ||
                    cam->lvl_offset[l] != o->d.lv[l].off)
                    return GFPL_E_INVALID;
        }
    }
    ORB_HIPCHK(hipSetDevice(o->device));
    OrbDev d = o->d;   // this call's view: the caller's pyramid array is the working pyramid
    if (pyramid) {
        d.pyr = pyramid;
        d.pyr_stride = pyr_stride;
    }
    hipStream_t s = o->stream;
    hipLaunchKernelGGL(k_orb_copy0, dim3(128, n), dim3(256), 0, s, d, images, n);
    for (int l = 1; l < d.nlevels; ++l)
        hipLaunchKernelGGL(k_orb_resize, dim3((d.lv[l].h + RESIZE_ROWS - 1) / RESIZE_ROWS, n), dim3(RESIZE_T),
                           o->resize_lds[l], s, d, l);
    const OrbLevel& L0 = d.lv[0];
    hipLaunchKernelGGL(k_orb_blur, dim3((L0.w + BLUR_TW - 1) / BLUR_TW, (L0.h + BLUR_TH - 1) / BLUR_TH, n * d.nlevels),
                       dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_orb_cellfast, dim3((d.ncell + d.cell_waves - 1) / d.cell_waves, n), dim3(64 * d.cell_waves),
                       4 * d.patch_cap * d.cell_waves, s, d);
    hipLaunchKernelGGL(k_orb_gather, dim3(n * d.nlevels), dim3(GATHER_T), 0, s, d);
    const size_t lds = orb_octree_lds(d.node_cap, d.key_lds);
    hipLaunchKernelGGL(k_orb_octree, dim3(n * d.nlevels), dim3(64), lds, s, d);
    const int max_tot = d.sel_cap * d.nlevels;
    hipLaunchKernelGGL(k_orb_describe, dim3((std::min(max_tot, o->kp_cap) + 7) / 8, n), dim3(256), 0, s, d, n, kps,
                       desc, n_kp, angle, response, o->kp_cap);
    ORB_HIPCHK(hipGetLastError());
    ORB_HIPCHK(o->st.enqueue(s));
    return GFPL_OK;
}

extern "C" int gfpl_orb_status(gfpl_orb* o) {
    if (!o) return GFPL_E_INVALID;
    int bits = 0;
    ORB_HIPCHK(o->st.wait(o->stream, &bits));
    return bits ? GFPL_E_CAPACITY : GFPL_OK;
}

extern "C" int gfpl_orb_extract(gfpl_orb* o, const uint8_t* images, int n, gfpl_keypoint* kps, uint8_t* desc,
                                int* n_kp, float* angle, float* response, uint8_t* pyramid, int64_t pyr_stride) {
    const int e = gfpl_orb_extract_async(o, images, n, kps, desc, n_kp, angle, response, pyramid, pyr_stride);
    if (e) return e;
    return gfpl_orb_status(o);
}
