// k_stereo.hip — stereo matching of one frame per sequence (gfx950).
//
//  k_stereo_points : extractStereoFeatures_ORBSLAM point branch
//                    (src/stereoFrame.cpp:453-630) + subPixelStereoRefine_ORBSLAM (:340-404)
//  k_stereo_lines  : extractStereoFeatures_ORBSLAM line branch (src/stereoFrame.cpp:633-767)
//  k_knn2          : BFMatcher::knnMatch(k=2) NORM_HAMMING / NORM_HAMMING2 (batched)
//  k_init_points / k_init_lines : extractInitialStereoFeatures (src/stereoFrame.cpp:173-336)
//  k_line_uncertainty : estimateStereoUncertainty on a frame slot
//
// One workgroup owns one sequence's frame: the band search, the (dist,iL) sort,
// the median gate and the order-preserving compaction are all block-local, so a
// frame never crosses workgroups and B sequences fill the 256 CUs.
#include <type_traits>

#include "gfpl_kernels.hpp"
#include "gfpl_knn.hpp"

namespace gfpl {

// ---------------------------------------------------------------- helpers
template <typename K>
__device__ void bitonic_sort(K* a, int n) {   // n power of two, ascending
    for (int k = 2; k <= n; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    bool up = ((i & k) == 0);
                    K x = a[i], y = a[ixj];
                    if ((x > y) == up) { a[i] = y; a[ixj] = x; }
                }
            }
            __syncthreads();
        }
}

// two independent arrays through one bitonic network (shared barriers)
template <typename K>
__device__ void bitonic_sort2(K* a, K* c, int n) {
    for (int k = 2; k <= n; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    bool up = ((i & k) == 0);
                    K x = a[i], y = a[ixj];
                    if ((x > y) == up) { a[i] = y; a[ixj] = x; }
                    K u = c[i], v = c[ixj];
                    if ((u > v) == up) { c[i] = v; c[ixj] = u; }
                }
            }
            __syncthreads();
        }
}

__device__ __forceinline__ int clamp_level(int o, int n) { return o < 0 ? 0 : (o >= n ? n - 1 : o); }

// subPixelStereoRefine_ORBSLAM (src/stereoFrame.cpp:340-404); ledger Q1: both
// patches come from the RIGHT pyramid.  SAD of integer-valued pixels is exact,
// so int accumulation equals cv::norm(NORM_L1).  U8: out-of-image windows reject.
//
// Four lanes (a DPP quad) refine one keypoint: lane q sums the 11 shifted SADs
// of window rows q, q+4, q+8 and the quad adds its partial sums (integers: the
// order is immaterial).  A workgroup pass therefore has only BLOCK/4 keypoints
// in flight, consecutive in row order, so its window rows stay in L1/L2 across
// neighbouring keypoints instead of being re-fetched from HBM per keypoint.
struct SadJob {
    const uint8_t* img;   // the pyramid of the sequence (256-B aligned)
    int64_t lvl;          // byte offset of level o in it
    int cols, o, vL, uL, uR;
    float scaleduR0;
};

// window validity (src/stereoFrame.cpp:351-365); false = disparity -1
__device__ __forceinline__ bool sad_setup(const KParams& p, int b, const gfpl_keypoint& kpL, const gfpl_keypoint& kpR,
                                          SadJob& J) {
    const float uR0 = kpR.x;
    const int o = clamp_level(kpL.octave, p.cam.n_levels);
    const float sf = p.cam.inv_scale[o];
    const float scaleduL = roundf(kpL.x * sf);
    const float scaledvL = roundf(kpL.y * sf);
    const float scaleduR0 = roundf(uR0 * sf);
    const int cols = p.cam.lvl_cols[o], rows = p.cam.lvl_rows[o];
    const float iniu = scaleduR0 + 5 - 5;
    const float endu = scaleduR0 + 5 + 5 + 1;
    if (iniu < 0 || endu >= cols) return false;
    const int vL = (int)scaledvL, uL = (int)scaleduL, uR = (int)scaleduR0;
    if (vL - 5 < 0 || vL + 5 >= rows || uL - 5 < 0 || uL + 5 >= cols || uR - 10 < 0 || uR + 10 >= cols) return false;
    J.img = p.in.pyr_r + (size_t)b * (size_t)p.cam.pyr_bytes;
    J.lvl = p.cam.lvl_offset[o];
    J.cols = cols; J.o = o; J.vL = vL; J.uL = uL; J.uR = uR; J.scaleduR0 = scaleduR0;
    return true;
}

// Each window row is read as aligned dwords and re-aligned with v_alignbyte:
// 4 loads for the 11-byte IL row and 6 for the 21-byte IR row instead of 32
// byte loads (the camera's pyramid tail keeps the last dword in bounds).
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ void sad_load_row(const SadJob& J, int y, uint32_t* il4, uint32_t* ir6) {
    // byte offsets from the (256-B aligned) pyramid base: their low 2 bits are the misalignment
    // (integer offsets keep the loads global_load, not flat)
    const int64_t rowo = J.lvl + (int64_t)y * J.cols;
    const int64_t pl = rowo + (J.uL - 5), pr = rowo + (J.uR - 10);
    const uint32_t* wl = reinterpret_cast<const uint32_t*>(J.img + (pl & ~(int64_t)3));
    const uint32_t* wr = reinterpret_cast<const uint32_t*>(J.img + (pr & ~(int64_t)3));
    const uint32_t shl = (uint32_t)(pl & 3), shr = (uint32_t)(pr & 3);
    // dword-aligned 16-B / 8-B vector loads (one load instruction per 4 / 2 dwords)
    const u32x4a4 a = *reinterpret_cast<const u32x4a4*>(wl);
    const u32x4a4 c0 = *reinterpret_cast<const u32x4a4*>(wr);
    const u32x2a4 c1 = *reinterpret_cast<const u32x2a4*>(wr + 4);
    const uint32_t c[6] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y};
    il4[0] = __builtin_amdgcn_alignbyte(a.y, a.x, shl);
    il4[1] = __builtin_amdgcn_alignbyte(a.z, a.y, shl);
    il4[2] = __builtin_amdgcn_alignbyte(a.w, a.z, shl);
#pragma unroll
    for (int i = 0; i < 5; ++i) ir6[i] = __builtin_amdgcn_alignbyte(c[i + 1], c[i], shr);
    ir6[5] = __builtin_amdgcn_alignbyte(c[5], c[5], shr);
}

__device__ __forceinline__ int byte_at(const uint32_t* w, int k) { return (int)((w[k >> 2] >> (8 * (k & 3))) & 0xFFu); }

// bytes c and c + 1 of a little-endian dword array as the two 16-bit halves of one register
// (one v_perm_b32; selector 0x0C yields a zero byte).  c is a compile-time constant.
__device__ __forceinline__ uint32_t pair16(const uint32_t* w, int c) {
    const uint32_t b = (uint32_t)(c & 3);
    if (b < 3) return __builtin_amdgcn_perm(0u, w[c >> 2], 0x0C000C00u | ((b + 1) << 16) | b);
    return __builtin_amdgcn_perm(w[(c >> 2) + 1], w[c >> 2], 0x0C040C03u);   // byte 3 | next dword's byte 0
}
// byte c in both 16-bit halves
__device__ __forceinline__ uint32_t dup16(const uint32_t* w, int c) {
    const uint32_t b = (uint32_t)(c & 3);
    return __builtin_amdgcn_perm(0u, w[c >> 2], 0x0C000C00u | (b << 16) | b);
}

// partial SADs of the window rows q, q+4, q+8 (q = lane within the quad; lane 3
// has no third row: it re-reads the centre row and drops that row's sums).  All
// four rows are loaded before any SAD so their latencies overlap.
// SAD_s = sum |(IL - cL) - (IR_s - cR_s)| = sum |(IL + cR_s) - (IR_s + cL)|, both sides
// <= 510: two columns per v_sad_u16.  Per row the right pairs (IR_c + cL, IR_c+1 + cL) are
// formed once for every column c and the left pairs once; per shift only the left pairs
// take cR_s (the centre pixels cR_s are shared by the lane's rows).
__device__ __forceinline__ void sad_rows(const SadJob& J, int q, uint32_t* acc) {
    uint32_t il4[3][3], ir6[3][6];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int r = q + 4 * i;
        sad_load_row(J, J.vL - 5 + (r < 11 ? r : 5), il4[i], ir6[i]);
    }
    // the centre row (window row 5) is lane 1's second row: its centre pixels cL (IL byte 5)
    // and cR_s (IR bytes 5..15, words 1-3) reach the quad by DPP quad_perm(1,1,1,1)
    uint32_t irc[4];
#pragma unroll
    for (int k = 1; k < 4; ++k) irc[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)ir6[1][k], 0x55, 0xF, 0xF, false);
    irc[0] = 0u;
    const int cL = (int)(((uint32_t)__builtin_amdgcn_mov_dpp((int)il4[1][1], 0x55, 0xF, 0xF, false) >> 8) & 0xFFu);
    const uint32_t cLL = (uint32_t)cL * 0x10001u;
    uint32_t cRR[11];
#pragma unroll
    for (int s = 0; s < 11; ++s) cRR[s] = dup16(irc, 5 + s);   // (cR_s, cR_s)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (q + 4 * i >= 11) break;
        const uint32_t* L = il4[i];
        const uint32_t* R = ir6[i];
        uint32_t ILp[5], RP[19];
#pragma unroll
        for (int k = 0; k < 5; ++k) ILp[k] = pair16(L, 2 * k);
#pragma unroll
        for (int c = 0; c < 19; ++c) RP[c] = pair16(R, c) + cLL;   // (IR_c + cL, IR_c+1 + cL)
        const uint32_t il10 = (uint32_t)byte_at(L, 10);
#pragma unroll
        for (int s = 0; s < 11; ++s) {
            uint32_t a = acc[s];
#pragma unroll
            for (int k = 0; k < 5; ++k) a = __builtin_amdgcn_sad_u16(ILp[k] + cRR[s], RP[s + 2 * k], a);
            // column 10: one 16-bit half (IR_{10+s} + cL is the low half of pair 10 + s)
            const uint32_t rt = (s + 10 < 19 ? RP[s + 10] : pair16(R, s + 10) + cLL) & 0xFFFFu;
            a = __builtin_amdgcn_sad_u16(il10 + (cRR[s] & 0xFFFFu), rt, a);
            acc[s] = a;
        }
    }
}

// best shift, parabola fit, disparity (src/stereoFrame.cpp:384-403)
__device__ __forceinline__ void sad_finish(const KParams& p, const SadJob& J, float xL,
                                           const uint32_t* acc, float& disparity, float& bestuR) {
    int bestDist = 2147483647;
    int bestinc = 0;
    float vD[11];
#pragma unroll
    for (int s = 0; s < 11; ++s) {
        float dist = (float)(int)acc[s];
        if (dist < (float)bestDist) { bestDist = (int)dist; bestinc = s - 5; }
        vD[s] = dist;
    }
    if (bestinc == -5 || bestinc == 5) return;
    const float dist1 = vD[5 + bestinc - 1];
    const float dist2 = vD[5 + bestinc];
    const float dist3 = vD[5 + bestinc + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) return;
    bestuR = p.cam.scale[J.o] * ((float)J.scaleduR0 + (float)bestinc + deltaR);
    disparity = (xL - bestuR);
}

// ------------------------------------------------------- stereo points --
#ifndef GFPL_SL_WAVES
#define GFPL_SL_WAVES 1
#endif
#ifndef GFPL_SP_WAVES
#define GFPL_SP_WAVES 6   // waves per SIMD: <= 84 VGPRs; LDS holds three 512-thread workgroups per CU (6 waves per SIMD)
#endif
#define SP_CHUNK 32       // sorted right-keypoint entries per staged descriptor chunk (k_stereo_points, SEG)
#ifndef GFPL_SP_TY
#define GFPL_SP_TY 3      // SAD job tiles (SEG): 2^TY rows x 2^TX columns, coarser when the bins exceed 4094
#endif
#ifndef GFPL_SP_TX
#define GFPL_SP_TX 6
#endif
#define SP_MINR_PAD 32    // minr bins span [-PAD, H + PAD) (k_stereo_points, SEG): every band is shorter

// LDS-only wave sync: the wave's earlier LDS writes / reads have completed (LDS executes a
// wave's accesses in order; the clobber keeps the compiler from moving accesses across it)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// dynamic LDS: rkey[KP2] u32 | order[KP2] u32 | pairs[KP2] u32 | recx[KP2] f32 |
//              recm[KP2] u16 | rowlo[nRows] u16 | misc[64] i32 | (SEG) stage[waves][SP_CHUNK][32 B]
// Right keypoints are sorted by their row band start (the reference's
// vRowIndices buckets, src/stereoFrame.cpp:459-485) and their x, octave and band
// height are copied next to the sorted keys, so the band scan of a left keypoint
// reads LDS only (its first candidate comes from a per-row table).  Left
// keypoints are processed in row order (order[]), so the lanes of a wave touch the
// same descriptors and overlapping SAD window rows.  Results are keyed by iL: the
// processing order has no effect on the output.
//
// SEG (the 512-thread layout when it fits 40 KB of LDS): the right keypoints are keyed by
// (octave segment, minr, iR) with one first-candidate table per octave, so a left
// keypoint scans only the octaves levelL-1..levelL+1 from their own band start (about
// half the entries of the single sorted list); keypoints whose octave is outside the
// pyramid form one extra segment, searched by bisection when it is not empty.  The
// candidates, hence the lexicographic (dist, iR) minimum, are the same either way.
// diagnostic build (-DGFPL_SP_CLOCK): the phase boundaries' wall clock per sequence (scr.dbg)
// Issue priority by phase (setup 3, band scan 2, sub-pixel SAD 1, emission 0): of two ready waves the
// arbiter favours the older, so without it the workgroups dispatched last trail at the end of the grid
#ifndef GFPL_SP_PRIO
#define GFPL_SP_PRIO 1
#endif
#if GFPL_SP_PRIO
#define SP_PRIO(k) __builtin_amdgcn_s_setprio(k)
#else
#define SP_PRIO(k) do { } while (0)
#endif
#ifdef GFPL_SP_CLOCK
#define SP_CLK(k) do { if (threadIdx.x == 0) p.scr.dbg[8 * (size_t)blockIdx.x + (k)] = (int64_t)wall_clock64(); } while (0)
#else
#define SP_CLK(k) do { } while (0)
#endif
template <int BLOCK, bool SEG>
__global__ void __launch_bounds__(BLOCK, GFPL_SP_WAVES) k_stereo_points(KParams p, int KP2) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int b = blockIdx.x;
    const int cap = p.kp_cap;
    const int nRows = p.cam.height;
    uint32_t* rkey = (uint32_t*)smem;
    uint32_t* order = rkey + KP2;
    uint32_t* pairs = order + KP2;
    float* recx = (float*)(pairs + KP2);
    uint16_t* recm = (uint16_t*)(recx + KP2);
    uint16_t* rowlo = recm + KP2;   // SEG: offr, the bin offsets of the counting sort
    const int nlev = p.cam.n_levels;
    const int NBIN = nRows + 2 * SP_MINR_PAD;   // SEG: minr bins per octave segment
    const int nrl = SEG ? (nlev + 1) * NBIN + 1 : nRows;
    int* misc = (int*)(rowlo + ((nrl + 1) & ~1));   // SEG: [22 + seg] band heights
    // SEG: per-wave staging of right descriptors, SP_CHUNK x 32 B per wave (16-B aligned); an
    // integer offset from smem keeps the pointer in the LDS address space
    uint32_t* stg = (uint32_t*)(smem + ((KP2 * 18 + ((nrl + 1) & ~1) * 2 + 32 * 4 + 15) & ~15));
    // mvDepth of the sub-pixel pass lives in recx: the right keypoints' x are dead once the
    // band scan is over (LDS, no scattered 4-B global stores)
    float* depth = recx;
    const int tid = threadIdx.x;
    SP_CLK(0);
    SP_PRIO(3);
    const int N = min(p.in.n_kp_l[b], cap), Nr = min(p.in.n_kp_r[b], cap);
    const gfpl_keypoint* KL = p.in.kp_l + (size_t)b * cap;
    const gfpl_keypoint* KR = p.in.kp_r + (size_t)b * cap;
    const uint8_t* DL = p.in.pdesc_l + (size_t)b * cap * 32;
    const uint8_t* DR = p.in.pdesc_r + (size_t)b * cap * 32;
    if (SEG) {
        // vRowIndices (src/stereoFrame.cpp:459-485) as a counting sort of the right keypoints
        // by (octave segment, minr) and of the left ones by row: the scan needs the band
        // candidates grouped by minr only (it takes the lexicographic (dist, iR) minimum of
        // every candidate with minr <= row, and stops at the first minr > row), so the order
        // inside a bin — the LDS atomics' — is immaterial, and the bin offsets are the table
        // of each row's first candidate.  minr is binned clamped to [-PAD, H + PAD): rows are
        // in [0, H) and bands are shorter than PAD, so clamping never reorders a candidate
        // across a row's start or stop.  Left keypoints go in row order (the processing
        // order, which has no effect on the output).
        uint32_t* hr = reinterpret_cast<uint32_t*>(rowlo);   // u16 counts, two per word
        uint32_t* hl = stg;                                  // left row counts (u16), in the stage buffer
        const int nbr = (nlev + 1) * NBIN, nbl = nRows + 1;
        for (int w = tid; w < (nbr + 2) / 2; w += BLOCK) hr[w] = 0u;
        for (int w = tid; w < (nbl + 1) / 2; w += BLOCK) hl[w] = 0u;
        if (tid < 32) misc[tid] = 0;
        __syncthreads();
        constexpr int RMAX = 2048 / BLOCK;   // kp_cap <= 2048 on this layout
        uint32_t rk[RMAX], rbr[RMAX], lbr[RMAX];
        float rx[RMAX];      // the record fields, kept from this pass (no second read of KR)
        uint32_t rm[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
            const int i = tid + r * BLOCK;
            rk[r] = 0xFFFFFFFFu;
            rbr[r] = 0u;
            lbr[r] = 0u;
            rx[r] = 0.0f;
            rm[r] = 0u;
            if (i < Nr) {
                const gfpl_keypoint kp = KR[i];
                const float rr = 2.0f * p.cam.scale[clamp_level(kp.octave, nlev)];
                const int maxr = (int)ceilf(kp.y + rr);
                const int minr = (int)floorf(kp.y - rr);
                const int oc = (kp.octave >= -127 && kp.octave <= 127) ? kp.octave : -128;
                rx[r] = kp.x;
                rm[r] = ((uint32_t)(maxr - minr) << 8) | ((uint32_t)oc & 0xFFu);
                const int seg = (kp.octave >= 0 && kp.octave < nlev) ? kp.octave : nlev;
                // rows are < 2048 (GFPL_MAX_IMAGE_DIM): the key keeps minr clamped to [-1024, 3071]
                const int mc = min(max(minr, -1024), 3071);
                rk[r] = ((uint32_t)seg << 28) | ((uint32_t)(mc + 1024) << 16) | (uint32_t)i;
                const int bin = seg * NBIN + min(max(minr + SP_MINR_PAD, 0), NBIN - 1);
                const uint32_t sh = 16u * (uint32_t)(bin & 1);
                const uint32_t old = atomicAdd(&hr[bin >> 1], 1u << sh);
                rbr[r] = (uint32_t)bin | (((old >> sh) & 0xFFFFu) << 16);   // bin | rank in bin
                atomicMax(&misc[22 + seg], maxr - minr);
            }
            if (i < N) {
                const float y = KL[i].y;
                const int row = (y >= 0.0f && y < (float)nRows) ? (int)y + 1 : 0;
                const uint32_t sh = 16u * (uint32_t)(row & 1);
                const uint32_t old = atomicAdd(&hl[row >> 1], 1u << sh);
                lbr[r] = (uint32_t)row | (((old >> sh) & 0xFFFFu) << 16);
            }
            if (i < KP2) pairs[i] = 0xFFFFFFFFu;
        }
        __syncthreads();
        // exclusive scans of both histograms in place (u16 offsets), block-wide
        uint16_t* offr = rowlo;
        uint16_t* offl = reinterpret_cast<uint16_t*>(hl);
        {   // one block scan for both: the right sums in the low, the left in the high 16 bits
            // (each total is at most kp_cap <= 2048, so the halves never carry into each other)
            const int pr = (nbr + BLOCK - 1) / BLOCK, r0 = min(tid * pr, nbr), r1 = min(r0 + pr, nbr);
            const int pq = (nbl + BLOCK - 1) / BLOCK, l0 = min(tid * pq, nbl), l1 = min(l0 + pq, nbl);
            int sr = 0, sl = 0;
            for (int x = r0; x < r1; ++x) sr += offr[x];
            for (int x = l0; x < l1; ++x) sl += offl[x];
            int tot;
            const int run2 = block_exclusive_scan<BLOCK>(sr | (sl << 16), misc + 4, &tot);
            int run = run2 & 0xFFFF;
            for (int x = r0; x < r1; ++x) { const int c = offr[x]; offr[x] = (uint16_t)run; run += c; }
            run = run2 >> 16;
            for (int x = l0; x < l1; ++x) { const int c = offl[x]; offl[x] = (uint16_t)run; run += c; }
            if (tid == 0) offr[nbr] = (uint16_t)(tot & 0xFFFF);
        }
        __syncthreads();
        // scatter: keys with their x, band height maxr - minr and octave (int8; -128 = out
        // of range, read from HBM) side by side; left keypoint indices in row order
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
            const int i = tid + r * BLOCK;
            if (i < Nr) {
                const int j = (int)offr[rbr[r] & 0xFFFFu] + (int)(rbr[r] >> 16);
                rkey[j] = rk[r];
                recx[j] = rx[r];
                recm[j] = (uint16_t)rm[r];
            }
            if (i < N) order[(int)offl[lbr[r] & 0xFFFFu] + (int)(lbr[r] >> 16)] = (uint32_t)i;
        }
        __syncthreads();
    } else {
    if (tid < 32) misc[tid] = 0;
    __syncthreads();
    // vRowIndices as (minr, iR) keys; left keypoints as (row, iL) keys
    for (int i = tid; i < KP2; i += blockDim.x) {
        if (i < Nr) {
            gfpl_keypoint kp = KR[i];
            const float r = 2.0f * p.cam.scale[clamp_level(kp.octave, p.cam.n_levels)];
            const int maxr = (int)ceilf(kp.y + r);
            const int minr = (int)floorf(kp.y - r);
            rkey[i] = ((uint32_t)(minr + 32768) << 16) | (uint32_t)i;
            atomicMax(&misc[0], maxr - minr);
        } else {
            rkey[i] = 0xFFFFFFFFu;
        }
        if (i < N) {
            const float y = KL[i].y;
            const int row = (y >= 0.0f && y < 65534.0f) ? (int)y + 1 : 0;
            order[i] = ((uint32_t)row << 16) | (uint32_t)i;
        } else {
            order[i] = 0xFFFFFFFFu;
        }
        pairs[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    bitonic_sort2(rkey, order, KP2);
    const int D = misc[0];
    // records in sorted order: x, band height maxr - minr (<= 16), octave (int8;
    // -128 = out of range, read from HBM)
    for (int j = tid; j < Nr; j += blockDim.x) {
        const int iR = (int)(rkey[j] & 0xFFFFu);
        const gfpl_keypoint kp = KR[iR];
        const float r = 2.0f * p.cam.scale[clamp_level(kp.octave, p.cam.n_levels)];
        const int band = (int)ceilf(kp.y + r) - (int)floorf(kp.y - r);
        const int oc = (kp.octave >= -127 && kp.octave <= 127) ? kp.octave : -128;
        recx[j] = kp.x;
        recm[j] = (uint16_t)(((uint32_t)band << 8) | ((uint32_t)oc & 0xFFu));
    }
    // first candidate of each row: lower bound of minr >= row - D
    for (int x = tid; x < nrl; x += blockDim.x) {
        int lo = 0, hi = Nr;
        const uint32_t lo_key = (uint32_t)(x - D + 32768) << 16;
        while (lo < hi) { int mid = (lo + hi) >> 1; if (rkey[mid] < lo_key) lo = mid + 1; else hi = mid; }
        rowlo[x] = (uint16_t)lo;
    }
    __syncthreads();
    }
    SP_CLK(1);
    SP_PRIO(2);
    // SEG: first candidate of segment o for a row: the first bin with minr >= row - D_o
    auto seg_start = [&](int o, int row) {
        return (int)rowlo[o * NBIN + min(max(row - misc[22 + o] + SP_MINR_PAD, 0), NBIN - 1)];
    };
    const float minD = 0;
    // (float)fx and (float)(fx b) from the kernel arguments (scalar registers): formed here they
    // sat in VGPRs, and maxD was the kernel's one spill at its 80-register budget
    const float maxD = p.sp_maxD;
    const float mbf = p.sp_mbf;
    // per left keypoint: band search + Hamming (src/stereoFrame.cpp:502-545).  A match
    // leaves (bestDist, bestIdxR) in pairs[iL] and iL in order[t] for the sub-pixel pass;
    // order[t] / pairs[iL] are private to the thread that owns slot t.
    auto finish_kp = [&](int t, int iL, const gfpl_keypoint& kpL, int bestDist, int bestIdxR) {
        uint32_t job = 0xFFFFFFFFu;
#ifdef GFPL_SP_PROBE_NOSAD   // timing probe only (wrong output): no sub-pixel jobs
        if (bestDist < 0) {
#else
        if (bestDist < 80) {
#endif
            atomicAdd(&misc[2], 1);
            SadJob J;
            // job: iL | uL << 16 (order[t]); bestDist | o << 7 | vL << 10 | uR << 21
            // (pairs[iL]); failed window checks keep only bestDist (disparity -1)
            if (sad_setup(p, b, kpL, KR[bestIdxR], J)) {
                pairs[iL] = (uint32_t)bestDist | ((uint32_t)J.o << 7) | ((uint32_t)J.vL << 10) |
                            ((uint32_t)J.uR << 21);
                job = (uint32_t)iL | ((uint32_t)J.uL << 16);
            }
        }
        order[t] = job;
    };
    if (SEG) {
        // Staged scan: a wave takes 64 row-consecutive left keypoints; per octave segment their
        // candidate ranges [rowlo, first minr > row) are walked in chunks of 32 sorted entries
        // whose right descriptors the wave first copies into its own LDS buffer (one 16-B load
        // per lane, all in flight together), so each distance reads LDS instead of a dependent
        // 32-B HBM gather.  Every lane still visits its candidates in ascending sorted order
        // with the same tests: the lexicographic (dist, iR) minimum is unchanged.
        const int lane = tid & 63;
        // explicitly LDS-qualified (a generic pointer here compiled to flat_load / flat_store)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
        lds_u32x4* wst = (lds_u32x4*)(stg + (tid >> 6) * (SP_CHUNK * 8));
        for (int base = tid & ~63; base < N; base += BLOCK) {
            const int t = base + lane;
            const int iL = t < N ? (int)(order[t] & 0xFFFFu) : 0;
            const gfpl_keypoint kpL = KL[iL];
            const int levelL = kpL.octave;
            const float vL = kpL.y, uL = kpL.x;
            const float minU = uL - maxD, maxU = uL - minD;
            const bool act = t < N && vL >= 0.0f && (unsigned)(int)vL < (unsigned)nRows && !(maxU < 0);
            const int row = act ? (int)vL : 0;
            uint32_t dl[8];
            load_desc(DL + (size_t)iL * 32, dl);
            // lexicographic (dist, iR) minimum as one packed key (iR < 2^16 on this layout);
            // the start value keeps bestDist = 100 (no candidate below it: no match)
            uint32_t best = (100u << 16) | 0xFFFFu;
            for (int o = 0; o <= nlev; ++o) {   // wave-uniform
                const bool need = act && (o < nlev ? ((long long)o >= (long long)levelL - 1 &&
                                                      (long long)o <= (long long)levelL + 1)
                                                   : rowlo[(nlev + 1) * NBIN] > rowlo[nlev * NBIN]);
                if (!__any(need)) continue;
                // candidates of segment o with minr in [row - D_o, row]: from the bin of row - D_o to
                // the bin of row + 1 (the counting sort's offsets), so the walk needs no stop test
                int j = need ? seg_start(o, row) : 0;
                const int jend = need ? (int)rowlo[o * NBIN + row + 1 + SP_MINR_PAD] : 0;
                bool more = j < jend;
                // segment o < nlev holds only octave-o keypoints, and a lane walks it only when o is
                // within levelL +- 1: the octave test is the out-of-range segment's alone
                auto walk = [&](auto oseg) {
                    while (__any(more)) {
                        // the chunk starts at the smallest pending j, which is the first pending
                        // lane's: lanes are in row order and the band bounds grow with the row, so
                        // the pending lanes' j never decrease with the lane index
                        const int c0 = __builtin_amdgcn_readlane(j, __builtin_ctzll(__ballot(more)));
                        {
                            const int je = c0 + (lane >> 1);
                            if (je < Nr && (rkey[je] >> 28) == (uint32_t)o) {
                                const int iR = (int)(rkey[je] & 0xFFFFu);
                                wst[lane] = *reinterpret_cast<const u32x4*>(DR + (size_t)iR * 32 + 16 * (lane & 1));   // entry lane >> 1, half lane & 1
                            }
                        }
                        wave_lds_sync();
                        const int jl = min(c0 + SP_CHUNK, jend);
                        for (; j < jl; ++j) {
                            // every LDS read of the entry issued together: one round trip per candidate
                            const uint32_t k = rkey[j];
                            const uint32_t m = recm[j];
                            const float uR = recx[j];
                            const u32x4 a = wst[2 * (j - c0)], c = wst[2 * (j - c0) + 1];
                            const int minr = (int)((k >> 16) & 0xFFFu) - 1024;
                            const int iR = (int)(k & 0xFFFFu);
                            const uint32_t dr[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#ifdef GFPL_SP_PROBE_NOHAM   // timing probe only (wrong output): the band scan without its distances
                            const uint32_t key = ((uint32_t)(90 + (dr[0] & dl[0] & 1u)) << 16) | (uint32_t)iR;
#else
                            const uint32_t key = ((uint32_t)hamming8<1>(dl, dr) << 16) | (uint32_t)iR;
#endif
                            // the tests as one mask and the minimum as a select: no branch around the distance
                            bool pass = (minr + (int)(m >> 8) >= row) & (uR >= minU) & (uR <= maxU);   // maxr >= row
                            if (!decltype(oseg)::value) {
                                int octR = (int)(int8_t)(uint8_t)(m & 0xFFu);
                                if (octR == -128) octR = KR[iR].octave;
                                pass = pass & (octR >= levelL - 1) & (octR <= levelL + 1);
                            }
                            best = min(best, pass ? key : 0xFFFFFFFFu);
                        }
                        more = j < jend;
                        wave_lds_sync();   // the chunk is read before the next one overwrites it
                    }
                };
                if (o < nlev) walk(std::true_type{});
                else walk(std::false_type{});
            }
            const int bestDist = (int)(best >> 16), bestIdxR = (int)(best & 0xFFFFu);
#ifdef GFPL_SP_PROBE_NOSAD   // (keeps the scan live: its keys folded into a diagnostic word)
            {
                uint32_t xk = best;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) xk ^= __shfl_xor(xk, o);
                if (lane == 0) p.scr.dbg[8 * (size_t)b + 7] += (int64_t)xk;
            }
#endif
            if (t < N) finish_kp(t, iL, kpL, bestDist, bestIdxR);
        }
    } else {
    for (int t = tid; t < N; t += blockDim.x) {
        const int iL = (int)(order[t] & 0xFFFFu);
        const gfpl_keypoint kpL = KL[iL];
        int bestDist = 100, bestIdxR = 0x7FFFFFFF;
        {
            const int levelL = kpL.octave;
            const float vL = kpL.y, uL = kpL.x;
            const float minU = uL - maxD, maxU = uL - minD;
            if (vL >= 0.0f && (unsigned)(int)vL < (unsigned)nRows && !(maxU < 0)) {
                const int row = (int)vL;
                uint32_t dl[8];
                load_desc(DL + (size_t)iL * 32, dl);
                for (int j = rowlo[row]; j < Nr; ++j) {
                    const uint32_t k = rkey[j];
                    const int minr = (int)(k >> 16) - 32768;
                    if (minr > row) break;
                    const uint32_t m = recm[j];
                    if (minr + (int)(m >> 8) < row) continue;   // maxr < row
                    const int iR = (int)(k & 0xFFFFu);
                    int octR = (int)(int8_t)(uint8_t)(m & 0xFFu);
                    if (octR == -128) octR = KR[iR].octave;
                    if (octR < levelL - 1 || octR > levelL + 1) continue;
                    const float uR = recx[j];
                    if (uR >= minU && uR <= maxU) {
                        uint32_t dr[8];
                        load_desc(DR + (size_t)iR * 32, dr);
                        const int dist = hamming8<1>(dl, dr);
                        // scan order of the reference is ascending iR with strict '<':
                        // lexicographic (dist, iR) minimum
                        if (dist < bestDist || (dist == bestDist && iR < bestIdxR)) { bestDist = dist; bestIdxR = iR; }
                    }
                }
            }
        }
        finish_kp(t, iL, kpL, bestDist, bestIdxR);
    }
    }
    __syncthreads();
    SP_CLK(2);
    SP_PRIO(1);
    // SEG: the SAD jobs counting-sorted by the tile of their window — (level, 8-row band,
    // 64-px column strip), coarser on large images so the tiles fit 4096 bins — so the 16 quads
    // of a wave read overlapping window rows (one cache line serves several lanes) instead of
    // 16 windows spread across the image width.  Each job refines its own keypoint: the order
    // has no effect on the output.
    const uint32_t* jobs = order;
    int njobs = N;
    if (SEG) {
        uint32_t* sj = rkey;                 // sorted jobs (rkey is dead after the band scan)
        uint32_t* hb = stg;                  // u16 tile counts, two per word (the stage buffers are dead)
        int ty = GFPL_SP_TY, tx = GFPL_SP_TX;   // log2 of the tile's rows / columns (8 x 64 px)
        auto nbins = [&](int a, int c) {
            return nlev * (((p.cam.lvl_rows[0] - 1) >> a) + 1) * (((p.cam.lvl_cols[0] - 1) >> c) + 1);
        };
        while (nbins(ty, tx) > 4094) { if (ty + 3 <= tx) ++ty; else ++tx; }   // (nb + 2) / 2 words <= 2048
        const int TY = ((p.cam.lvl_rows[0] - 1) >> ty) + 1, TX = ((p.cam.lvl_cols[0] - 1) >> tx) + 1;
        const int nb = nlev * TY * TX;
        for (int w = tid; w < (nb + 2) / 2; w += BLOCK) hb[w] = 0u;
        __syncthreads();
        constexpr int RMAX = 2048 / BLOCK;
        uint32_t jb[RMAX], jr[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
            const int i = tid + r * BLOCK;
            jb[r] = 0xFFFFFFFFu;
            jr[r] = 0u;
            if (i < N) {
                const uint32_t job = order[i];
                if (job != 0xFFFFFFFFu) {
                    const uint32_t pr = pairs[job & 0xFFFFu];
                    const int o = (int)((pr >> 7) & 7u), vL = (int)((pr >> 10) & 0x7FFu), uL = (int)(job >> 16);
                    const int bin = (o * TY + min(vL >> ty, TY - 1)) * TX + min(uL >> tx, TX - 1);
                    const uint32_t sh = 16u * (uint32_t)(bin & 1);
                    const uint32_t old = atomicAdd(&hb[bin >> 1], 1u << sh);
                    jb[r] = job;
                    jr[r] = (uint32_t)bin | (((old >> sh) & 0xFFFFu) << 16);
                }
            }
        }
        __syncthreads();
        uint16_t* off = reinterpret_cast<uint16_t*>(hb);
        {
            const int per = (nb + BLOCK - 1) / BLOCK, b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
            int sum = 0;
            for (int x = b0; x < b1; ++x) sum += off[x];
            int tot;
            int run = block_exclusive_scan<BLOCK>(sum, misc + 4, &tot);
            for (int x = b0; x < b1; ++x) { const int c = off[x]; off[x] = (uint16_t)run; run += c; }
            njobs = tot;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
            if (jb[r] != 0xFFFFFFFFu) sj[(int)off[jr[r] & 0xFFFFu] + (int)(jr[r] >> 16)] = jb[r];
        __syncthreads();
        SP_CLK(3);
        jobs = sj;
    }
    // sub-pixel refinement + disparity gate (src/stereoFrame.cpp:547-583), one DPP quad
    // per matched keypoint, BLOCK/4 consecutive (tile- or row-ordered) keypoints per pass
    for (int base = 0; base < njobs; base += BLOCK / 4) {
        const int t = base + (tid >> 2), q = tid & 3;
        const uint32_t job = (t < njobs) ? jobs[t] : 0xFFFFFFFFu;
        uint32_t acc[11];
#pragma unroll
        for (int s = 0; s < 11; ++s) acc[s] = 0;
        SadJob J;
        float xL = 0.0f;
        uint32_t pr = 0;
        if (job != 0xFFFFFFFFu) {
            const int iL = (int)(job & 0xFFFFu);
            xL = KL[iL].x;
            pr = pairs[iL];
            J.o = (int)((pr >> 7) & 7u);
            J.vL = (int)((pr >> 10) & 0x7FFu);
            J.uR = (int)(pr >> 21);
            J.uL = (int)(job >> 16);
            J.cols = p.cam.lvl_cols[J.o];
            J.img = p.in.pyr_r + (size_t)b * (size_t)p.cam.pyr_bytes;
            J.lvl = p.cam.lvl_offset[J.o];
            J.scaleduR0 = (float)J.uR;
#ifdef GFPL_SP_PROBE_SAMEWIN   // timing probe only (wrong output): every job reads one window (L1 hits)
            J.o = 0; J.vL = 20; J.uL = 60; J.uR = 40;
            J.cols = p.cam.lvl_cols[0]; J.lvl = p.cam.lvl_offset[0];
#endif
            sad_rows(J, q, acc);
        }
#pragma unroll
        for (int s = 0; s < 11; ++s) {
            uint32_t v = acc[s];
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad xor 1
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad xor 2
            acc[s] = v;
        }
        if (job != 0xFFFFFFFFu && q == 0) {
            const int iL = (int)(job & 0xFFFFu);
            float disparity = -1, bestuR;
            sad_finish(p, J, xL, acc, disparity, bestuR);
            uint32_t key = 0xFFFFFFFFu;
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) { disparity = 0.01f; bestuR = (float)((double)xL - 0.01); }
                depth[iL] = mbf / disparity;
                key = ((pr & 0x7Fu) << 16) | (uint32_t)iL;
            }
            pairs[iL] = key;
        }
    }
    __syncthreads();
    SP_CLK(4);
    SP_PRIO(0);
    // sort(vDistIdx) (src/stereoFrame.cpp:585): the (dist, iL) keys ascending
    uint32_t* keys = pairs;
    if (SEG) {
        // A stable counting sort by dist (< 128) of the keys in iL order — the order sorting
        // the (dist, iL) pairs gives.  Ranks among equal dists: within a wave by ballots (a
        // multisplit on the 7 dist bits), across the waves of a round and across rounds (iL
        // ascending) by per-dist counters; the sorted keys go to order[] (free after the SAD).
        constexpr int NW = BLOCK / 64;
        int* cnt = reinterpret_cast<int*>(stg);   // [128] dist counts -> running offsets
        int* wcnt = cnt + 128;                    // [NW][128] this round's per-wave counts
        for (int x = tid; x < 128 * (NW + 1); x += BLOCK) cnt[x] = 0;
        __syncthreads();
        for (int i = tid; i < N; i += BLOCK) {   // (keys live at iL < N; the rest stay ~0)
            const uint32_t k = pairs[i];
            if (k != 0xFFFFFFFFu) atomicAdd(&cnt[k >> 16], 1);
        }
        __syncthreads();
        if (tid < 64) {   // exclusive scan of the 128 counts, two per lane
            const int c0 = cnt[2 * tid], c1 = cnt[2 * tid + 1];
            int x = c0 + c1;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o, 64);
                if (tid >= o) x += y;
            }
            const int ex = x - (c0 + c1);
            cnt[2 * tid] = ex;
            cnt[2 * tid + 1] = ex + c0;
            if (tid == 63) misc[1] = x;   // valid keys
        }
        __syncthreads();
        const int wave = tid >> 6, lane = tid & 63;
        const unsigned long long lt = (1ull << lane) - 1ull;
        keys = order;
        for (int r0 = 0; r0 < N; r0 += BLOCK) {   // block-uniform
            const int i = r0 + tid;
            const uint32_t k = i < N ? pairs[i] : 0xFFFFFFFFu;
            const bool v = k != 0xFFFFFFFFu;
            const int d = (int)(k >> 16) & 127;
            unsigned long long peers = __ballot(v);
#pragma unroll
            for (int bit = 0; bit < 7; ++bit) {
                const bool on = (d >> bit) & 1;
                const unsigned long long m = __ballot(on);
                peers &= on ? m : ~m;
            }
            const int rnk = __popcll(peers & lt);
            if (v && rnk == 0) wcnt[wave * 128 + d] = __popcll(peers);
            __syncthreads();
            if (v) {
                int pos = cnt[d] + rnk;
                for (int w = 0; w < wave; ++w) pos += wcnt[w * 128 + d];
                keys[pos] = k;
            }
            __syncthreads();
            if (tid < 128) {
                int sum = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) { sum += wcnt[w * 128 + tid]; wcnt[w * 128 + tid] = 0; }
                cnt[tid] += sum;
            }
            __syncthreads();
        }
    } else {
        bitonic_sort(pairs, KP2);
        for (int i = tid; i < KP2; i += blockDim.x) {
            bool v = pairs[i] != 0xFFFFFFFFu;
            bool vn = (i + 1 < KP2) ? (pairs[i + 1] != 0xFFFFFFFFu) : false;
            if (v && !vn) misc[1] = i + 1;
        }
        __syncthreads();
    }
    const int nv = misc[1];
    float thDist = 0.0f;
    if (nv > 0) {
        const float median = (float)(keys[nv / 2] >> 16);
        thDist = 1.5f * 1.4f * median;
    }
    // emission in sorted order while dist < thDist, skipping negative disparities
    // (src/stereoFrame.cpp:600-626); U5: empty -> no points
    DevPoints& C = p.curr.pt;
    const size_t base = (size_t)b * cap;
    int off = 0;
    for (int c0 = 0; c0 < nv; c0 += BLOCK) {   // block-uniform
        const int i = c0 + tid;
        int flag = 0;
        float disparity = 0.0f;
        int iL = 0;
        if (i < nv) {
            const uint32_t k = keys[i];
            const int dist = (int)(k >> 16);
            iL = (int)(k & 0xFFFFu);
            if ((float)dist < thDist) {
                disparity = mbf / depth[iL];   // Q6: float round trip
                flag = (disparity < 0) ? 0 : 1;
            }
        }
        int tot;
        const int pos = off + block_exclusive_scan<BLOCK>(flag, misc + 4, &tot);
        if (flag) {
            const gfpl_keypoint kp = KL[iL];
            const size_t q = base + pos;
            const double plx = kp.x, ply = kp.y, disp = (double)disparity;
            double P[3];
            backProjection(p.cam, plx, ply, disp, P);
            C.pl[2 * q] = plx; C.pl[2 * q + 1] = ply;
            C.disp[q] = disp;
            C.P[3 * q] = P[0]; C.P[3 * q + 1] = P[1]; C.P[3 * q + 2] = P[2];
            const int lv = clamp_level(kp.octave, p.cam.n_levels);
            C.sigma2[q] = p.cam.sigma2_pt[lv];
            C.idx[q] = pos;
            C.level[q] = kp.octave;
            C.inlier[q] = 1;
            const uint4* s = reinterpret_cast<const uint4*>(DL + (size_t)iL * 32);
            uint4* d = reinterpret_cast<uint4*>(C.desc + q * 32);
            d[0] = s[0]; d[1] = s[1];
        }
        off += tot;
    }
    if (tid == 0) {
        C.n[b] = off;
        p.curr.pose.time_stamp[b] = p.in.time_stamp[b];
        p.scr.n_subpix[b] = misc[2];
    }
    SP_CLK(5);
}

// ------------------------------------------------------- stereo lines --
#ifndef GFPL_SL_PRIO
#define GFPL_SL_PRIO 1
#endif
#if GFPL_SL_PRIO
#define SL_PRIO(k) __builtin_amdgcn_s_setprio(k)
#else
#define SL_PRIO(k) do { } while (0)
#endif
struct LineOut {
    double spl[2], epl[2], sdisp, edisp, sP[3], eP[3], le[3], angle;
    int level;
};

// The line gate's test "largest eigenvalue < th" (src/stereoFrame.cpp:743-751, 992-1000) settled
// without the eigenvalues when bounds decide it the way eig_sym's values would: 1 = the largest value
// eig_sym returns is < th, 0 = it is >= th, -1 = open (non-finite entries, or th inside the bounds).
//  * >= th: a Jacobi rotation turns the (p, q) diagonal pair into app - t apq, aqq + t apq with
//    t apq of the sign of aqq - app, so the larger entry only grows (rounding is monotone): the
//    largest returned value is >= max_i c_ii.
//  * < th: every returned value is a diagonal entry of an orthogonal similarity of C up to the
//    rotations' rounding (<= 150 rotations, ~1e-13 M), hence <= Gershgorin's max_i (c_ii +
//    sum_j |c_ij|) + 4e-9 M, M = max |c_ij|.
__device__ __forceinline__ int eig_gate_bound(const double* C, double th) {
    double M = 0.0, G = -__builtin_inf(), D = -__builtin_inf();
    bool fin = true;
#pragma unroll
    for (int i = 0; i < 9; ++i) { fin = fin && (C[i] - C[i] == 0.0); M = fmax(M, fabs(C[i])); }
    if (!fin) return -1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double d = C[4 * i];
        const double r = (d + fabs(C[3 * i + (i + 1) % 3])) + fabs(C[3 * i + (i + 2) % 3]);
        G = fmax(G, r);
        D = fmax(D, d);
    }
    if (D >= th) return 0;
    if (G + 4e-9 * M < th) return 1;
    return -1;
}

// Line triangulation: initial (src/stereoFrame.cpp:301-330) / per-frame (:684-760)
__device__ bool triangulate(const KParams& p, const gfpl_keyline& a, const gfpl_keyline& c, bool initial,
                            LineOut* L) {
    const DevCam& cam = p.cam;
    double sp_l[3] = {a.sx, a.sy, 1.0}, ep_l[3] = {a.ex, a.ey, 1.0};
    double le_l[3] = {sp_l[1] * ep_l[2] - sp_l[2] * ep_l[1], sp_l[2] * ep_l[0] - sp_l[0] * ep_l[2],
                      sp_l[0] * ep_l[1] - sp_l[1] * ep_l[0]};
    double nrm = sqrt(le_l[0] * le_l[0] + le_l[1] * le_l[1]);
    le_l[0] = le_l[0] / nrm; le_l[1] = le_l[1] / nrm; le_l[2] = le_l[2] / nrm;
    double sp_r[3] = {c.sx, c.sy, 1.0}, ep_r[3] = {c.ex, c.ey, 1.0};
    double le_r[3] = {sp_r[1] * ep_r[2] - sp_r[2] * ep_r[1], sp_r[2] * ep_r[0] - sp_r[0] * ep_r[2],
                      sp_r[0] * ep_r[1] - sp_r[1] * ep_r[0]};
    double overlap = overlapStereo(sp_l[1], ep_l[1], sp_r[1], ep_r[1]);
    double spx = (-(le_r[2] + le_r[1] * (double)a.sy)) / le_r[0];
    double epx = (-(le_r[2] + le_r[1] * (double)a.ey)) / le_r[0];
    double disp_s = (double)a.sx - spx;
    double disp_e = (double)a.ex - epx;
    double horiz = initial ? (double)fabsf((float)le_r[0]) : (double)fabsf((float)le_l[0]);
    if (!(disp_s >= p.cfg.min_disp && disp_e >= p.cfg.min_disp && horiz > p.cfg.line_horiz_th &&
          overlap > p.cfg.stereo_overlap_th))
        return false;
    if (!initial) {
        double cS[9], cE[9];
        endpointCov(cam, sp_l[0], sp_l[1], disp_s, cS);
        endpointCov(cam, ep_l[0], ep_l[1], disp_e, cE);
        // the gate max(largest eigenvalue) < th, from bounds where they settle it (eig_gate_bound),
        // else from eig_sym's values as the oracle takes them
        const double th = p.cfg.line_cov_th;
        const int gS = eig_gate_bound(cS, th), gE = eig_gate_bound(cE, th);
        if (gS == 0 || gE == 0) return false;
        if (!(gS == 1 && gE == 1)) {
            double wS[3], wE[3];
            eig_sym<3>(cS, wS);
            eig_sym<3>(cE, wE);
            double max_eig = std_max(wS[2], wE[2]);
            if (!(max_eig < th)) return false;
        }
    }
    L->spl[0] = sp_l[0]; L->spl[1] = sp_l[1];
    L->epl[0] = ep_l[0]; L->epl[1] = ep_l[1];
    L->sdisp = disp_s; L->edisp = disp_e;
    backProjection(cam, sp_l[0], sp_l[1], disp_s, L->sP);
    backProjection(cam, ep_l[0], ep_l[1], disp_e, L->eP);
    L->le[0] = le_l[0]; L->le[1] = le_l[1]; L->le[2] = le_l[2];
    L->angle = (double)a.angle;
    L->level = a.octave;
    return true;
}

// estimateStereoUncertainty for one line (src/stereoFrame.cpp:1453-1483)
__device__ void line_uncertainty(const KParams& p, const double* spl, const double* epl, double sdisp,
                                 double edisp, const double* le, double* covS, double* covE) {
    double sdisp_std, edisp_std;
    if (fabs(le[0]) > 0.15) {
        sdisp_std = p.cfg.ratio_disp_std * sdisp;
        edisp_std = p.cfg.ratio_disp_std * edisp;
    } else {
        sdisp_std = p.cfg.ratio_disp_std_hor * sdisp;
        edisp_std = p.cfg.ratio_disp_std_hor * edisp;
    }
    covMat2D_3D(p.cam, spl[0], spl[1], 1.0, sdisp, sdisp_std, covS);
    covMat2D_3D(p.cam, epl[0], epl[1], 1.0, edisp, edisp_std, covE);
}

__device__ void write_line(const KParams& p, DevLines& C, size_t q, const LineOut& L, int idx, const uint8_t* desc) {
    C.spl[2 * q] = L.spl[0]; C.spl[2 * q + 1] = L.spl[1];
    C.epl[2 * q] = L.epl[0]; C.epl[2 * q + 1] = L.epl[1];
    C.sdisp[q] = L.sdisp; C.edisp[q] = L.edisp;
    for (int k = 0; k < 3; ++k) { C.sP[3 * q + k] = L.sP[k]; C.eP[3 * q + k] = L.eP[k]; C.le[3 * q + k] = L.le[k]; }
    C.angle[q] = L.angle;
    C.level[q] = L.level;
    C.sigma2[q] = p.cam.sigma2_ln[clamp_level(L.level, GFPL_MAX_LEVELS)];
    C.idx[q] = idx;
    C.inlier[q] = 1;
    C.cut[2 * q] = 0.0; C.cut[2 * q + 1] = 0.0;
    const uint4* s = reinterpret_cast<const uint4*>(desc);
    uint4* d = reinterpret_cast<uint4*>(C.desc + q * 32);
    d[0] = s[0]; d[1] = s[1];
}

// knn-2 of row i of Q against T (both in LDS or global), insertion rule of
// cv::batchDistance (ledger T1): ties keep the lower train index.
template <int CELL>
__device__ __forceinline__ void knn2_row(const uint32_t* q, const uint32_t* T, int nt, int& i0, int& d0, int& d1) {
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

// dynamic LDS: knn LUT | tb[cap*8] u32 (train rows R, knn_stage_views) |
//              lr_i[cap] lr_d0 lr_d1 rl_i | hist[260] | misc[64]
// Query rows stream from HBM into registers; only the train set sits in LDS, so
// 2000 lines per side (config 5) fit.
// diagnostic build (-DGFPL_SL_CLOCK): the phase boundaries' wall clock per sequence (scr.dbg): start,
// train rows staged, knn pass, medians, end (tools/sp_phases.py --lines)
#ifdef GFPL_SL_CLOCK
#define SL_CLK(k) do { if (threadIdx.x == 0 && !INITIAL) p.scr.dbg[8 * (size_t)blockIdx.x + (k)] = (int64_t)wall_clock64(); } while (0)
#else
#define SL_CLK(k) do { } while (0)
#endif
template <int CELL, bool INITIAL, int BLOCK>
__global__ void __launch_bounds__(BLOCK, GFPL_SL_WAVES) k_stereo_lines(KParams p) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int b = blockIdx.x;
    const int cap = p.kl_cap;
    uint32_t* lut = (uint32_t*)smem;   // (first: a compile-time LDS address, folded into the reads' offsets)
    uint32_t* tb = lut + knn_lut_dwords<CELL>();
    int* lr_i = (int*)(tb + cap * 8);
    int* lr_d0 = lr_i + cap;
    int* lr_d1 = lr_d0 + cap;
    int* rl_i = lr_d1 + cap;
    int* hist = rl_i + cap;
    int* misc = hist + 260;
    const int tid = threadIdx.x;
    const int NL = min(p.in.n_kl_l[b], cap), NR = min(p.in.n_kl_r[b], cap);
    DevLines& C = p.curr.ls;   // INITIAL writes the slot passed as curr
    if (NL < 2 || NR < 2) {    // empty -> skipped by the reference; 1 row -> U4 guard
        if (tid == 0) C.n[b] = 0;
        return;
    }
    const uint8_t* DLg = p.in.ldesc_l + (size_t)b * cap * 32;
    const uint8_t* DRg = p.in.ldesc_r + (size_t)b * cap * 32;
    SL_CLK(0);
    SL_PRIO(3);   // issue priority by phase (as k_stereo_points: the last-dispatched workgroups keep up)
    knn_stage_views<CELL>(tb, cap, DRg, NR);
    for (int i = tid; i < 260; i += blockDim.x) hist[i] = 0;
    for (int j = tid; j < NR; j += blockDim.x) rl_i[j] = -1;   // R->L keys (atomicMin)
    knn_lut_fill<CELL>(lut);
    __syncthreads();
    SL_CLK(1);
    // L->R knn-2 on the matrix cores (gfpl_knn.hpp): keys (dist << 16 | iR); the R->L knn
    // (only its best index is used) from the same distance tiles (RL)
    knn2_mfma<CELL, true, true>(tb, cap, NR, DLg, NL, (uint32_t*)lr_i, (uint32_t*)lr_d1, lut, (uint32_t*)rl_i);
    __syncthreads();
    SL_CLK(2);
    SL_PRIO(1);
    for (int i = tid; i < NL; i += blockDim.x) {
        const uint32_t k0 = (uint32_t)lr_i[i], k1 = (uint32_t)lr_d1[i];
        const int d0 = (int)(k0 >> 16), d1 = (int)(k1 >> 16);
        lr_i[i] = (int)(k0 & 0xFFFFu); lr_d0[i] = d0; lr_d1[i] = d1;
        atomicAdd(&hist[d1 - d0], 1);   // lineDescriptorMAD deviations |d1-d0| (U1 pin)
    }
    for (int j = tid; j < NR; j += blockDim.x) rl_i[j] = (int)((uint32_t)rl_i[j] & 0xFFFFu);
    __syncthreads();
    if (tid < 64) {   // (wave 0)
        const int v = wave_hist_rank(hist, NL / 2, 257);
        if (tid == 0) {
            double th = (1.4826 * (double)(float)v) * p.cfg.desc_th_l;
            reinterpret_cast<double*>(misc + 8)[0] = th;
        }
    }
    __syncthreads();
    const double nn12_dist_th = reinterpret_cast<double*>(misc + 8)[0];
    SL_CLK(3);
    const int n_matches = min(NL, NR);   // Q5
    const gfpl_keyline* KL = p.in.kl_l + (size_t)b * cap;
    const gfpl_keyline* KR = p.in.kl_r + (size_t)b * cap;
    const size_t base = (size_t)b * cap;
    int off = 0;
    for (int c0 = 0; c0 < n_matches; c0 += BLOCK) {
        const int i = c0 + tid;
        int flag = 0;
        LineOut L;
        if (i < n_matches) {
            const int lr_tdx = lr_i[i];
            const int rl_tdx = rl_i[lr_tdx];
            const double dist_12 = (double)((float)lr_d1[i] - (float)lr_d0[i]);
            if (i == rl_tdx && dist_12 > nn12_dist_th)
                flag = triangulate(p, KL[i], KR[lr_tdx], INITIAL, &L) ? 1 : 0;
        }
        int tot;
        const int pos = off + block_exclusive_scan<BLOCK>(flag, misc + 16, &tot);
        if (flag) write_line(p, C, base + pos, L, INITIAL ? pos : -1, DLg + (size_t)i * 32);
        off += tot;
    }
    if (tid == 0) C.n[b] = off;
    SL_CLK(4);
}

// ------------------------------------------------------- knn2 (global) --
// rows of q / t of sequence b at q + b*qstride*32 (counts nq[b], nt[b] or fixed)
template <int CELL>
__global__ void __launch_bounds__(256) k_knn2(const uint8_t* q, const int* nq_arr, int nq_fixed, size_t q_stride,
                                             const uint8_t* t, const int* nt_arr, int nt_fixed, size_t t_stride,
                                             int cap_clamp, int32_t* out_idx, float* out_dist, int32_t* packed,
                                             size_t out_stride) {
    const int b = blockIdx.y;
    const int nq = nq_arr ? min(nq_arr[b], cap_clamp) : nq_fixed;
    const int nt = nt_arr ? min(nt_arr[b], cap_clamp) : nt_fixed;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const uint8_t* Q = q + (size_t)b * q_stride * 32;
    const uint8_t* T = t + (size_t)b * t_stride * 32;
    uint32_t qd[8];
    load_desc(Q + (size_t)i * 32, qd);
    int dist0 = 2147483647, dist1 = 2147483647, idx0 = -1, idx1 = -1;
    for (int j = 0; j < nt; ++j) {
        uint32_t td[8];
        load_desc(T + (size_t)j * 32, td);
        const int d = hamming8<CELL>(qd, td);
        if (d < dist1) {
            if (dist0 > d) { dist1 = dist0; idx1 = idx0; dist0 = d; idx0 = j; }
            else { dist1 = d; idx1 = j; }
        }
    }
    if (out_idx) {
        out_idx[2 * i] = idx0; out_idx[2 * i + 1] = idx1;
        out_dist[2 * i] = (float)dist0; out_dist[2 * i + 1] = (float)dist1;
    }
    if (packed) {
        int32_t* o = packed + (size_t)b * out_stride * 3;
        o[3 * i] = idx0; o[3 * i + 1] = dist0; o[3 * i + 2] = dist1;
    }
}

// -------------------------------------------------- initial-frame points --
// src/stereoFrame.cpp:206-245 on knn results in scratch:
//   knn[b][0][i] = (idx0,d0,d1) of L->R, knn[b][1][j] of R->L
__global__ void __launch_bounds__(512) k_init_points(KParams p) {
    __shared__ int misc[32];
    const int b = blockIdx.x;
    const int cap = p.kp_cap;
    const int tid = threadIdx.x;
    DevPoints& C = p.curr.pt;
    const int N = min(p.in.n_kp_l[b], cap), Nr = min(p.in.n_kp_r[b], cap);
    if (N < 2 || Nr < 2) {   // U4 guard
        if (tid == 0) { C.n[b] = 0; p.curr.pose.time_stamp[b] = p.in.time_stamp[b]; }
        return;
    }
    const int32_t* lr = p.scr.knn + (size_t)b * 2 * cap * 3;
    const int32_t* rl = lr + (size_t)cap * 3;
    const gfpl_keypoint* KL = p.in.kp_l + (size_t)b * cap;
    const gfpl_keypoint* KR = p.in.kp_r + (size_t)b * cap;
    const uint8_t* DL = p.in.pdesc_l + (size_t)b * cap * 32;
    const size_t base = (size_t)b * cap;
    int off = 0;
    for (int c0 = 0; c0 < N; c0 += 512) {
        const int i = c0 + tid;
        int flag = 0;
        double disp_ = 0.0;
        if (i < N) {
            const int t = lr[3 * i];
            const int rl_tdx = rl[3 * t];
            const double dist_12 = (double)((float)lr[3 * i + 1] / (float)lr[3 * i + 2]);
            if (i == rl_tdx && dist_12 <= p.cfg.max_ratio_12_p) {
                const gfpl_keypoint kl = KL[i], kr = KR[t];
                if ((double)fabsf(kl.y - kr.y) <= p.cfg.max_dist_epip) {
                    disp_ = (double)(kl.x - kr.x);
                    if (disp_ >= p.cfg.min_disp) flag = 1;
                }
            }
        }
        int tot;
        const int pos = off + block_exclusive_scan<512>(flag, misc, &tot);
        if (flag) {
            const gfpl_keypoint kl = KL[i];
            const size_t q = base + pos;
            double P[3];
            const double plx = kl.x, ply = kl.y;
            backProjection(p.cam, plx, ply, disp_, P);
            C.pl[2 * q] = plx; C.pl[2 * q + 1] = ply;
            C.disp[q] = disp_;
            C.P[3 * q] = P[0]; C.P[3 * q + 1] = P[1]; C.P[3 * q + 2] = P[2];
            C.sigma2[q] = p.cam.sigma2_pt[clamp_level(kl.octave, p.cam.n_levels)];
            C.idx[q] = pos;
            C.level[q] = kl.octave;
            C.inlier[q] = 1;
            const uint4* s = reinterpret_cast<const uint4*>(DL + (size_t)i * 32);
            uint4* d = reinterpret_cast<uint4*>(C.desc + q * 32);
            d[0] = s[0]; d[1] = s[1];
        }
        off += tot;
    }
    if (tid == 0) {
        C.n[b] = off;
        p.curr.pose.time_stamp[b] = p.in.time_stamp[b];
    }
}

// initial pose: Tfw = Tfw_cov = DT = I, DT_cov = 0 (src/stereoFrameHandler.cpp:50-52)
__global__ void k_init_pose(KParams p) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    DevPose& P = p.curr.pose;
    for (int i = 0; i < 16; ++i) { P.Tfw[16 * b + i] = (i % 5 == 0) ? 1.0 : 0.0; P.DT[16 * b + i] = (i % 5 == 0) ? 1.0 : 0.0; }
    for (int i = 0; i < 36; ++i) { P.Tfw_cov[36 * b + i] = (i % 7 == 0) ? 1.0 : 0.0; P.DT_cov[36 * b + i] = 0.0; }
    for (int i = 0; i < 6; ++i) P.DT_cov_eig[6 * b + i] = 0.0;
    P.err_norm[b] = 0.0;
    p.tr.num_frame_loss[b] = 0;
    p.tr.n_matched_pt[b] = 0;
    p.tr.n_matched_ls[b] = 0;
    p.tr.n_inliers[b] = 0; p.tr.n_inliers_pt[b] = 0; p.tr.n_inliers_ls[b] = 0;
    // SLAM variables for KF decision (src/stereoFrameHandler.cpp:54-58)
    for (int i = 0; i < 16; ++i) p.tr.kf_T[16 * b + i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int i = 0; i < 36; ++i) p.tr.kf_cov[36 * b + i] = 0.0;
    p.tr.kf_prev_iskf[b] = 1;
    p.tr.kf_nsince[b] = 0;
    p.tr.kf_entropy0[b] = 0.0;
    p.tr.kf_ratio[b] = 0.0;
    p.tr.kf_flag[b] = 0;
}

// estimateStereoUncertainty on the slot passed as `prev`
// lane per line; the two 9-double covariances go through LDS so the block writes its
// lines' covS / covE ranges with consecutive lanes on consecutive doubles
__global__ void __launch_bounds__(256) k_line_uncertainty(KParams p) {
    __shared__ double cs[256 * 9], ce[256 * 9];
    const int b = blockIdx.y;
    const int i0 = blockIdx.x * blockDim.x;
    const int i = i0 + threadIdx.x;
    DevLines& L = p.prev.ls;
    const int n = L.n[b];
    if (i0 >= n) return;   // uniform per block
    if (i < n) {
        const size_t q = (size_t)b * p.kl_cap + i;
        double spl[2] = {L.spl[2 * q], L.spl[2 * q + 1]}, epl[2] = {L.epl[2 * q], L.epl[2 * q + 1]};
        double le[3] = {L.le[3 * q], L.le[3 * q + 1], L.le[3 * q + 2]};
        double cS[9], cE[9];
        line_uncertainty(p, spl, epl, L.sdisp[q], L.edisp[q], le, cS, cE);
#pragma unroll
        for (int k = 0; k < 9; ++k) { cs[9 * threadIdx.x + k] = cS[k]; ce[9 * threadIdx.x + k] = cE[k]; }
    }
    __syncthreads();
    const int m = 9 * min(256, n - i0);
    double* dS = L.covS + 9 * ((size_t)b * p.kl_cap + i0);
    double* dE = L.covE + 9 * ((size_t)b * p.kl_cap + i0);
    for (int k = threadIdx.x; k < m; k += 256) { dS[k] = cs[k]; dE[k] = ce[k]; }
}

// Algorithmic HBM bytes of one step of one sequence, per stage (DESIGN.md
// §Roofline): the bytes each stage must read or write at minimum, from the
// runtime counts.  bytes[b*STEP_REC + s], s = 0 stereo_points, 1 stereo_lines,
// 2 cross_points (+ prev line uncertainty), 3 cross_lines, 4 line_cut, 5 pose,
// 6 total, 7 k_cut_search; 8-15 the counts they are priced on.
__global__ void k_step_bytes(KParams p) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    const int64_t No = (int64_t)p.in.n_kp_l[b] + p.in.n_kp_r[b];
    const int64_t Nk = (int64_t)p.in.n_kl_l[b] + p.in.n_kl_r[b];
    const int64_t Mo = p.scr.n_subpix[b];
    const int64_t Sp = p.prev.pt.n[b], Sl = p.prev.ls.n[b];
    const int64_t Sp2 = p.curr.pt.n[b], Sl2 = p.curr.ls.n[b];
    const int64_t Mp = p.tr.n_matched_pt[b], Ml = p.tr.n_matched_ls[b];
    int64_t st[6];
    st[0] = 44 * No + (121 + 231) * Mo + 97 * Sp2;          // kps+descs, SAD windows, curr points
    st[1] = 56 * Nk + 193 * Sl2;                             // keylines+descs, curr lines
    st[2] = 216 * Sl + 60 * Sp + 48 * Sp2 + 25 * Mp + 256;   // uncertainty, projections, radius/gate, lists
    st[3] = 36 * Sl + 32 * Sl2 + 153 * Ml;                   // line knn both ways, obs copy, lists
    st[4] = 608 * Ml + 44 * Mp;                              // cut: line/point info inputs, cut endpoints + invCov
    st[5] = 54 * Mp + 86 * Ml + 1504;                        // GN inputs once, inlier flags, pose + covariances
    int64_t tot = 0;
    int64_t* rec = p.scr.bytes + (size_t)STEP_REC * b;
    for (int i = 0; i < 6; ++i) { rec[i] = st[i]; tot += st[i]; }
    rec[6] = tot;
    // k_cut_search alone: per matched line its cut inputs (sP eP covS covE le_obs
    // 208 B + index 4 B), its r = 0 info from k_cut_prep (168 B), the cut ratio
    // written (16 B); per sequence invCov_sum + metric + DT_inv (272 B)
    rec[7] = (p.cfg.use_line_conf_cut && Ml > 0) ? 396 * Ml + 272 : 0;
    // the counts the bytes are priced on (the bench's per-step means)
    rec[8] = No; rec[9] = Nk; rec[10] = Mo; rec[11] = Sp2; rec[12] = Sl2; rec[13] = Mp; rec[14] = Ml;
    rec[15] = p.tr.n_inliers[b];
    if (!(p.cfg.use_line_conf_cut && Ml > 0)) rec[16] = rec[17] = 0;   // k_cut_search writes them otherwise
    rec[18] = rec[15];   // until optimize_pose (k_pose_finish) records its inliers
    if (!(p.cfg.use_line_conf_cut && Ml > 0)) rec[19] = 0;   // k_cut_search writes it otherwise
    // 20-23: the proven line cut's counts (k_cut_verify, cut_proof 1 / 3); zero for a step without it
    if (!(p.cfg.use_line_conf_cut && (p.cfg.cut_proof == 1 || p.cfg.cut_proof == 3)))
        rec[20] = rec[21] = rec[22] = rec[23] = 0;
    // insertStereoPair's last statement, numFrameSinceKeyframe++ (src/stereoFrameHandler.cpp:150):
    // this per-sequence kernel closes every gfpl_insert_stereo_pair
    p.tr.kf_nsince[b] = p.tr.kf_nsince[b] + 1;
}

// ------------------------------------------------------------ launchers --
static inline int next_pow2(int v) { int p = 1; while (p < v) p <<= 1; return p; }

// small batches (B <= SP_WIDE_MAX_B, GFPL_SP_WIDE_MAX_B overrides): one sequence's stereo matching is
// the latency, and a CU holds at most one or two sequences — 16 waves per sequence instead of 8
#ifndef SP_WIDE_MAX_B
#define SP_WIDE_MAX_B 256
#endif
int sp_wide_max_b() {
    const char* e = getenv("GFPL_SP_WIDE_MAX_B");
    return e ? atoi(e) : SP_WIDE_MAX_B;
}

hipError_t launch_stereo_points(const KParams& p, hipStream_t s) {
    const int KP2 = next_pow2(p.kp_cap);
    const size_t lds = (size_t)KP2 * 18 + (size_t)((p.cam.height + 1) & ~1) * 2 + 64 * 4;
    const int nrl_seg = (p.cam.n_levels + 1) * (p.cam.height + 2 * SP_MINR_PAD) + 1;
    const size_t lds_seg = (size_t)KP2 * 18 + (size_t)((nrl_seg + 1) & ~1) * 2 + 32 * 4 + 16 +
                           (size_t)(512 / 64) * SP_CHUNK * 32;
    const size_t lds_seg_w = lds_seg + (size_t)(512 / 64) * SP_CHUNK * 32;   // (16 waves' staging)
    if (p.B <= sp_wide_max_b() && p.kp_cap <= 2048 && lds_seg_w <= 64 * 1024) {
        hipLaunchKernelGGL((k_stereo_points<1024, true>), dim3(p.B), dim3(1024), lds_seg_w, s, p, KP2);
        return hipGetLastError();
    }
    // the large-capacity layout leaves LDS for one workgroup per CU: give it 16 waves
    if (p.kp_cap > 2048)
        hipLaunchKernelGGL((k_stereo_points<1024, false>), dim3(p.B), dim3(1024), lds, s, p, KP2);
    else if (lds_seg <= 54 * 1024 && p.kp_cap <= 2048)   // three workgroups per CU
        hipLaunchKernelGGL((k_stereo_points<512, true>), dim3(p.B), dim3(512), lds_seg, s, p, KP2);
    else
        hipLaunchKernelGGL((k_stereo_points<512, false>), dim3(p.B), dim3(512), lds, s, p, KP2);
    return hipGetLastError();
}

size_t stereo_lines_lds(int cap) { return (size_t)cap * 32 + (size_t)cap * 16 + 260 * 4 + 64 * 4 + 1024 * 4; }

hipError_t launch_stereo_lines(const KParams& p, hipStream_t s) {
    // large-capacity LDS layout (one workgroup per CU) and small batches: 16 waves
    if (p.kl_cap > 1024 || p.B <= sp_wide_max_b())
        hipLaunchKernelGGL((k_stereo_lines<2, false, 1024>), dim3(p.B), dim3(1024), stereo_lines_lds(p.kl_cap), s, p);
    else
        hipLaunchKernelGGL((k_stereo_lines<2, false, 512>), dim3(p.B), dim3(512), stereo_lines_lds(p.kl_cap), s, p);
    return hipGetLastError();
}

hipError_t launch_line_uncertainty(const KParams& p, hipStream_t s) {
    hipLaunchKernelGGL(k_line_uncertainty, dim3((p.kl_cap + 255) / 256, p.B), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_init(const KParams& p, hipStream_t s) {
    // points: knn-2 NORM_HAMMING L->R and R->L into scratch, then gates
    const int cap = p.kp_cap;
    int32_t* lr = p.scr.knn;
    // MFMA knn (gfpl_knn.hpp): 128 queries per workgroup, train rows streamed through LDS
    const dim3 gm((cap + 127) / 128, p.B);
    hipLaunchKernelGGL((k_knn2m<1>), gm, dim3(256), 0, s, p.in.pdesc_l, p.in.n_kp_l, 0, (size_t)cap,
                       p.in.pdesc_r, p.in.n_kp_r, 0, (size_t)cap, cap, (int32_t*)nullptr, (float*)nullptr,
                       lr, (size_t)cap * 2);
    hipLaunchKernelGGL((k_knn2m<1>), gm, dim3(256), 0, s, p.in.pdesc_r, p.in.n_kp_r, 0, (size_t)cap,
                       p.in.pdesc_l, p.in.n_kp_l, 0, (size_t)cap, cap, (int32_t*)nullptr, (float*)nullptr,
                       lr + (size_t)cap * 3, (size_t)cap * 2);
    hipLaunchKernelGGL(k_init_points, dim3(p.B), dim3(512), 0, s, p);
    if (p.kl_cap > 1024)
        hipLaunchKernelGGL((k_stereo_lines<1, true, 1024>), dim3(p.B), dim3(1024), stereo_lines_lds(p.kl_cap), s, p);
    else
        hipLaunchKernelGGL((k_stereo_lines<1, true, 512>), dim3(p.B), dim3(512), stereo_lines_lds(p.kl_cap), s, p);
    hipLaunchKernelGGL(k_init_pose, dim3((p.B + 63) / 64), dim3(64), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_step_bytes(const KParams& p, hipStream_t s) {
    hipLaunchKernelGGL(k_step_bytes, dim3((p.B + 63) / 64), dim3(64), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, int32_t* idx, float* dist,
                       hipStream_t s) {
    if (nt <= 65536) {   // MFMA path: the packed key holds a 16-bit train index
        const dim3 g((nq + 127) / 128, 1);
        if (cell == 2)
            hipLaunchKernelGGL((k_knn2m<2>), g, dim3(256), 0, s, q, (const int*)nullptr, nq, (size_t)0, t,
                               (const int*)nullptr, nt, (size_t)0, 0, idx, dist, (int32_t*)nullptr, (size_t)0);
        else
            hipLaunchKernelGGL((k_knn2m<1>), g, dim3(256), 0, s, q, (const int*)nullptr, nq, (size_t)0, t,
                               (const int*)nullptr, nt, (size_t)0, 0, idx, dist, (int32_t*)nullptr, (size_t)0);
        return hipGetLastError();
    }
    dim3 g((nq + 255) / 256, 1);
    if (cell == 2)
        hipLaunchKernelGGL((k_knn2<2>), g, dim3(256), 0, s, q, (const int*)nullptr, nq, (size_t)0, t,
                           (const int*)nullptr, nt, (size_t)0, 0, idx, dist, (int32_t*)nullptr, (size_t)0);
    else
        hipLaunchKernelGGL((k_knn2<1>), g, dim3(256), 0, s, q, (const int*)nullptr, nq, (size_t)0, t,
                           (const int*)nullptr, nt, (size_t)0, 0, idx, dist, (int32_t*)nullptr, (size_t)0);
    return hipGetLastError();
}

}  // namespace gfpl
