// gfpl_knn.hpp — knn-2 Hamming matching on the matrix cores (gfx950 i8 MFMA).
//
// BFMatcher::knnMatch(k = 2) with NORM_HAMMING / NORM_HAMMING2 (OpenCV 3.4.1
// batchDistance; ledger T1) restated as an exact integer GEMM:
//   HAMMING  : dist(t, q) = popc(t) + popc(q) - 2 <t_bits, q_bits>
//              = <t_bits, 1 - 2 q_bits> + popc(q)            (K = 256, one i8 per bit)
//   HAMMING2 : dist(t, q) = 128 - <onehot(t), onehot(q)>     (K = 512, each 2-bit
//              cell one-hot over its 4 values: equal cells contribute 1; the query
//              side is negated and the accumulator starts at 128)
// v_mfma_i32_32x32x32_i8 takes a 32x32 tile of (train row t) x (query column q)
// per wave; the C layout puts one query column on each lane (col = lane & 31) and
// 16 train rows in its registers (row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)), so
// the per-query top-2 is lane-local.  The top-2 is the lexicographic minimum of
// the packed key (dist << 16 | t) — the OpenCV insertion rule (strict '<', ties
// keep the lower train index) is exactly that, independent of visiting order.
// The k-index each (lane half, element) holds is the same for A and B, so the
// dot products are exact whatever the hardware's k permutation inside a step.
#pragma once
#include "gfpl_device.hpp"
#include <type_traits>

namespace gfpl {

typedef int mfma_v4i __attribute__((ext_vector_type(4)));
typedef int mfma_v16i __attribute__((ext_vector_type(16)));

// 4 bits -> 4 bytes of 0 / 1
__device__ __forceinline__ uint32_t spread4(uint32_t nib) { return (nib * 0x00204081u) & 0x01010101u; }

// operand fragment of k-step ks for a 32-byte descriptor held as 8 dwords.
// CELL 2 (one-hot): lane half h takes descriptor byte 2 ks + h (4 cells -> 16 i8)
// CELL 1 (bits)   : lane half h takes bytes 4 ks + 2 h, +1 (16 bits -> 16 i8).
// SIGNED (query side): CELL 1 maps bit b to 1 - 2 b, CELL 2 makes the one-hot -1.
template <int CELL, bool SIGNED>
__device__ __forceinline__ mfma_v4i knn_frag(const uint32_t* d, int ks, int h) {
    mfma_v4i f;
    if (CELL == 2) {   // byte 2 ks + h lives in dword ks >> 1 (compile-time index)
        const uint32_t v = (d[ks >> 1] >> (8u * (2u * (ks & 1) + (uint32_t)h))) & 0xFFu;
        const uint32_t one = SIGNED ? 0xFFu : 0x01u;   // SIGNED: the one-hot byte is -1
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = (int)(one << (8u * ((v >> (2 * i)) & 3u)));
    } else {           // bytes 4 ks + 2 h, +1 live in dword ks
        const uint32_t v = (d[ks] >> (16u * (uint32_t)h)) & 0xFFFFu;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t x = spread4((v >> (4 * i)) & 0xFu);
            f[i] = SIGNED ? (int)((x * 0xFEu) | 0x01010101u) : (int)x;
        }
    }
    return f;
}

__device__ __forceinline__ int popc8(const uint32_t* d) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += __popc(d[i]);
    return s;
}

// Expansion table for the train (A) side, filled once per workgroup in LDS:
// CELL 2: byte -> 4 dwords of one-hot cells (16 i8); CELL 1: byte -> 2 dwords of bits (8 i8).
template <int CELL>
__device__ void knn_lut_fill(uint32_t* lut) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) {
        if (CELL == 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i) lut[4 * b + i] = 1u << (8u * ((b >> (2 * i)) & 3u));
        } else {
            lut[2 * b] = spread4(b & 0xFu);
            lut[2 * b + 1] = spread4((uint32_t)b >> 4);
        }
    }
}
template <int CELL>
constexpr int knn_lut_dwords() { return CELL == 2 ? 1024 : 512; }

// A fragment of k-step ks from the LUT (same element order as knn_frag).  GFPL_KNN_ALUT 0: formed by
// VALU instead (knn_frag), under the MFMA's cycles, without the LUT's LDS reads and bank conflicts
#ifndef GFPL_KNN_ALUT
#define GFPL_KNN_ALUT 1
#endif
template <int CELL>
__device__ __forceinline__ mfma_v4i knn_frag_lut(const uint32_t* lut, const uint32_t* d, int ks, int h) {
    if (!GFPL_KNN_ALUT) return knn_frag<CELL, false>(d, ks, h);
    mfma_v4i f;
    if (CELL == 2) {
        const uint32_t v = (d[ks >> 1] >> (8u * (2u * (ks & 1) + (uint32_t)h))) & 0xFFu;
        const uint4 e = *reinterpret_cast<const uint4*>(lut + 4 * v);
        f[0] = (int)e.x; f[1] = (int)e.y; f[2] = (int)e.z; f[3] = (int)e.w;
    } else {
        const uint32_t v = (d[ks] >> (16u * (uint32_t)h)) & 0xFFFFu;
        const uint2 lo = *reinterpret_cast<const uint2*>(lut + 2 * (v & 0xFFu));
        const uint2 hi = *reinterpret_cast<const uint2*>(lut + 2 * (v >> 8));
        f[0] = (int)lo.x; f[1] = (int)lo.y; f[2] = (int)hi.x; f[3] = (int)hi.y;
    }
    return f;
}

// Stage nt descriptor rows (32 B each, global) into LDS as structure-of-arrays:
// dword i of row t at T[i * stride + t], so a wave reading 32 consecutive rows
// touches consecutive banks.
__device__ __forceinline__ void knn_stage_soa(uint32_t* T, int stride, const uint8_t* src, int nt) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    for (int k = threadIdx.x; k < nt * 2; k += blockDim.x) {   // coalesced 16-B reads
        const uint4 v = s4[k];
        const int t = k >> 1, i0 = (k & 1) * 4;
        T[(i0 + 0) * stride + t] = v.x;
        T[(i0 + 1) * stride + t] = v.y;
        T[(i0 + 2) * stride + t] = v.z;
        T[(i0 + 3) * stride + t] = v.w;
    }
}

// Train rows for knn2_mfma, staged once per workgroup as per-lane-half views: the A fragment of
// k-step ks on lane half h takes descriptor byte 2 ks + h (CELL 2) or bytes 4 ks + 2 h, +1 (CELL 1),
// so view h of row t holds, in its dwords j = 0..3, exactly the bytes half h reads for k-steps
// 4j..4j+3 (CELL 2) / 2j, 2j+1 (CELL 1), in k-step order: V[(4 h + j) * stride + t].  A lane then
// reads its row's 16 bytes (4 dwords) per tile, and every fragment byte sits at a compile-time
// position of a view dword (no lane-dependent shifts).
template <int CELL>
__device__ __forceinline__ void knn_stage_views(uint32_t* T, int stride, const uint8_t* src, int nt) {
    constexpr uint32_t S0 = CELL == 2 ? 0x06040200u : 0x05040100u;   // v_perm selectors: bytes of (d[2j+1]:d[2j])
    constexpr uint32_t S1 = CELL == 2 ? 0x07050301u : 0x07060302u;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    for (int k = threadIdx.x; k < nt * 2; k += blockDim.x) {   // coalesced 16-B reads: dwords 4p .. 4p+3 of row t
        const uint4 v = s4[k];
        const int t = k >> 1, j = (k & 1) * 2;
        T[(0 + j) * stride + t] = __builtin_amdgcn_perm(v.y, v.x, S0);
        T[(1 + j) * stride + t] = __builtin_amdgcn_perm(v.w, v.z, S0);
        T[(4 + j) * stride + t] = __builtin_amdgcn_perm(v.y, v.x, S1);
        T[(5 + j) * stride + t] = __builtin_amdgcn_perm(v.w, v.z, S1);
    }
}

// One knn pass of a workgroup: every query q < nq against the train rows of T (LDS,
// knn_stage_views).  Queries are read from Q (global, 32-byte rows).  Writes out_k0[q] =
// lexicographic minimum key (dist << 16 | t) and, when TOP2, out_k1[q] = the second one.  Waves
// split the query column tiles.  The accumulator starts at 0 (the first MFMA takes an inline
// constant) and the distance offset (128 for HAMMING2 with the query one-hot negated, popc(q) for
// HAMMING) is added with the keys: acc + off is the distance, and (acc << 16) + (off << 16) its
// key bits (mod 2^32).
// lut: knn_lut_fill<CELL> table in LDS — at LDS address 0 (the start of the caller's dynamic LDS,
// with no static LDS in the kernel): the reads use that address directly.
// inlined into its callers: as a called function its register save area sat in
// scratch and capped k_stereo_lines at 128 VGPRs (inlined: 121, no scratch; 4.95 -> 4.27 ms)
#ifndef GFPL_KNN_INLINE
#define GFPL_KNN_INLINE __forceinline__
#endif
// RL (the reverse direction in the same pass): Hamming distance is symmetric, so tile
// (t, q) also holds the train-side query's distances — for every train row t the
// lexicographic minimum of (dist << 16 | q) over the queries is taken over the 16 lanes of each
// DPP row by a reduce-scatter (in the epilogue), then one LDS atomicMin per lane into
// rl_key[t] (initialised to 0xFFFFFFFF by the caller): the knn-1 of the train rows
// against the queries, the OpenCV tie rule included, without a second MFMA pass.  A padded
// query column (q >= nq) carries keys above every real one (0x7FFF0000 + dist << 16).
// The tile epilogue has no per-row branches (round 6: 356 -> 180 VALU per tile); full tiles skip
// the row-bound tests.
template <int CELL, bool TOP2, bool RL = false>
__device__ GFPL_KNN_INLINE void knn2_mfma(const uint32_t* T, int tstride, int nt, const uint8_t* Q, int nq, uint32_t* out_k0,
                          uint32_t* out_k1, const uint32_t* lut, uint32_t* rl_key = nullptr) {
    constexpr int KS = CELL == 2 ? 16 : 8;   // k-steps of 32
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
    const int h = lane >> 5, c = lane & 31;
    const int nct = (nq + 31) >> 5, nrt = (nt + 31) >> 5;
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) const u32x4v lds_cu4;
    typedef __attribute__((address_space(3))) const u32x2v lds_cu2;
    // the table's LDS address: both callers place it first in their dynamic LDS and have no static
    // LDS, so it is 0 (as a constant the address of a table entry is one SDWA shift of the byte)
    constexpr uint32_t lb = 0;
    (void)lut;
    const uint32_t* Th = T + 4 * h * tstride;   // this lane half's view
    const int pr = lane & 15;   // position in the 16-lane DPP row: the train row (of the lane half) it reduces
    const bool rb3 = (pr & 8) != 0, rb2 = (pr & 4) != 0, rb1 = (pr & 2) != 0, rb0 = (pr & 1) != 0;
    const uint32_t lro = (uint32_t)(4 * h + (pr & 3) + 8 * (pr >> 2));
    for (int ct = wave; ct < nct; ct += nwave) {
        const int q = ct * 32 + c;
        uint32_t qd[8];
        if (q < nq) load_desc(Q + (size_t)q * 32, qd);
        else {
#pragma unroll
            for (int i = 0; i < 8; ++i) qd[i] = 0;
        }
        mfma_v4i bq[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            bq[ks] = knn_frag<CELL, true>(qd, ks, h);
        }
        const uint32_t offk = (uint32_t)(CELL == 2 ? 128 : popc8(qd)) << 16;
        const uint32_t qo = offk + (q < nq ? (uint32_t)q : 0x7FFF0000u);   // (RL)
        uint32_t k0 = 0xFFFFFFFFu, k1 = 0xFFFFFFFFu;
        for (int rt = 0; rt < nrt; ++rt) {
            const int t = rt * 32 + c;
            uint32_t tv[4];
            if (rt * 32 + 32 <= nt) {   // (wave-uniform: a full tile loads without bound tests)
#pragma unroll
                for (int j = 0; j < 4; ++j) tv[j] = Th[j * tstride + t];
            } else if (t < nt) {
#pragma unroll
                for (int j = 0; j < 4; ++j) tv[j] = Th[j * tstride + t];
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) tv[j] = 0;
            }
            mfma_v16i acc = {};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                // table reads at integer LDS addresses (lut is at LDS offset 0): a byte's address is
                // then one shift with an SDWA byte select
                mfma_v4i f;
                if (CELL == 2) {
                    const uint32_t a = lb + (((tv[ks >> 2] >> (8 * (ks & 3))) & 0xFFu) << 4);
                    const u32x4v e = *reinterpret_cast<lds_cu4*>((uintptr_t)a);
                    f[0] = (int)e.x; f[1] = (int)e.y; f[2] = (int)e.z; f[3] = (int)e.w;
                } else {
                    const uint32_t w = tv[ks >> 1];
                    const uint32_t alo = lb + (((w >> (16 * (ks & 1))) & 0xFFu) << 3);
                    const uint32_t ahi = lb + (((w >> (16 * (ks & 1) + 8)) & 0xFFu) << 3);
                    const u32x2v lo = *reinterpret_cast<lds_cu2*>((uintptr_t)alo);
                    const u32x2v hi = *reinterpret_cast<lds_cu2*>((uintptr_t)ahi);
                    f[0] = (int)lo.x; f[1] = (int)lo.y; f[2] = (int)hi.x; f[3] = (int)hi.y;
                }
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(f, bq[ks], acc, 0, 0, 0);
            }
            const uint32_t tb = (uint32_t)(rt * 32 + 4 * h);
            const uint32_t tko = offk + tb;
            // RL by a reduce-scatter over each 16-lane DPP row: four exchange steps (row_mirror,
            // row_half_mirror, quad_perm 3210, quad_perm 1032: partners p ^ 15, p ^ 7, p ^ 3, p ^ 1)
            // each halve the rows a lane carries — it keeps the half its lane bit selects and takes
            // the partner's minimum of that half — so lane p ends with the 16-lane minimum of row p
            // (45 operations instead of 16 rows x 4 DPP minima), and every lane does one atomic
            auto epilogue = [&](auto chk_t) {
                constexpr bool chk = decltype(chk_t)::value;
                auto top2 = [&](int r, uint32_t sh) {
                    const uint32_t ro = (uint32_t)((r & 3) + 8 * (r >> 2));
                    uint32_t key = sh + tko + ro;
                    if (chk && (int)(tb + ro) >= nt) key = 0xFFFFFFFFu;
                    if (TOP2) {   // k0 <= k1: the new second key is med3(k0, k1, key)
                        asm("v_med3_u32 %0, %1, %2, %3" : "=v"(k1) : "v"(k0), "v"(k1), "v"(key));
                        k0 = min(k0, key);
                    } else {
                        k0 = min(k0, key);
                    }
                };
                if (!RL) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) top2(r, (uint32_t)acc[r] << 16);
                    return;
                }
                auto xchg = [](uint32_t a, uint32_t b, bool upper, auto ctrl_t) {   // keep one, take the partner's other
                    const uint32_t send = upper ? a : b, keep = upper ? b : a;
                    return min(keep, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)send, decltype(ctrl_t)::value, 0xF, 0xF, false));
                };
                uint32_t y[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t s0 = (uint32_t)acc[j] << 16, s1 = (uint32_t)acc[j + 8] << 16;
                    top2(j, s0);
                    top2(j + 8, s1);
                    y[j] = xchg(s0 + qo, s1 + qo, rb3, std::integral_constant<int, 0x140>{});   // row_mirror
                }
                uint32_t z[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) z[j] = xchg(y[j], y[j + 4], rb2, std::integral_constant<int, 0x141>{});   // row_half_mirror
                const uint32_t w0 = xchg(z[0], z[2], rb1, std::integral_constant<int, 0x1B>{});   // quad_perm 3210
                const uint32_t w1 = xchg(z[1], z[3], rb1, std::integral_constant<int, 0x1B>{});
                const uint32_t f = xchg(w0, w1, rb0, std::integral_constant<int, 0xB1>{});       // quad_perm 1032
                const uint32_t tr = (uint32_t)(rt * 32) + lro;
                if (!chk || (int)tr < nt) atomicMin(&rl_key[tr], f);
            };
            if (rt * 32 + 32 <= nt) epilogue(std::false_type{});   // (wave-uniform)
            else epilogue(std::true_type{});
        }
        // the two lane halves hold disjoint train rows of the same query column
        const uint32_t o0 = __shfl_xor(k0, 32, 64);
        if (TOP2) {
            const uint32_t o1 = __shfl_xor(k1, 32, 64);
            const uint32_t lo = min(k0, o0), hi0 = max(k0, o0);
            k1 = min(hi0, min(k1, o1));
            k0 = lo;
        } else {
            k0 = min(k0, o0);
        }
        if (h == 0 && q < nq) {
            out_k0[q] = k0;
            if (TOP2) out_k1[q] = k1;
        }
    }
}

// Batched knn-2 over global descriptor sets (BFMatcher::knnMatch for the initial
// frame, src/stereoFrame.cpp:183-197, and gfpl_knn2_hamming): grid (query tiles of
// 128, sequences); each wave keeps one 32-query column tile in registers while the
// train rows stream through LDS in chunks of KNN_CHUNK; train index < 65536.
#define KNN_CHUNK 1024
template <int CELL>
__global__ void __launch_bounds__(256) k_knn2m(const uint8_t* q, const int* nq_arr, int nq_fixed, size_t q_stride,
                                              const uint8_t* t, const int* nt_arr, int nt_fixed, size_t t_stride,
                                              int cap_clamp, int32_t* out_idx, float* out_dist, int32_t* packed,
                                              size_t out_stride) {
    __shared__ __align__(16) uint32_t T[KNN_CHUNK * 8];
    __shared__ __align__(16) uint32_t lut[knn_lut_dwords<CELL>()];
    constexpr int KS = CELL == 2 ? 16 : 8;
    const int b = blockIdx.y;
    const int nq = nq_arr ? min(nq_arr[b], cap_clamp) : nq_fixed;
    const int nt = nt_arr ? min(nt_arr[b], cap_clamp) : nt_fixed;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, c = lane & 31;
    const int qi = (blockIdx.x * 4 + wave) * 32 + c;
    if (blockIdx.x * 128 >= nq) return;   // uniform per workgroup
    const uint8_t* Q = q + (size_t)b * q_stride * 32;
    const uint8_t* Tg = t + (size_t)b * t_stride * 32;
    knn_lut_fill<CELL>(lut);
    uint32_t qd[8];
    if (qi < nq) load_desc(Q + (size_t)qi * 32, qd);
    else {
#pragma unroll
        for (int i = 0; i < 8; ++i) qd[i] = 0;
    }
    mfma_v4i bq[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) bq[ks] = knn_frag<CELL, true>(qd, ks, h);
    const int off = CELL == 2 ? 128 : popc8(qd);
    uint32_t k0 = 0xFFFFFFFFu, k1 = 0xFFFFFFFFu;
    for (int c0 = 0; c0 < nt; c0 += KNN_CHUNK) {
        const int nc = min(KNN_CHUNK, nt - c0);
        __syncthreads();
        knn_stage_soa(T, KNN_CHUNK, Tg + (size_t)c0 * 32, nc);
        __syncthreads();
        const int nrt = (nc + 31) >> 5;
        for (int rt = 0; rt < nrt; ++rt) {
            const int tl = rt * 32 + c;
            uint32_t td[8];
            if (tl < nc) {
#pragma unroll
                for (int i = 0; i < 8; ++i) td[i] = T[i * KNN_CHUNK + tl];
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) td[i] = 0;
            }
            mfma_v16i acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = off;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(knn_frag_lut<CELL>(lut, td, ks, h), bq[ks], acc, 0, 0, 0);
            const uint32_t tb = (uint32_t)(c0 + rt * 32 + 4 * h);
            const bool full = rt * 32 + 32 <= nc;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t tr = tb + (uint32_t)((r & 3) + 8 * (r >> 2));
                uint32_t key = ((uint32_t)acc[r] << 16) + tr;
                if (!full && (int)(tr - (uint32_t)c0) >= nc) key = 0xFFFFFFFFu;
                const uint32_t hi = max(k0, key);
                k0 = min(k0, key);
                k1 = min(k1, hi);
            }
        }
    }
    const uint32_t o0 = __shfl_xor(k0, 32, 64), o1 = __shfl_xor(k1, 32, 64);
    const uint32_t lo = min(k0, o0), hi0 = max(k0, o0);
    k1 = min(hi0, min(k1, o1));
    k0 = lo;
    if (h == 0 && qi < nq) {
        const int i0 = k0 == 0xFFFFFFFFu ? -1 : (int)(k0 & 0xFFFFu), i1 = k1 == 0xFFFFFFFFu ? -1 : (int)(k1 & 0xFFFFu);
        const int d0 = k0 == 0xFFFFFFFFu ? 2147483647 : (int)(k0 >> 16), d1 = k1 == 0xFFFFFFFFu ? 2147483647 : (int)(k1 >> 16);
        if (out_idx) {
            out_idx[2 * qi] = i0; out_idx[2 * qi + 1] = i1;
            out_dist[2 * qi] = (float)d0; out_dist[2 * qi + 1] = (float)d1;
        }
        if (packed) {
            int32_t* o = packed + (size_t)b * out_stride * 3;
            o[3 * qi] = i0; o[3 * qi + 1] = d0; o[3 * qi + 2] = d1;
        }
    }
}

}  // namespace gfpl
