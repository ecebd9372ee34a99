// k_lbd.hip — LBD line descriptors on the GPU (descriptor part):
// line_descriptor::BinaryDescriptor::compute(image, keylines, descriptors)
// (3rdparty/line_descriptor/src/binary_descriptor_custom.cpp:539-687) as
// StereoFrame::detectLineFeatures calls it (src/stereoFrame.cpp:1194,1220) on the keylines
// of one octave (Config::lsdOctaveNum = 1), over a batch of images resident in HBM; the
// arithmetic of the OpenCV / libm calls pinned as the CPU oracle's ledger L1-L5
// (oracle/gfpl_lbd_oracle.cpp).  Kernels, per launch over all images:
//  k_lbd_grad     GaussianBlur 5x5 sigma 1 (computeGaussianPyramid :350-371, L1) and
//                 cv::Sobel 3x3 dx and dy, 8U -> 16S (computeSobel :373-399, L2), exact,
//                 fused per 64x32 tile through LDS (the blurred image stays on chip)
//  k_lbd_describe one wave per keyline (computeLBD :1026-1372): lane h < 63 walks row h
//                 of the 9-band x 7-row line support region (its start point after h
//                 sequential float steps, as the reference steps it), the row sums to
//                 LDS, one lane per (band, statistic) sums its <= 21 rows in row order,
//                 the band means / stds, the two normalisations and the 0.4 clamp on lane
//                 0's sequential sums, and lane c < 32 forms byte c (binaryConversion :401-413)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "gfpl_kernels.hpp"

namespace gfpl {

#define LBD_BANDS 9
#define LBD_BANDW 7
#define LBD_ROWS (LBD_BANDS * LBD_BANDW)

struct LbdDev {
    int W, H;
    int kl_cap;
    int blur_k[5];
    float coefL[3 * LBD_BANDW];   // gaussCoefL_ (L4)
    float coefG[LBD_ROWS];        // gaussCoefG_
    int pairs[32];                // band pair c: i | j << 4
    uint32_t* grad;               // [n][W*H] dx (low 16 bits) | dy (high 16 bits)
    int* err;                     // bit 0: a keyline of another octave
};

namespace {
__device__ __forceinline__ int refl1(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }
// LDS written by some lanes of a wave and read by others: the wave's DS operations complete
// in order; the clobber keeps the compiler from moving accesses across
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// L5: correctly rounded float sqrt.  __fsqrt_rn lowers to the bare v_sqrt_f32 (1 ulp); the f64
// sqrt is correctly rounded (N1) and rounding its result to float is exact for sqrt (53 >= 2*24+2)
__device__ __forceinline__ float sqrt_rn(float x) { return (float)sqrt((double)x); }
}  // namespace

// L1 + L2 fused: GaussianBlur 5x5 (rows exact, columns (s + 2^15) >> 16, REFLECT_101) and
// cv::Sobel 3x3 of the blurred image (REFLECT_101) for one 64x32 output tile: the (32+6) x
// (64+6) source bytes (sources reflected, clamped past the image's reflection span: those
// tile columns feed no output), the rows pass, the columns pass into a (32+2) x (64+2)
// blurred tile, then dx / dy from LDS.  The blurred image never leaves the chip: a blurred
// value just outside the image, computed from reflected sources, equals the reflected
// blurred value Sobel's border wants (the taps are symmetric).  Images >= 8 px.
#define LBD_TW 64
#define LBD_TH 32
__global__ void __launch_bounds__(256) k_lbd_grad(LbdDev o, const uint8_t* images) {
    __shared__ int tile[LBD_TH + 6][LBD_TW + 8];    // source bytes, later the blurred tile
    __shared__ int rows[LBD_TH + 6][LBD_TW + 3];    // rows pass
    const int img = blockIdx.z;
    const int x0 = blockIdx.x * LBD_TW, y0 = blockIdx.y * LBD_TH;
    const size_t npx = (size_t)o.W * o.H;
    const uint8_t* S = images + img * npx;
    const int tx = threadIdx.x & 63, ty0 = threadIdx.x >> 6;
    {   // tile column j = source column x0 - 3 + j (j < 70), tile row i = source row y0 - 3 + i
        const int sx0 = refl1(min(x0 + tx - 3, o.W + 2), o.W);
        const int sx1 = refl1(min(x0 + tx + 61, o.W + 2), o.W);
        uint8_t a[10], b[10];
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int r = min(ty0 + 4 * q, LBD_TH + 5);
            const size_t row = (size_t)refl1(min(y0 + r - 3, o.H + 2), o.H) * o.W;
            a[q] = S[row + sx0];
            b[q] = tx < 6 ? S[row + sx1] : 0;
        }
#pragma unroll
        for (int q = 0; q < 10; ++q) {
            const int r = ty0 + 4 * q;
            if (r < LBD_TH + 6) {
                tile[r][tx] = a[q];
                if (tx < 6) tile[r][tx + 64] = b[q];
            }
        }
    }
    __syncthreads();
    const int k0 = o.blur_k[0], k1 = o.blur_k[1], k2 = o.blur_k[2];
    // rows pass: blurred-tile column c (image column x0 - 1 + c) from tile columns c .. c + 4
    for (int i = threadIdx.x; i < (LBD_TH + 6) * (LBD_TW + 2); i += 256) {
        const int r = i / (LBD_TW + 2), c = i - r * (LBD_TW + 2);
        const int* T = &tile[r][c];
        rows[r][c] = k0 * (T[0] + T[4]) + k1 * (T[1] + T[3]) + k2 * T[2];
    }
    __syncthreads();
    // columns pass: blurred-tile row r (image row y0 - 1 + r) from rows pass rows r .. r + 4
    for (int i = threadIdx.x; i < (LBD_TH + 2) * (LBD_TW + 2); i += 256) {
        const int r = i / (LBD_TW + 2), c = i - r * (LBD_TW + 2);
        const int a = k2 * rows[r + 2][c] + k1 * (rows[r + 1][c] + rows[r + 3][c]) + k0 * (rows[r][c] + rows[r + 4][c]);
        tile[r][c] = min(max((a + (1 << 15)) >> 16, 0), 255);
    }
    __syncthreads();
    // Sobel: thread (tx, ty0) outputs column x0 + tx, rows y0 + 8 ty0 .. + 7
    const int x = x0 + tx;
    if (x >= o.W) return;
    const int r0 = 8 * ty0;
    int v[10][3];
#pragma unroll
    for (int t = 0; t < 10; ++t)
#pragma unroll
        for (int c = 0; c < 3; ++c) v[t][c] = tile[r0 + t][tx + c];
    uint32_t* D = o.grad + img * npx + x;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int y = y0 + r0 + q;
        if (y < o.H) {
            // rows q (y - 1), q + 1 (y), q + 2 (y + 1); columns 0 (x - 1), 1 (x), 2 (x + 1)
            const int gx = (v[q][2] - v[q][0]) + 2 * (v[q + 1][2] - v[q + 1][0]) + (v[q + 2][2] - v[q + 2][0]);
            const int gy = (v[q + 2][0] - v[q][0]) + 2 * (v[q + 2][1] - v[q][1]) + (v[q + 2][2] - v[q][2]);
            D[(size_t)y * o.W] = (uint32_t)(uint16_t)(int16_t)gx | ((uint32_t)(uint16_t)(int16_t)gy << 16);
        }
    }
}

// one wave per keyline; LDS per wave: the 63 rows' eight values, the 72 band statistics
__global__ void __launch_bounds__(256) k_lbd_describe(LbdDev o, const gfpl_keyline* kls, const int* n_kl,
                                                      uint8_t* desc) {
    __shared__ float rowv[4][8][64];
    __shared__ float dv[4][LBD_BANDS * 8];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int img = blockIdx.y, li = blockIdx.x * 4 + wave;
    // the reference describes every keyline: more than kl_cap is an error, not a truncation
    if (li == 0 && lane == 0 && n_kl[img] > o.kl_cap) atomicOr(o.err, 2);
    if (li >= min(n_kl[img], o.kl_cap)) return;
    const gfpl_keyline kl = kls[(size_t)img * o.kl_cap + li];
    uint8_t* out = desc + ((size_t)img * o.kl_cap + li) * 32;
    if (kl.octave != 0) {   // lsdOctaveNum = 1: no pyramid octave to read
        if (lane == 0) atomicOr(o.err, 1);
        return;
    }
    const size_t npx = (size_t)o.W * o.H;
    const uint32_t* G = o.grad + img * npx;
    // numOfPixels: cv::LineIterator count of the rounded endpoints (8-connectivity)
    const int ax = __float2int_rn(kl.sx), ay = __float2int_rn(kl.sy);
    const int bx = __float2int_rn(kl.ex), by = __float2int_rn(kl.ey);
    const int L = (int)(short)(max(abs(bx - ax), abs(by - ay)) + 1);
    const int halfWidth = (L - 1) / 2, halfHeight = (LBD_ROWS - 1) / 2;
    const float midX = (kl.sx + kl.ex) * 0.5f, midY = (kl.sy + kl.ey) * 0.5f;
    const float dL0 = (float)det_cos((double)kl.angle), dL1 = (float)det_sin((double)kl.angle);   // L3
    const float dO0 = -dL1, dO1 = dL0;
    const float sX00 = -dL0 * (float)halfWidth + dL1 * (float)halfHeight + midX;
    const float sY00 = -dL1 * (float)halfWidth - dL0 * (float)halfHeight + midY;
    // row h starts where h sequential steps (sCorX0 -= dL[1], sCorY0 += dL[0]) lead
    float sX = 0.0f, sY = 0.0f;
    {
        float cx = sX00, cy = sY00;
        for (int k = 0; k < LBD_ROWS; ++k) {
            if (k == lane) { sX = cx; sY = cy; }
            cx -= dL1;
            cy += dL0;
        }
    }
    float pl = 0.0f, nl = 0.0f, po = 0.0f, no = 0.0f;
    if (lane < LBD_ROWS) {
        const int iw = o.W - 1, ih = o.H - 1;
#pragma unroll 4
        for (int w = 0; w < L; ++w) {
            int t = (int)(short)(int)roundf(sX);
            const int xc = t < 0 ? 0 : (t > iw ? iw : t);
            t = (int)(short)(int)roundf(sY);
            const int yc = t < 0 ? 0 : (t > ih ? ih : t);
            const uint32_t g = G[(size_t)yc * o.W + xc];
            const float dx = (float)(int16_t)(g & 0xFFFFu), dy = (float)(int16_t)(g >> 16);
            const float gDL = dx * dL0 + dy * dL1;
            const float gDO = dx * dO0 + dy * dO1;
            if (gDL > 0) pl += gDL; else nl -= gDL;
            if (gDO > 0) po += gDO; else no -= gDO;
            sX += dL0;
            sY += dL1;
        }
        const float c = o.coefG[lane];
        pl = c * pl; nl = c * nl; po = c * po; no = c * no;
    }
    // per row: pL nL pL2 nL2 pO nO pO2 nO2 (the order of the band statistics below)
    rowv[wave][0][lane] = pl; rowv[wave][1][lane] = nl; rowv[wave][2][lane] = pl * pl; rowv[wave][3][lane] = nl * nl;
    rowv[wave][4][lane] = po; rowv[wave][5][lane] = no; rowv[wave][6][lane] = po * po; rowv[wave][7][lane] = no * no;
    lds_sync();
    // band sums: statistic s of band b over the rows of bands b-1, b, b+1 in row order
    float bs[2];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const int j = pass * 64 + lane;
        float acc = 0.0f;
        if (j < LBD_BANDS * 8) {
            const int b = j >> 3, s = j & 7;
            const bool square = s == 2 || s == 3 || s == 6 || s == 7;
            const int h0 = max(0, (b - 1) * LBD_BANDW), h1 = min(LBD_ROWS, (b + 2) * LBD_BANDW);
            for (int h = h0; h < h1; ++h) {
                const int hb = h / LBD_BANDW;
                // the row's own band uses coefL[h%7 + 7], the band above it (b = hb - 1)
                // coefL[h%7 + 14], the band below it (b = hb + 1) coefL[h%7]
                const float cc = o.coefL[h % LBD_BANDW + (hb == b ? LBD_BANDW : (hb == b + 1 ? 2 * LBD_BANDW : 0))];
                const float v = rowv[wave][s][h];
                acc += square ? (cc * cc) * v : cc * v;
            }
        }
        bs[pass] = acc;
    }
    // band statistic j -> (mean, std) entries of the descriptor vector
    lds_sync();
    float* D = dv[wave];
    float* S72 = &rowv[wave][0][0];   // the band sums, j = 8 b + s (rows are dead now)
    lds_sync();
    S72[lane] = bs[0];
    if (lane < 8) S72[64 + lane] = bs[1];
    lds_sync();
    if (lane < LBD_BANDS * 4) {
        const int b = lane >> 2, k = lane & 3;   // k: pL nL pO nO
        const float invN = (b == 0 || b == LBD_BANDS - 1) ? (float)(1.0 / (LBD_BANDW * 2.0)) : (float)(1.0 / (LBD_BANDW * 3.0));
        const int sm = (k < 2 ? 0 : 4) + (k & 1), s2 = sm + 2;
        const float t = S72[8 * b + sm] * invN;
        D[8 * b + k] = t;
        D[8 * b + 4 + k] = sqrt_rn(S72[8 * b + s2] * invN - t * t);
    }
    lds_sync();
    // normalisation (sequential sums in the reference's order), clamp, renormalisation
    float tm = 0.0f, ts = 0.0f;
    for (int b = 0; b < LBD_BANDS; ++b) {
#pragma unroll
        for (int k = 0; k < 4; ++k) tm += D[8 * b + k] * D[8 * b + k];
#pragma unroll
        for (int k = 4; k < 8; ++k) ts += D[8 * b + k] * D[8 * b + k];
    }
    tm = __fdiv_rn(1.0f, sqrt_rn(tm));
    ts = __fdiv_rn(1.0f, sqrt_rn(ts));
    float e[2];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const int i = pass * 64 + lane;
        float v = 0.0f;
        if (i < LBD_BANDS * 8) {
            v = D[i] * ((i & 7) < 4 ? tm : ts);
            if ((double)v > 0.4) v = (float)0.4;
        }
        e[pass] = v;
    }
    lds_sync();
    D[lane] = e[0];
    if (lane < 8) D[64 + lane] = e[1];
    lds_sync();
    float t2 = 0.0f;
    for (int i = 0; i < LBD_BANDS * 8; ++i) t2 += D[i] * D[i];
    t2 = __fdiv_rn(1.0f, sqrt_rn(t2));
    if (lane < 32) {
        const int pi = o.pairs[lane] & 15, pj = o.pairs[lane] >> 4;
        uint32_t r = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float f1 = D[8 * pi + i] * t2, f2 = D[8 * pj + i] * t2;
            if (f1 > f2) r += 1u << i;
        }
        out[lane] = (uint8_t)r;
    }
}

}  // namespace gfpl

// ======================================================================= ABI ==
using namespace gfpl;

struct gfpl_lbd {
    int device = 0;
    hipStream_t stream = nullptr;
    gfpl_ctx* ctx = nullptr;   // counted in while this object lives
    AsyncStatus st;
    int max_images = 0;
    LbdDev d{};
    void* base = nullptr;
};

extern "C" int gfpl_lbd_create(gfpl_ctx* ctx, int width, int height, int max_images, int kl_cap, gfpl_lbd** out) {
    if (!ctx || !out || max_images < 1 || kl_cap < 1 || width < 8 || height < 8 || width > 8192 || height > 8192)
        return GFPL_E_INVALID;
    const int dev = gfpl_ctx_device(ctx);
    if (hipSetDevice(dev) != hipSuccess) return GFPL_E_HIP;
    gfpl_lbd* o = new gfpl_lbd();
    o->device = dev;
    o->stream = (hipStream_t)gfpl_ctx_stream(ctx);
    o->max_images = max_images;
    LbdDev& d = o->d;
    d.W = width;
    d.H = height;
    d.kl_cap = kl_cap;
    {   // L1 taps: getGaussianKernel(5, 1) in float, rounded to 8-bit fixed point
        float cf[5];
        double sum = 0;
        for (int i = 0; i < 5; ++i) {
            const double x = i - 2.0;
            cf[i] = (float)std::exp(-0.5 * x * x);
            sum += cf[i];
        }
        sum = 1. / sum;
        for (int i = 0; i < 5; ++i) d.blur_k[i] = (int)std::nearbyintf((float)(cf[i] * sum) * 256.0f);
    }
    {   // L4: BinaryDescriptor::BinaryDescriptor (:217-260)
        double u = (LBD_BANDW * 3 - 1) / 2;
        double sigma = (LBD_BANDW * 2 + 1) / 2;
        double inv = -1 / (2 * sigma * sigma);
        for (int i = 0; i < LBD_BANDW * 3; ++i) {
            const double dd = i - u;
            d.coefL[i] = (float)std::exp(dd * dd * inv);
        }
        u = (LBD_ROWS - 1) / 2;
        sigma = u;
        inv = -1 / (2 * sigma * sigma);
        for (int i = 0; i < LBD_ROWS; ++i) {
            const double dd = i - u;
            d.coefG[i] = (float)std::exp(dd * dd * inv);
        }
    }
    {   // the 32 band pairs (binary_descriptor_custom.cpp:74-106): i < j lexicographic,
        // without the four pairs joining bands 0/1 with 7/8
        int c = 0;
        for (int i = 0; i < LBD_BANDS; ++i)
            for (int j = i + 1; j < LBD_BANDS; ++j)
                if (!(i <= 1 && j >= 7)) d.pairs[c++] = i | (j << 4);
    }
    const size_t npx = (size_t)width * height, M = (size_t)max_images;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t b_g = al(4 * M * npx);
    if (hipMalloc(&o->base, b_g + 256) != hipSuccess) { delete o; return GFPL_E_HIP; }
    char* p = (char*)o->base;
    d.grad = (uint32_t*)p; p += b_g;
    d.err = (int*)p;
    if (o->st.init(d.err, o->stream) != hipSuccess) { o->st.destroy(); (void)hipFree(o->base); delete o; return GFPL_E_HIP; }
    o->ctx = ctx;
    gfpl_ctx_attach(ctx);
    *out = o;
    return GFPL_OK;
}

extern "C" int gfpl_lbd_destroy(gfpl_lbd* o) {
    if (!o) return GFPL_E_INVALID;
    (void)hipStreamSynchronize(o->stream);
    o->st.destroy();
    if (o->base) (void)hipFree(o->base);
    gfpl_ctx_detach(o->ctx);
    delete o;
    return GFPL_OK;
}

extern "C" int gfpl_lbd_gradients(gfpl_lbd* o, const uint8_t* image, uint32_t* grad) {
    if (!o || !image || !grad) return GFPL_E_INVALID;
    if (hipSetDevice(o->device) != hipSuccess) return GFPL_E_HIP;
    const LbdDev& d = o->d;
    hipLaunchKernelGGL(k_lbd_grad, dim3((d.W + LBD_TW - 1) / LBD_TW, (d.H + LBD_TH - 1) / LBD_TH, 1), dim3(256), 0,
                       o->stream, d, image);
    if (hipMemcpyAsync(grad, d.grad, 4 * (size_t)d.W * d.H, hipMemcpyDeviceToDevice, o->stream) != hipSuccess)
        return GFPL_E_HIP;
    return hipStreamSynchronize(o->stream) == hipSuccess ? GFPL_OK : GFPL_E_HIP;
}

extern "C" int gfpl_lbd_compute_async(gfpl_lbd* o, const uint8_t* images, int n, const gfpl_keyline* keylines,
                                      const int* n_kl, uint8_t* desc) {
    if (!o || !images || n < 1 || n > o->max_images || !keylines || !n_kl || !desc) return GFPL_E_INVALID;
    if (hipSetDevice(o->device) != hipSuccess) return GFPL_E_HIP;
    const LbdDev& d = o->d;
    hipStream_t s = o->stream;
    hipLaunchKernelGGL(k_lbd_grad, dim3((d.W + LBD_TW - 1) / LBD_TW, (d.H + LBD_TH - 1) / LBD_TH, n), dim3(256), 0, s, d,
                       images);
    hipLaunchKernelGGL(k_lbd_describe, dim3((d.kl_cap + 3) / 4, n), dim3(256), 0, s, d, keylines, n_kl, desc);
    if (hipGetLastError() != hipSuccess) return GFPL_E_HIP;
    return o->st.enqueue(s) == hipSuccess ? GFPL_OK : GFPL_E_HIP;
}

extern "C" int gfpl_lbd_status(gfpl_lbd* o) {
    if (!o) return GFPL_E_INVALID;
    int bits = 0;
    if (o->st.wait(o->stream, &bits) != hipSuccess) return GFPL_E_HIP;
    if (bits & 1) return GFPL_E_UNSUPPORTED;   // a keyline of another octave
    return (bits & 2) ? GFPL_E_CAPACITY : GFPL_OK;   // more keylines than kl_cap
}

extern "C" int gfpl_lbd_compute(gfpl_lbd* o, const uint8_t* images, int n, const gfpl_keyline* keylines,
                                const int* n_kl, uint8_t* desc) {
    const int e = gfpl_lbd_compute_async(o, images, n, keylines, n_kl, desc);
    if (e) return e;
    return gfpl_lbd_status(o);
}
