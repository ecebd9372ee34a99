// gfpl_lbd_oracle.cpp — CPU ORACLE of the LBD descriptor row (part).
// TEST INFRASTRUCTURE ONLY (see gfpl_oracle.h): the checker of the GPU LBD path.
//
// Restates line_descriptor::BinaryDescriptor::compute(image, keylines, descriptors) as
// StereoFrame::detectLineFeatures calls it (src/stereoFrame.cpp:1194, 1220) with the
// reference's parameters (3rdparty/line_descriptor/src/binary_descriptor_custom.cpp:
// Params :110-117 — one octave, band width 7, 9 bands; Config::lsdOctaveNum = 1,
// src/config.cpp:146, so every keyline is octave 0):
//   computeImpl :539-687 -> computeSobel :373-399 (computeGaussianPyramid :350-371: the
//   image through GaussianBlur 5x5 sigma 1), computeLBD :1026-1372 (line support region of
//   9 bands x 7 rows, gradient projections, band statistics, normalisation, 0.4 clamp),
//   binaryConversion :401-413 over the 32 band pairs of `combinations` (:74-106).
// numOfPixels of a keyline is LSDDetectorC's cv::LineIterator count (src/LSDDetector_custom.cpp
// :282-283): the endpoints rounded to int, max(|dx|, |dy|) + 1 for 8-connectivity.
//
// Arithmetic of the OpenCV / libm calls it makes (ledger L1-L5; PARITY UNPINNED
// against the reference binary, like O1-O7):
//   L1 GaussianBlur 5x5 sigma 1 8U: getGaussianKernel in float rounded to 8-bit taps
//      (14 63 103 63 14 — sum 257), exact row pass, column pass (s + 2^15) >> 16, REFLECT_101.
//   L2 Sobel 3x3 8U -> 16S, dx and dy: exact integer [-1 0 1] x [1 2 1], REFLECT_101.
//   L3 the float cos / sin of the float line direction: the float of the fdlibm double value.
//   L4 gaussCoefL_ / gaussCoefG_: libm exp in double (host), used as float as the reference does.
//   L5 no FP contraction; std::round = round half away from zero; float sqrt correctly rounded.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "gfpl_oracle.h"

namespace {

constexpr int kBands = 9;   // NUM_OF_BANDS (binary_descriptor_custom.cpp:57)
constexpr int kBandW = 7;   // widthOfBand_ (:113)
constexpr int kRows = kBands * kBandW;

inline int refl101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
}

// L1
void gauss5(const uint8_t* s, int w, int h, uint8_t* d) {
    float cf[5];
    double sum = 0;
    for (int i = 0; i < 5; ++i) {
        const double x = i - 2.0;
        cf[i] = (float)std::exp(-0.5 * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    int k[5];
    for (int i = 0; i < 5; ++i) k[i] = (int)std::nearbyintf((float)(cf[i] * sum) * 256.0f);
    std::vector<int> rows((size_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int a = 0;
            for (int t = 0; t < 5; ++t) a += k[t] * s[(size_t)y * w + refl101(x + t - 2, w)];
            rows[(size_t)y * w + x] = a;
        }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int a = 0;
            for (int t = 0; t < 5; ++t) a += k[t] * rows[(size_t)refl101(y + t - 2, h) * w + x];
            a = (a + (1 << 15)) >> 16;
            d[(size_t)y * w + x] = (uint8_t)(a < 0 ? 0 : (a > 255 ? 255 : a));
        }
}

// L2
void sobel(const uint8_t* b, int w, int h, int16_t* dx, int16_t* dy) {
    auto at = [&](int x, int y) { return (int)b[(size_t)refl101(y, h) * w + refl101(x, w)]; };
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int gx = 0, gy = 0;
            const int kw[3] = {1, 2, 1};
            for (int t = -1; t <= 1; ++t) {
                gx += kw[t + 1] * (at(x + 1, y + t) - at(x - 1, y + t));
                gy += kw[t + 1] * (at(x + t, y + 1) - at(x + t, y - 1));
            }
            dx[(size_t)y * w + x] = (int16_t)gx;
            dy[(size_t)y * w + x] = (int16_t)gy;
        }
}

// the 32 band pairs of the binary descriptor: every pair i < j in lexicographic order
// except the four that join one of the two outer bands on each side (0/1 with 7/8)
void band_pairs(int pairs[32][2]) {
    int c = 0;
    for (int i = 0; i < kBands; ++i)
        for (int j = i + 1; j < kBands; ++j)
            if (!(i <= 1 && j >= 7)) { pairs[c][0] = i; pairs[c][1] = j; ++c; }
}

}  // namespace

extern "C" int gfplo_lbd_coefs(float* coef_l, float* coef_g) {
    // BinaryDescriptor::BinaryDescriptor (:217-260), L4
    double u = (kBandW * 3 - 1) / 2;
    double sigma = (kBandW * 2 + 1) / 2;
    double inv = -1 / (2 * sigma * sigma);
    for (int i = 0; i < kBandW * 3; ++i) {
        const double d = i - u;
        coef_l[i] = (float)std::exp(d * d * inv);
    }
    u = (kRows - 1) / 2;
    sigma = u;
    inv = -1 / (2 * sigma * sigma);
    for (int i = 0; i < kRows; ++i) {
        const double d = i - u;
        coef_g[i] = (float)std::exp(d * d * inv);
    }
    return GFPL_OK;
}

extern "C" int gfplo_lbd_num_pixels(const gfpl_keyline* kl, int width, int height) {
    // cv::LineIterator(img, Point(sx, sy), Point(ex, ey)) count, 8-connectivity; the
    // endpoints of LSD keylines lie in the image (checkLineExtremes), so no clipping
    (void)width;
    (void)height;
    const int x1 = (int)std::nearbyintf(kl->sx), y1 = (int)std::nearbyintf(kl->sy);
    const int x2 = (int)std::nearbyintf(kl->ex), y2 = (int)std::nearbyintf(kl->ey);
    const int dx = std::abs(x2 - x1), dy = std::abs(y2 - y1);
    return (dx > dy ? dx : dy) + 1;
}

extern "C" int gfplo_lbd_gradients(const uint8_t* image, int width, int height, uint8_t* blur, int16_t* dx,
                                   int16_t* dy) {
    if (!image || width < 2 || height < 2) return GFPL_E_INVALID;
    std::vector<uint8_t> b((size_t)width * height);
    gauss5(image, width, height, b.data());
    if (blur) std::memcpy(blur, b.data(), b.size());
    if (dx && dy) sobel(b.data(), width, height, dx, dy);
    return GFPL_OK;
}

extern "C" int gfplo_lbd_compute(const uint8_t* image, int width, int height, const gfpl_keyline* kls, int n,
                                 uint8_t* desc, float* desc_f) {
    if (!image || (!kls && n > 0) || n < 0 || width < 2 || height < 2) return GFPL_E_INVALID;
    for (int i = 0; i < n; ++i)
        if (kls[i].octave != 0) return GFPL_E_UNSUPPORTED;   // lsdOctaveNum = 1
    std::vector<int16_t> gx((size_t)width * height), gy((size_t)width * height);
    gfplo_lbd_gradients(image, width, height, nullptr, gx.data(), gy.data());
    float coefL[kBandW * 3], coefG[kRows];
    gfplo_lbd_coefs(coefL, coefG);
    int pairs[32][2];
    band_pairs(pairs);
    const short imageWidth = (short)(width - 1), imageHeight = (short)(height - 1);
    for (int li = 0; li < n; ++li) {
        const gfpl_keyline& kl = kls[li];
        // computeLBD (:1026-1372) for one line
        float pL[kBands] = {}, nL[kBands] = {}, pL2[kBands] = {}, nL2[kBands] = {};
        float pO[kBands] = {}, nO[kBands] = {}, pO2[kBands] = {}, nO2[kBands] = {};
        const short lengthOfLSP = (short)gfplo_lbd_num_pixels(&kl, width, height);
        const short halfWidth = (short)((lengthOfLSP - 1) / 2);
        const short halfHeight = (short)((kRows - 1) / 2);
        const float midX = (float)(0.5 * (kl.sx + kl.ex)), midY = (float)(0.5 * (kl.sy + kl.ey));
        const float dL0 = (float)gfplo_cos((double)kl.angle), dL1 = (float)gfplo_sin((double)kl.angle);   // L3
        const float dO0 = -dL1, dO1 = dL0;
        float sX0 = -dL0 * halfWidth + dL1 * halfHeight + midX;
        float sY0 = -dL1 * halfWidth - dL0 * halfHeight + midY;
        for (int h = 0; h < kRows; ++h) {
            float sX = sX0, sY = sY0;
            float pl = 0, nl = 0, po = 0, no = 0;
            for (int w = 0; w < lengthOfLSP; ++w) {
                short t = (short)std::round(sX);
                const short xc = t < 0 ? 0 : (t > imageWidth ? imageWidth : t);
                t = (short)std::round(sY);
                const short yc = t < 0 ? 0 : (t > imageHeight ? imageHeight : t);
                const short dx = gx[(size_t)yc * width + xc], dy = gy[(size_t)yc * width + xc];
                const float gDL = dx * dL0 + dy * dL1;
                const float gDO = dx * dO0 + dy * dO1;
                if (gDL > 0) pl += gDL; else nl -= gDL;
                if (gDO > 0) po += gDO; else no -= gDO;
                sX += dL0;
                sY += dL1;
            }
            sX0 -= dL1;
            sY0 += dL0;
            float c = coefG[h];
            pl = c * pl; nl = c * nl;
            const float pl2 = pl * pl, nl2 = nl * nl;
            po = c * po; no = c * no;
            const float po2 = po * po, no2 = no * no;
            auto add = [&](int b, float cc) {
                pL[b] += cc * pl; nL[b] += cc * nl; pL2[b] += cc * cc * pl2; nL2[b] += cc * cc * nl2;
                pO[b] += cc * po; nO[b] += cc * no; pO2[b] += cc * cc * po2; nO2[b] += cc * cc * no2;
            };
            const int band = h / kBandW;
            add(band, coefL[h % kBandW + kBandW]);
            if (band - 1 >= 0) add(band - 1, coefL[h % kBandW + 2 * kBandW]);
            if (band + 1 < kBands) add(band + 1, coefL[h % kBandW]);
        }
        float d[kBands * 8];
        const float invN2 = (float)(1.0 / (kBandW * 2.0)), invN3 = (float)(1.0 / (kBandW * 3.0));
        for (int b = 0; b < kBands; ++b) {
            const float invN = (b == 0 || b == kBands - 1) ? invN2 : invN3;
            float t = pL[b] * invN;
            d[8 * b] = t;
            d[8 * b + 4] = std::sqrt(pL2[b] * invN - t * t);
            t = nL[b] * invN;
            d[8 * b + 1] = t;
            d[8 * b + 5] = std::sqrt(nL2[b] * invN - t * t);
            t = pO[b] * invN;
            d[8 * b + 2] = t;
            d[8 * b + 6] = std::sqrt(pO2[b] * invN - t * t);
            t = nO[b] * invN;
            d[8 * b + 3] = t;
            d[8 * b + 7] = std::sqrt(nO2[b] * invN - t * t);
        }
        float tm = 0, ts = 0;
        for (int b = 0; b < kBands; ++b) {
            for (int k = 0; k < 4; ++k) tm += d[8 * b + k] * d[8 * b + k];
            for (int k = 4; k < 8; ++k) ts += d[8 * b + k] * d[8 * b + k];
        }
        tm = 1 / std::sqrt(tm);
        ts = 1 / std::sqrt(ts);
        for (int b = 0; b < kBands; ++b) {
            for (int k = 0; k < 4; ++k) d[8 * b + k] = d[8 * b + k] * tm;
            for (int k = 4; k < 8; ++k) d[8 * b + k] = d[8 * b + k] * ts;
        }
        for (int i = 0; i < kBands * 8; ++i)
            if (d[i] > 0.4) d[i] = (float)0.4;
        float t = 0;
        for (int i = 0; i < kBands * 8; ++i) t += d[i] * d[i];
        t = 1 / std::sqrt(t);
        for (int i = 0; i < kBands * 8; ++i) d[i] = d[i] * t;
        if (desc_f) std::memcpy(desc_f + (size_t)li * kBands * 8, d, sizeof d);
        if (desc)
            for (int c = 0; c < 32; ++c) {
                const float* f1 = d + 8 * pairs[c][0];
                const float* f2 = d + 8 * pairs[c][1];
                uint8_t r = 0;
                for (int i = 0; i < 8; ++i)
                    if (f1[i] > f2[i]) r = (uint8_t)(r + (1u << i));
                desc[32 * (size_t)li + c] = r;
            }
    }
    return GFPL_OK;
}
