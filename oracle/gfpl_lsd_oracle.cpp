// gfpl_lsd_oracle.cpp — CPU ORACLE of the LSD line detection row.
// TEST INFRASTRUCTURE ONLY (see gfpl_oracle.h): the checker of the GPU LSD path.
//
// Restates line_descriptor::LSDDetectorC::detect(image, keylines, scale, numOctaves, opts)
// (3rdparty/line_descriptor/src/LSDDetector_custom.cpp:218-316) as
// StereoFrame::detectLineFeatures calls it (src/stereoFrame.cpp:1160-1186) with the
// reference's Config (src/config.cpp:143-152: refine 1 = LSD_REFINE_STD, scale 1, one
// octave, quant 2, ang_th 22.5, density_th 0.6, n_bins 1024, nfeatures 300):
//   cv::LineSegmentDetector::detect (OpenCV 3.4.1 modules/imgproc/src/lsd.cpp, absent from
//   the image — restated from its published algorithm): flsd -> ll_angle (gradient, angle,
//   1024-bin norm keys, std::sort), the seed loop over the sorted pixels, region_grow,
//   region2rect / get_theta, refine / reduce_region_radius (REFINE_STD: no NFA), the 0.5 offset;
//   then LSDDetector_custom.cpp:266-306 (checkLineExtremes :78-103, the min-length test,
//   KeyLine fields) and the response sort + resize of src/stereoFrame.cpp:1177-1185.
//
// Ledger (PARITY UNPINNED against the reference binary, like O1-O7 / L1-L5):
//   S1 scale == 1: no Gaussian sampling; the gradient is lsd.cpp's 2x2 integer difference,
//      norm = sqrt((gx*gx + gy*gy) / 4.0) in double, angle = fastAtan2(gx, -gy) (O4) * DEG_TO_RADS
//      (CV_PI / 180 as a double constant); pixels with norm <= rho = quant / sin(prec) and the
//      last row / column are NOTDEF (-1024).
//   S2 the seed order is std::sort of the (W-1)(H-1) row-major pixels by the descending key
//      int(norm * (n_bins - 1) / max_grad) — libstdc++'s introsort (GCC >= 4.9 median-of-three
//      __move_median_to_first, Hoare __unguarded_partition, depth 2*lg(n) with heapsort,
//      threshold 16, final insertion sort): its permutation of equal keys is the reference's
//      only where the reference was built against a libstdc++ with the same algorithm.
//   S3 cos / sin of float(angle) in region_grow (float overloads) and float(cos(double)) of the
//      seed: the float of the fdlibm double value (as L3); double cos / sin of theta: fdlibm (N3).
//   S4 atan2(float, float) of KeyLine::angle: the float of fdlibm's double atan2 (e_atan2.c,
//      s_atan.c) — atan2f / ::atan2 agree with it except in rare last-bit cases.
//   S5 log10 / sin of the per-image constants (LOG_NT, min_reg_size, rho) from the host libm;
//      pow(float, 2) exact (the square of a float fits a double).
//   S6 list sums in list order, no FP contraction; the region list keeps lsd.cpp's order
//      (BFS push order; reduce_region_radius's swap-with-last removal).
//   S7 the response sort is std::sort (S2's algorithm) of the keylines by response, descending.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "gfpl_oracle.h"

namespace {

const double kPi = 3.1415926535897932384626433832795;   // CV_PI
const double k32Pi = (3 * kPi) / 2;                       // M_3_2_PI
const double k2Pi = 2 * kPi;                              // M_2__PI
const double kNotDef = -1024.0;                           // NOTDEF
const double kDeg2Rad = kPi / 180;                        // DEG_TO_RADS

inline uint32_t hi_word(double x) { uint64_t u; std::memcpy(&u, &x, 8); return (uint32_t)(u >> 32); }
inline uint32_t lo_word(double x) { uint64_t u; std::memcpy(&u, &x, 8); return (uint32_t)u; }

// S4: fdlibm s_atan.c
const double atanhi[] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                         1.57079632679489655800e+00};
const double atanlo[] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                         6.12323399573676603587e-17};
const double aT[] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                     -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                     6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                     -3.65315727442169155270e-02, 1.62858201153657823623e-02};

double fd_atan(double x) {
    const int32_t hx = (int32_t)hi_word(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) {   // |x| >= 2^66 (finite inputs only on this path)
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3fdc0000) {    // |x| < 0.4375
        if (ix < 0x3e200000) return x;
        id = -1;
    } else {
        x = std::fabs(x);
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

// S4: fdlibm e_atan2.c (finite arguments)
double fd_atan2(double y, double x) {
    const double pi_o_2 = 1.5707963267948965580e+00, pi = 3.1415926535897931160e+00,
                 pi_lo = 1.2246467991473531772e-16, tiny = 1.0e-300;
    const int32_t hx = (int32_t)hi_word(x), hy = (int32_t)hi_word(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const uint32_t lx = lo_word(x), ly = lo_word(y);
    if ((((uint32_t)hx - 0x3ff00000u) | lx) == 0) return fd_atan(y);   // x = 1.0 (unsigned: no overflow)
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if ((iy | ly) == 0) {
        switch (m) {
            case 0: case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if ((ix | lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0;
    else z = fd_atan(std::fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

inline float cosf_(double a) { return (float)gfplo_cos((double)(float)a); }   // S3: cos(float(angle))
inline float sinf_(double a) { return (float)gfplo_sin((double)(float)a); }

struct NormPoint { int x, y, norm; };
struct RegionPoint { int x, y; double angle, modgrad; };
struct Rect { double x1, y1, x2, y2, width, x, y, theta, dx, dy, prec, p; };

inline double dist(double x1, double y1, double x2, double y2) {
    return std::sqrt((x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1));
}
inline double dist_sq(double x1, double y1, double x2, double y2) {
    return (x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1);
}
inline double angle_diff_signed(double a, double b) {
    double diff = a - b;
    while (diff <= -kPi) diff += k2Pi;
    while (diff > kPi) diff -= k2Pi;
    return diff;
}
inline double angle_diff(double a, double b) { return std::fabs(angle_diff_signed(a, b)); }

struct Lsd {
    int W, H;
    double prec, p, rho, density_th;
    int n_bins;
    size_t min_reg_size;
    std::vector<double> angles, modgrad;
    std::vector<uint8_t> used;
    std::vector<NormPoint> ordered;

    double ang(int x, int y) const { return angles[(size_t)y * W + x]; }

    // ll_angle (S1, S2)
    void ll_angle(const uint8_t* img) {
        angles.assign((size_t)W * H, kNotDef);
        modgrad.assign((size_t)W * H, 0.0);
        double max_grad = -1;
        for (int y = 0; y < H - 1; ++y)
            for (int x = 0; x < W - 1; ++x) {
                const int DA = img[(size_t)(y + 1) * W + x + 1] - img[(size_t)y * W + x];
                const int BC = img[(size_t)y * W + x + 1] - img[(size_t)(y + 1) * W + x];
                const int gx = DA + BC, gy = DA - BC;
                const double norm = std::sqrt((gx * gx + gy * gy) / 4.0);
                modgrad[(size_t)y * W + x] = norm;
                if (norm <= rho) {
                    angles[(size_t)y * W + x] = kNotDef;
                } else {
                    angles[(size_t)y * W + x] = gfplo_fast_atan2((float)gx, (float)-gy) * kDeg2Rad;
                    if (norm > max_grad) max_grad = norm;
                }
            }
        const double bin_coef = (max_grad > 0) ? double(n_bins - 1) / max_grad : 0;
        ordered.clear();
        ordered.reserve((size_t)(W - 1) * (H - 1));
        for (int y = 0; y < H - 1; ++y)
            for (int x = 0; x < W - 1; ++x)
                ordered.push_back({x, y, (int)(modgrad[(size_t)y * W + x] * bin_coef)});
        std::sort(ordered.begin(), ordered.end(), [](const NormPoint& a, const NormPoint& b) { return a.norm > b.norm; });
    }

    bool is_aligned(int x, int y, double theta, double pr) const {
        if (x < 0 || y < 0 || x >= W || y >= H) return false;
        const double a = ang(x, y);
        if (a == kNotDef) return false;
        double n_theta = theta - a;
        if (n_theta < 0) n_theta = -n_theta;
        if (n_theta > k32Pi) {
            n_theta -= k2Pi;
            if (n_theta < 0) n_theta = -n_theta;
        }
        return n_theta <= pr;
    }

    void region_grow(int sx, int sy, std::vector<RegionPoint>& reg, double& reg_angle, double pr) {
        reg.clear();
        reg_angle = ang(sx, sy);
        reg.push_back({sx, sy, reg_angle, modgrad[(size_t)sy * W + sx]});
        float sumdx = (float)gfplo_cos(reg_angle);   // S3: float(std::cos(double))
        float sumdy = (float)gfplo_sin(reg_angle);
        used[(size_t)sy * W + sx] = 1;
        for (size_t i = 0; i < reg.size(); ++i) {
            const int rx = reg[i].x, ry = reg[i].y;
            const int xx_min = std::max(rx - 1, 0), xx_max = std::min(rx + 1, W - 1);
            const int yy_min = std::max(ry - 1, 0), yy_max = std::min(ry + 1, H - 1);
            for (int yy = yy_min; yy <= yy_max; ++yy)
                for (int xx = xx_min; xx <= xx_max; ++xx) {
                    uint8_t& is_used = used[(size_t)yy * W + xx];
                    if (is_used != 1 && is_aligned(xx, yy, reg_angle, pr)) {
                        const double a = ang(xx, yy);
                        is_used = 1;
                        reg.push_back({xx, yy, a, modgrad[(size_t)yy * W + xx]});
                        sumdx += cosf_(a);
                        sumdy += sinf_(a);
                        reg_angle = gfplo_fast_atan2(sumdy, sumdx) * kDeg2Rad;
                    }
                }
        }
    }

    double get_theta(const std::vector<RegionPoint>& reg, double x, double y, double reg_angle, double pr) const {
        double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
        for (const RegionPoint& r : reg) {
            const double dx = (double)r.x - x, dy = (double)r.y - y;
            Ixx += dy * dy * r.modgrad;
            Iyy += dx * dx * r.modgrad;
            Ixy -= dx * dy * r.modgrad;
        }
        const double lambda = 0.5 * (Ixx + Iyy - std::sqrt((Ixx - Iyy) * (Ixx - Iyy) + 4.0 * Ixy * Ixy));
        double theta = (std::fabs(Ixx) > std::fabs(Iyy)) ? double(gfplo_fast_atan2(float(lambda - Ixx), float(Ixy)))
                                                         : double(gfplo_fast_atan2(float(Ixy), float(lambda - Iyy)));
        theta *= kDeg2Rad;
        if (angle_diff(theta, reg_angle) > pr) theta += kPi;
        return theta;
    }

    void region2rect(const std::vector<RegionPoint>& reg, double reg_angle, Rect& rec) const {
        double x = 0, y = 0, sum = 0;
        for (const RegionPoint& r : reg) {
            x += (double)r.x * r.modgrad;
            y += (double)r.y * r.modgrad;
            sum += r.modgrad;
        }
        x /= sum;
        y /= sum;
        const double theta = get_theta(reg, x, y, reg_angle, prec);
        const double dx = gfplo_cos(theta), dy = gfplo_sin(theta);
        double l_min = 0, l_max = 0, w_min = 0, w_max = 0;
        for (const RegionPoint& r : reg) {
            const double rdx = (double)r.x - x, rdy = (double)r.y - y;
            const double l = rdx * dx + rdy * dy;
            const double w = -rdx * dy + rdy * dx;
            if (l > l_max) l_max = l;
            else if (l < l_min) l_min = l;
            if (w > w_max) w_max = w;
            else if (w < w_min) w_min = w;
        }
        rec.x1 = x + l_min * dx;
        rec.y1 = y + l_min * dy;
        rec.x2 = x + l_max * dx;
        rec.y2 = y + l_max * dy;
        rec.width = w_max - w_min;
        rec.x = x;
        rec.y = y;
        rec.theta = theta;
        rec.dx = dx;
        rec.dy = dy;
        rec.prec = prec;
        rec.p = p;
        if (rec.width < 1.0) rec.width = 1.0;
    }

    bool reduce_region_radius(std::vector<RegionPoint>& reg, double reg_angle, Rect& rec, double density) {
        const double xc = (double)reg[0].x, yc = (double)reg[0].y;
        const double rad1 = dist_sq(xc, yc, rec.x1, rec.y1), rad2 = dist_sq(xc, yc, rec.x2, rec.y2);
        double rad_sq = rad1 > rad2 ? rad1 : rad2;
        while (density < density_th) {
            rad_sq *= 0.75 * 0.75;
            for (size_t i = 0; i < reg.size(); ++i) {
                if (dist_sq(xc, yc, (double)reg[i].x, (double)reg[i].y) > rad_sq) {
                    used[(size_t)reg[i].y * W + reg[i].x] = 0;
                    std::swap(reg[i], reg[reg.size() - 1]);
                    reg.pop_back();
                    --i;
                }
            }
            if (reg.size() < 2) return false;
            region2rect(reg, reg_angle, rec);
            density = (double)reg.size() / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
        }
        return true;
    }

    bool refine(std::vector<RegionPoint>& reg, double reg_angle, Rect& rec) {
        double density = (double)reg.size() / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
        if (density >= density_th) return true;
        const double xc = (double)reg[0].x, yc = (double)reg[0].y;
        const double ang_c = reg[0].angle;
        double sum = 0, s_sum = 0;
        int n = 0;
        for (size_t i = 0; i < reg.size(); ++i) {
            used[(size_t)reg[i].y * W + reg[i].x] = 0;
            if (dist(xc, yc, (double)reg[i].x, (double)reg[i].y) < rec.width) {
                const double ang_d = angle_diff_signed(reg[i].angle, ang_c);
                sum += ang_d;
                s_sum += ang_d * ang_d;
                ++n;
            }
        }
        const double mean_angle = sum / (double)n;
        const double tau = 2.0 * std::sqrt((s_sum - 2.0 * mean_angle * sum) / (double)n + mean_angle * mean_angle);
        region_grow(reg[0].x, reg[0].y, reg, reg_angle, tau);
        if (reg.size() < 2) return false;
        region2rect(reg, reg_angle, rec);
        density = (double)reg.size() / (dist(rec.x1, rec.y1, rec.x2, rec.y2) * rec.width);
        if (density < density_th) return reduce_region_radius(reg, reg_angle, rec, density);
        return true;
    }

    void flsd(const uint8_t* img, std::vector<float>& lines) {
        ll_angle(img);
        used.assign((size_t)W * H, 0);
        std::vector<RegionPoint> reg;
        for (const NormPoint& np : ordered) {
            if (used[(size_t)np.y * W + np.x] != 0 || ang(np.x, np.y) == kNotDef) continue;
            double reg_angle;
            region_grow(np.x, np.y, reg, reg_angle, prec);
            if (reg.size() < min_reg_size) continue;
            Rect rec;
            region2rect(reg, reg_angle, rec);
            if (!refine(reg, reg_angle, rec)) continue;   // LSD_REFINE_STD: no rect_improve / NFA
            rec.x1 += 0.5;
            rec.y1 += 0.5;
            rec.x2 += 0.5;
            rec.y2 += 0.5;
            lines.push_back((float)rec.x1);
            lines.push_back((float)rec.y1);
            lines.push_back((float)rec.x2);
            lines.push_back((float)rec.y2);
        }
    }
};

struct Kl { float sx, sy, ex, ey, angle, response; };

}  // namespace

extern "C" double gfplo_atan2(double y, double x) { return fd_atan2(y, x); }

// S2: the library's std::sort by descending high 32 bits (what the GPU restatement must equal)
extern "C" int gfplo_sort_desc(uint64_t* a, int n) {
    if (!a || n < 0) return GFPL_E_INVALID;
    std::sort(a, a + n, [](uint64_t x, uint64_t y) { return (uint32_t)(x >> 32) > (uint32_t)(y >> 32); });
    return GFPL_OK;
}

// per-image constants of flsd (S5), shared with the GPU path's host setup
extern "C" int gfplo_lsd_constants(const gfpl_lsd_params* prm, int width, int height, double* prec, double* rho,
                                   int* min_reg_size) {
    if (!prm || width < 2 || height < 2) return GFPL_E_INVALID;
    const double pr = kPi * prm->ang_th / 180;
    const double p = prm->ang_th / 180;
    if (prec) *prec = pr;
    if (rho) *rho = prm->quant / std::sin(pr);
    const double log_nt = 5 * (std::log10((double)width) + std::log10((double)height)) / 2 + std::log10(11.0);
    if (min_reg_size) *min_reg_size = (int)(size_t)(-log_nt / std::log10(p));
    return GFPL_OK;
}

extern "C" int gfplo_lsd_detect(const gfpl_lsd_params* prm, const uint8_t* image, int width, int height, int kl_cap,
                                gfpl_keyline* kls, float* response, int* n_kl, float* segs, int seg_cap,
                                int* n_seg) {
    if (!prm || !image || width < 8 || height < 8 || !n_kl) return GFPL_E_INVALID;
    if (prm->refine != 1 || prm->scale != 1.0) return GFPL_E_UNSUPPORTED;
    Lsd L;
    L.W = width;
    L.H = height;
    L.n_bins = prm->n_bins;
    L.density_th = prm->density_th;
    L.p = prm->ang_th / 180;
    int mrs = 0;
    gfplo_lsd_constants(prm, width, height, &L.prec, &L.rho, &mrs);
    L.min_reg_size = (size_t)mrs;
    std::vector<float> lines;
    L.flsd(image, lines);
    const int ns = (int)(lines.size() / 4);
    if (n_seg) *n_seg = ns;
    if (segs) std::memcpy(segs, lines.data(), sizeof(float) * 4 * std::min(ns, seg_cap));
    // LSDDetector_custom.cpp:266-306
    std::vector<Kl> out;
    const int mx = std::max(width, height);
    for (int k = 0; k < ns; ++k) {
        float e[4] = {lines[4 * k], lines[4 * k + 1], lines[4 * k + 2], lines[4 * k + 3]};
        // checkLineExtremes (:78-103)
        for (int c = 0; c < 4; c += 2) {
            if (e[c] < 0) e[c] = 0;
            if (e[c] >= width) e[c] = (float)width - 1.0f;
            if (e[c + 1] < 0) e[c + 1] = 0;
            if (e[c + 1] >= height) e[c + 1] = (float)height - 1.0f;
        }
        const float d0 = e[0] - e[2], d1 = e[1] - e[3];
        const double length = (float)std::sqrt((double)d0 * (double)d0 + (double)d1 * (double)d1);   // S5
        if (!(length > prm->min_length)) continue;
        Kl kl;
        kl.sx = e[0];
        kl.sy = e[1];
        kl.ex = e[2];
        kl.ey = e[3];
        kl.angle = (float)fd_atan2((double)(kl.ey - kl.sy), (double)(kl.ex - kl.sx));   // S4
        kl.response = (float)length / (float)mx;
        out.push_back(kl);
    }
    // src/stereoFrame.cpp:1177-1185 (S7)
    if ((int)out.size() > prm->n_features && prm->n_features != 0) {
        std::sort(out.begin(), out.end(), [](const Kl& a, const Kl& b) { return a.response > b.response; });
        out.resize(prm->n_features);
    }
    *n_kl = (int)out.size();
    if ((int)out.size() > kl_cap) return GFPL_E_CAPACITY;
    for (size_t i = 0; i < out.size(); ++i) {
        if (kls) kls[i] = {out[i].sx, out[i].sy, out[i].ex, out[i].ey, out[i].angle, 0};
        if (response) response[i] = out[i].response;
    }
    return GFPL_OK;
}
