// gfpl_orb_oracle.cpp — CPU ORACLE of the ORB extraction row.
// TEST INFRASTRUCTURE ONLY (see gfpl_oracle.h): the checker of the GPU ORB path.
//
// Restates ORB_SLAM2::ORBextractor::operator() (src/ORBextractor.cc:1043-1105) as the
// reference constructs it on the path (src/stereoFrame.cpp:33-36: Config::orbNFeatures,
// Config::orbScaleFactor, Config::orbNLevels, iniThFAST 20, minThFAST 7):
//   ComputePyramid (:1107-1132), ComputeKeyPointsOctTree (:765-853) with FAST in 30-px
//   cells and DistributeOctTree (:539-763), IC_Angle (:77-104), GaussianBlur 7x7 sigma 2 +
//   computeOrbDescriptor (:108-148, :1034-1041), keypoint scaling (:1094-1101).
//
// The arithmetic of the OpenCV 3.4.1 calls it makes is third-party code absent from this
// image; the restatement pins the portable (scalar) OpenCV semantics, ledger O1-O7 (DESIGN.md
// §3): PARITY UNPINNED against the reference binary — x86 OpenCV builds may route resize /
// GaussianBlur / FAST through SIMD or IPP code that rounds some pixels differently.
//   O1 cv::resize INTER_LINEAR 8UC1: resizeGeneric_ with 11-bit fixed-point coefficients
//      (saturate_cast<short>(w * 2048)), HResizeLinear (exact int), VResizeLinear with
//      FixedPtCast<int, uchar, 22> ((s + 2^21) >> 22), rows clamped, xofs border rules.
//   O2 cv::GaussianBlur 7x7, sigma 2, BORDER_REFLECT_101, 8U: getGaussianKernel(CV_32F)
//      rounded to 8-bit integer taps, exact int row pass, column pass with
//      FixedPtCastEx<int, uchar>(16): (s + 2^15) >> 16.
//   O3 cv::FAST TYPE_9_16 with non-max suppression: FAST_t<16> + cornerScore<16>.
//   O4 cv::fastAtan2: the scalar float polynomial (degrees).
//   O5 computeOrbDescriptor's (float)cos / (float)sin of the float angle: the float of
//      the double (fdlibm) value.
//   O6 DistributeOctTree's sort of (size, node pointer) pairs: equal sizes ordered by node
//      creation (the reference orders them by heap address, which is allocator-dependent).
//   O7 no FP contraction (-ffp-contract=off), cvRound = round half to even.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <vector>

#include "../gf-pl-slam_amd/csrc/gfpl_orb_pattern.h"
#include "gfpl_oracle.h"

namespace {

constexpr int PATCH_SIZE = 31;
constexpr int HALF_PATCH_SIZE = 15;
constexpr int EDGE_THRESHOLD = 19;

inline int cv_round(double v) { return (int)std::nearbyint(v); }   // O7
inline int cv_round(float v) { return (int)std::nearbyintf(v); }
inline int cv_floor(double v) { return (int)std::floor(v); }
inline int cv_ceil(double v) { return (int)std::ceil(v); }
inline short sat_short(float v) {
    const int r = cv_round(v);
    return (short)std::min(std::max(r, -32768), 32767);
}
inline uint8_t sat_u8(int v) { return (uint8_t)std::min(std::max(v, 0), 255); }

struct Img {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
};

// ORBextractor::ORBextractor (:410-470)
struct Params {
    int nfeatures, nlevels, iniTh, minTh;
    float scaleFactor;
    std::vector<float> scale, invScale;
    std::vector<int> nPerLevel, umax;
};

Params make_params(const gfpl_orb_params& p) {
    Params o;
    o.nfeatures = p.nfeatures;
    o.scaleFactor = p.scale_factor;
    o.nlevels = p.nlevels;
    o.iniTh = p.ini_th_fast;
    o.minTh = p.min_th_fast;
    o.scale.assign(o.nlevels, 1.0f);
    for (int i = 1; i < o.nlevels; ++i) o.scale[i] = o.scale[i - 1] * o.scaleFactor;
    o.invScale.resize(o.nlevels);
    for (int i = 0; i < o.nlevels; ++i) o.invScale[i] = 1.0f / o.scale[i];
    o.nPerLevel.resize(o.nlevels);
    const float factor = 1.0f / o.scaleFactor;
    float nDesired = o.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)o.nlevels));
    int sum = 0;
    for (int l = 0; l < o.nlevels - 1; ++l) {
        o.nPerLevel[l] = cv_round(nDesired);
        sum += o.nPerLevel[l];
        nDesired *= factor;
    }
    o.nPerLevel[o.nlevels - 1] = std::max(o.nfeatures - sum, 0);
    o.umax.assign(HALF_PATCH_SIZE + 1, 0);
    const int vmax = cv_floor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
    const int vmin = cv_ceil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (int v = 0; v <= vmax; ++v) o.umax[v] = cv_round(std::sqrt(hp2 - v * v));
    for (int v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {   // symmetric
        while (o.umax[v0] == o.umax[v0 + 1]) ++v0;
        o.umax[v] = v0;
        ++v0;
    }
    return o;
}

// O1 — cv::resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR) for 8UC1
Img resize_linear(const Img& s, int dw, int dh) {
    const double scale_x = 1. / ((double)dw / s.w), scale_y = 1. / ((double)dh / s.h);
    std::vector<int> xofs(dw);
    std::vector<short> alpha(2 * (size_t)dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= s.w) {
            xmax = std::min(xmax, dx);
            if (sx >= s.w - 1) { fx = 0; sx = s.w - 1; }
        }
        xofs[dx] = sx;
        alpha[2 * dx] = sat_short((1.f - fx) * 2048);
        alpha[2 * dx + 1] = sat_short(fx * 2048);
    }
    auto hrow = [&](int y, std::vector<int>& D) {
        const uint8_t* S = &s.px[(size_t)y * s.w];
        for (int dx = 0; dx < dw; ++dx) {
            const int sx = xofs[dx];
            D[dx] = dx < xmax ? S[sx] * alpha[2 * dx] + S[sx + 1] * alpha[2 * dx + 1] : S[sx] * 2048;
        }
    };
    Img d;
    d.w = dw;
    d.h = dh;
    d.px.resize((size_t)dw * dh);
    std::vector<int> r0(dw), r1(dw);
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = cv_floor(fy);
        fy -= sy;
        const short b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
        auto clip = [&](int y) { return y >= 0 ? (y < s.h ? y : s.h - 1) : 0; };
        hrow(clip(sy), r0);
        hrow(clip(sy + 1), r1);
        for (int dx = 0; dx < dw; ++dx)
            d.px[(size_t)dy * dw + dx] = sat_u8((r0[dx] * b0 + r1[dx] * b1 + (1 << 21)) >> 22);
    }
    return d;
}

// ComputePyramid (:1107-1132); the level images (the bordered copies are never read:
// FAST cells, IC_Angle patches and descriptor patterns stay inside the level image)
std::vector<Img> pyramid(const Params& P, const Img& img) {
    std::vector<Img> pyr(P.nlevels);
    pyr[0] = img;
    for (int l = 1; l < P.nlevels; ++l)
        pyr[l] = resize_linear(pyr[l - 1], cv_round((float)img.w * P.invScale[l]), cv_round((float)img.h * P.invScale[l]));
    return pyr;
}

struct Kp {
    float x, y, response, angle;
    int octave;
};

// O3 — FAST_t<16> offsets (x, y) of the Bresenham circle, makeOffsets
const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                            {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// cornerScore<16>: the largest threshold at which the point is still a corner, minus 1
int corner_score(const Img& im, int x, int y, int threshold) {
    const int v = im.at(x, y);
    short d[25];
    for (int k = 0; k < 25; ++k) d[k] = (short)(v - im.at(x + kCircle[k & 15][0], y + kCircle[k & 15][1]));
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 5]);
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

// the segment test: >= 9 contiguous circle pixels all darker than v - t or all brighter
// than v + t (the circle wrapped to 25 entries, FAST_t's count > K)
bool is_corner(const Img& im, int x, int y, int t) {
    const int v = im.at(x, y);
    for (int pass = 0; pass < 2; ++pass) {
        int count = 0;
        for (int k = 0; k < 25; ++k) {
            const int p = im.at(x + kCircle[k & 15][0], y + kCircle[k & 15][1]);
            const bool hit = pass == 0 ? p < v - t : p > v + t;
            if (hit) {
                if (++count > 8) return true;
            } else {
                count = 0;
            }
        }
    }
    return false;
}

// cv::FAST(img(rowRange(y0, y1), colRange(x0, x1)), kps, t, true): keypoints in ROI
// coordinates, row-major; non-max suppression over the 3x3 neighbourhood of scores with
// 0 outside the ROI's detectable area [3, w - 3) x [3, h - 3)
void fast_roi(const Img& im, int x0, int y0, int x1, int y1, int t, std::vector<Kp>& out) {
    const int w = x1 - x0, h = y1 - y0;
    out.clear();
    if (w < 7 || h < 7) return;
    std::vector<int> score((size_t)w * h, 0);
    for (int y = 3; y < h - 3; ++y)
        for (int x = 3; x < w - 3; ++x)
            if (is_corner(im, x0 + x, y0 + y, t)) score[(size_t)y * w + x] = corner_score(im, x0 + x, y0 + y, t);
    for (int y = 3; y < h - 3; ++y)
        for (int x = 3; x < w - 3; ++x) {
            const int s = score[(size_t)y * w + x];
            if (!s && !is_corner(im, x0 + x, y0 + y, t)) continue;
            bool mx = true;
            for (int dy = -1; dy <= 1 && mx; ++dy)
                for (int dx = -1; dx <= 1; ++dx)
                    if ((dx || dy) && !(s > score[(size_t)(y + dy) * w + (x + dx)])) { mx = false; break; }
            if (mx) out.push_back(Kp{(float)x, (float)y, (float)s, -1.f, 0});
        }
}

// ExtractorNode / DistributeOctTree (:481-763)
struct Node {
    int ulx, uly, urx, ury, blx, bly, brx, bry;
    std::vector<Kp> keys;
    bool noMore = false;
    long long id = 0;   // creation order (O6)
};

void divide(const Node& n, Node& n1, Node& n2, Node& n3, Node& n4) {
    const int halfX = (int)std::ceil(static_cast<float>(n.urx - n.ulx) / 2);
    const int halfY = (int)std::ceil(static_cast<float>(n.bry - n.uly) / 2);
    n1.ulx = n.ulx; n1.uly = n.uly; n1.urx = n.ulx + halfX; n1.ury = n.uly;
    n1.blx = n.ulx; n1.bly = n.uly + halfY; n1.brx = n.ulx + halfX; n1.bry = n.uly + halfY;
    n2.ulx = n1.urx; n2.uly = n1.ury; n2.urx = n.urx; n2.ury = n.ury;
    n2.blx = n1.brx; n2.bly = n1.bry; n2.brx = n.urx; n2.bry = n.uly + halfY;
    n3.ulx = n1.blx; n3.uly = n1.bly; n3.urx = n1.brx; n3.ury = n1.bry;
    n3.blx = n.blx; n3.bly = n.bly; n3.brx = n1.brx; n3.bry = n.bly;
    n4.ulx = n3.urx; n4.uly = n3.ury; n4.urx = n2.brx; n4.ury = n2.bry;
    n4.blx = n3.brx; n4.bly = n3.bry; n4.brx = n.brx; n4.bry = n.bry;
    for (const Kp& kp : n.keys) {
        if (kp.x < n1.urx) {
            if (kp.y < n1.bry) n1.keys.push_back(kp);
            else n3.keys.push_back(kp);
        } else if (kp.y < n1.bry) {
            n2.keys.push_back(kp);
        } else {
            n4.keys.push_back(kp);
        }
    }
    n1.noMore = n1.keys.size() == 1;
    n2.noMore = n2.keys.size() == 1;
    n3.noMore = n3.keys.size() == 1;
    n4.noMore = n4.keys.size() == 1;
}

std::vector<Kp> distribute(const std::vector<Kp>& keys, int minX, int maxX, int minY, int maxY, int N) {
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    const float hX = static_cast<float>(maxX - minX) / nIni;
    long long next_id = 0;
    std::list<Node> nodes;
    std::vector<Node*> ini(nIni);
    for (int i = 0; i < nIni; ++i) {
        Node n;
        n.ulx = (int)(hX * static_cast<float>(i)); n.uly = 0;
        n.urx = (int)(hX * static_cast<float>(i + 1)); n.ury = 0;
        n.blx = n.ulx; n.bly = maxY - minY;
        n.brx = n.urx; n.bry = maxY - minY;
        n.id = next_id++;
        nodes.push_back(n);
        ini[i] = &nodes.back();
    }
    for (const Kp& kp : keys) ini[(size_t)(kp.x / hX)]->keys.push_back(kp);
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) { it->noMore = true; ++it; }
        else if (it->keys.empty()) it = nodes.erase(it);
        else ++it;
    }
    using Entry = std::pair<std::pair<int, long long>, std::list<Node>::iterator>;   // (size, creation id)
    std::vector<Entry> toExpand;
    auto push_children = [&](Node& n1, Node& n2, Node& n3, Node& n4, int* nToExpand) {
        for (Node* c : {&n1, &n2, &n3, &n4}) {
            if (c->keys.empty()) continue;
            c->id = next_id++;
            nodes.push_front(std::move(*c));
            if (nodes.front().keys.size() > 1) {
                if (nToExpand) ++*nToExpand;
                toExpand.push_back({{(int)nodes.front().keys.size(), nodes.front().id}, nodes.begin()});
            }
        }
    };
    bool finish = false;
    while (!finish) {
        const int prevSize = (int)nodes.size();
        int nToExpand = 0;
        toExpand.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {
            if (it->noMore) { ++it; continue; }
            Node n1, n2, n3, n4;
            divide(*it, n1, n2, n3, n4);
            push_children(n1, n2, n3, n4, &nToExpand);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == prevSize) {
            finish = true;
        } else if ((int)nodes.size() + nToExpand * 3 > N) {
            while (!finish) {
                const int prev = (int)nodes.size();
                std::vector<Entry> prevExpand = toExpand;
                toExpand.clear();
                std::sort(prevExpand.begin(), prevExpand.end(),
                          [](const Entry& a, const Entry& b) { return a.first < b.first; });
                for (int j = (int)prevExpand.size() - 1; j >= 0; --j) {
                    Node n1, n2, n3, n4;
                    divide(*prevExpand[j].second, n1, n2, n3, n4);
                    push_children(n1, n2, n3, n4, nullptr);
                    nodes.erase(prevExpand[j].second);
                    if ((int)nodes.size() >= N) break;
                }
                if ((int)nodes.size() >= N || (int)nodes.size() == prev) finish = true;
            }
        }
    }
    std::vector<Kp> out;
    for (const Node& n : nodes) {
        const Kp* best = &n.keys[0];
        for (size_t k = 1; k < n.keys.size(); ++k)
            if (n.keys[k].response > best->response) best = &n.keys[k];
        out.push_back(*best);
    }
    return out;
}

// O4 — cv::fastAtan2 (degrees)
float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI), p3 = -0.3258083974640975f * (float)(180 / M_PI),
                p5 = 0.1555786518463281f * (float)(180 / M_PI), p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// IC_Angle (:77-104)
float ic_angle(const Img& im, const Kp& kp, const std::vector<int>& umax) {
    int m_01 = 0, m_10 = 0;
    const int cx = cv_round(kp.x), cy = cv_round(kp.y);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * im.at(cx + u, cy);
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            const int val_plus = im.at(cx + u, cy + v), val_minus = im.at(cx + u, cy - v);
            v_sum += val_plus - val_minus;
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2((float)m_01, (float)m_10);
}

// O2 — cv::GaussianBlur(src, dst, Size(7, 7), 2, 2, BORDER_REFLECT_101) for 8U
Img gaussian_blur(const Img& s) {
    float cf[7];
    double sum = 0;
    const double scale2X = -0.5 / (2.0 * 2.0);
    for (int i = 0; i < 7; ++i) {
        const double x = i - 3.0;
        cf[i] = (float)std::exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    int k[7];
    for (int i = 0; i < 7; ++i) k[i] = cv_round((float)(cf[i] * sum) * 256.0f);
    auto refl = [](int i, int n) {   // BORDER_REFLECT_101
        if (n == 1) return 0;
        while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
        return i;
    };
    std::vector<int> rows((size_t)s.w * s.h);
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            int a = 0;
            for (int t = 0; t < 7; ++t) a += k[t] * s.at(refl(x + t - 3, s.w), y);
            rows[(size_t)y * s.w + x] = a;
        }
    Img d = s;
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            int a = k[3] * rows[(size_t)y * s.w + x];
            for (int t = 1; t <= 3; ++t)
                a += k[3 + t] * (rows[(size_t)refl(y + t, s.h) * s.w + x] + rows[(size_t)refl(y - t, s.h) * s.w + x]);
            d.px[(size_t)y * s.w + x] = sat_u8((a + (1 << 15)) >> 16);
        }
    return d;
}

// computeOrbDescriptor (:108-148); O5
void orb_descriptor(const Img& blur, const Kp& kp, uint8_t* desc) {
    const float factorPI = (float)(M_PI / 180.f);
    const float angle = kp.angle * factorPI;
    const float a = (float)gfplo_cos((double)angle), b = (float)gfplo_sin((double)angle);
    const int cx = cv_round(kp.x), cy = cv_round(kp.y);
    auto get = [&](int idx) {
        const int px = kOrbPattern[2 * idx], py = kOrbPattern[2 * idx + 1];
        const int dy = cv_round(px * b + py * a), dx = cv_round(px * a - py * b);
        return (int)blur.at(cx + dx, cy + dy);
    };
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int bit = 0; bit < 8; ++bit) {
            const int t0 = get(16 * i + 2 * bit), t1 = get(16 * i + 2 * bit + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

}  // namespace

extern "C" int gfplo_orb_extract(const gfpl_orb_params* prm, const uint8_t* image, int width, int height,
                                 int kp_cap, gfpl_keypoint* kps, float* angle, float* response, uint8_t* desc,
                                 int* n_kp, uint8_t* pyr_out) {
    if (!prm || !image || width < 2 * EDGE_THRESHOLD || height < 2 * EDGE_THRESHOLD || !n_kp) return GFPL_E_INVALID;
    if (prm->nlevels < 1 || prm->nlevels > GFPL_MAX_LEVELS || !(prm->scale_factor > 1.0f)) return GFPL_E_INVALID;
    const Params P = make_params(*prm);
    // levels without a 30-px cell or an initial octree node are undefined behaviour in the
    // reference (nCols = 0 divides by zero, nIni = 0 indexes an empty vector): refused
    for (int l = 0; l < P.nlevels; ++l) {
        const int lw = cv_round((float)width * P.invScale[l]), lh = cv_round((float)height * P.invScale[l]);
        const float wf = (float)(lw - 2 * EDGE_THRESHOLD + 6), hf = (float)(lh - 2 * EDGE_THRESHOLD + 6);
        if ((int)(wf / 30) < 1 || (int)(hf / 30) < 1 || (int)std::round(wf / hf) < 1) return GFPL_E_INVALID;
    }
    Img img;
    img.w = width;
    img.h = height;
    img.px.assign(image, image + (size_t)width * height);
    const std::vector<Img> pyr = pyramid(P, img);
    if (pyr_out) {
        size_t off = 0;
        for (const Img& l : pyr) {
            std::memcpy(pyr_out + off, l.px.data(), l.px.size());
            off += l.px.size();
        }
    }
    // ComputeKeyPointsOctTree (:765-853)
    std::vector<std::vector<Kp>> all(P.nlevels);
    const float W = 30;
    std::vector<Kp> cell;
    for (int level = 0; level < P.nlevels; ++level) {
        const Img& im = pyr[level];
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = im.w - EDGE_THRESHOLD + 3, maxBorderY = im.h - EDGE_THRESHOLD + 3;
        std::vector<Kp> toDistribute;
        const float width_f = (float)(maxBorderX - minBorderX), height_f = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width_f / W), nRows = (int)(height_f / W);
        const int wCell = (int)std::ceil(width_f / nCols), hCell = (int)std::ceil(height_f / nRows);
        for (int i = 0; i < nRows; ++i) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; ++j) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                fast_roi(im, (int)iniX, (int)iniY, (int)maxX, (int)maxY, P.iniTh, cell);
                if (cell.empty()) fast_roi(im, (int)iniX, (int)iniY, (int)maxX, (int)maxY, P.minTh, cell);
                for (Kp kp : cell) {
                    kp.x += j * wCell;
                    kp.y += i * hCell;
                    toDistribute.push_back(kp);
                }
            }
        }
        std::vector<Kp>& keypoints = all[level];
        keypoints = distribute(toDistribute, minBorderX, maxBorderX, minBorderY, maxBorderY, P.nPerLevel[level]);
        for (Kp& kp : keypoints) {
            kp.x += minBorderX;
            kp.y += minBorderY;
            kp.octave = level;
        }
        for (Kp& kp : keypoints) kp.angle = ic_angle(im, kp, P.umax);   // computeOrientation (:850-852)
    }
    int n = 0;
    for (int level = 0; level < P.nlevels; ++level) n += (int)all[level].size();
    if (n > kp_cap) return GFPL_E_CAPACITY;
    int o = 0;
    for (int level = 0; level < P.nlevels; ++level) {
        std::vector<Kp>& keypoints = all[level];
        if (keypoints.empty()) continue;
        const Img blur = gaussian_blur(pyr[level]);
        for (Kp& kp : keypoints) {
            if (desc) orb_descriptor(blur, kp, desc + 32 * (size_t)o);
            if (level != 0) {
                kp.x *= P.scale[level];
                kp.y *= P.scale[level];
            }
            if (kps) kps[o] = gfpl_keypoint{kp.x, kp.y, kp.octave};
            if (angle) angle[o] = kp.angle;
            if (response) response[o] = kp.response;
            ++o;
        }
    }
    *n_kp = n;
    return GFPL_OK;
}

// components, for the known-answer tests
extern "C" int gfplo_orb_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    Img s;
    s.w = sw;
    s.h = sh;
    s.px.assign(src, src + (size_t)sw * sh);
    const Img d = resize_linear(s, dw, dh);
    std::memcpy(dst, d.px.data(), d.px.size());
    return GFPL_OK;
}

extern "C" int gfplo_orb_blur(const uint8_t* src, int w, int h, uint8_t* dst) {
    Img s;
    s.w = w;
    s.h = h;
    s.px.assign(src, src + (size_t)w * h);
    const Img d = gaussian_blur(s);
    std::memcpy(dst, d.px.data(), d.px.size());
    return GFPL_OK;
}

extern "C" int gfplo_orb_fast(const uint8_t* img, int w, int h, int threshold, int cap, float* xy_score) {
    Img s;
    s.w = w;
    s.h = h;
    s.px.assign(img, img + (size_t)w * h);
    std::vector<Kp> out;
    fast_roi(s, 0, 0, w, h, threshold, out);
    const int n = (int)std::min<size_t>(out.size(), (size_t)cap);
    for (int i = 0; i < n; ++i) {
        xy_score[3 * i] = out[i].x;
        xy_score[3 * i + 1] = out[i].y;
        xy_score[3 * i + 2] = out[i].response;
    }
    return (int)out.size();
}

extern "C" float gfplo_fast_atan2(float y, float x) { return fast_atan2(y, x); }
