// Deterministic synthetic stereo frames (see gfpl_synth.h).
//
// Recipe (SURVEY.md §8(d) "Per-frame generation recipe"):
//  * landmarks / 3-D segments sampled in the first camera's frustum, fixed per
//    sequence; camera moves forward with a constant yaw rate (or follows a
//    given ground-truth trajectory, e.g. EuRoC config/asl/gt-ass/*/groundtruth.txt);
//  * ORB octave per landmark drawn with ORBextractor's per-level quotas
//    (src/ORBextractor.cc:433-446); keypoints = projections + jitter;
//  * a random 256-bit code per landmark, each observation flips ~1/16 of the
//    bits; distractors carry random codes;
//  * right pyramid = uint8 noise; for each stereo-visible landmark the same
//    11x11 patch is stamped at (uL, vL) and (uR, vL) of its octave so the
//    right-pyramid self-SAD of subPixelStereoRefine_ORBSLAM (quirk Q1,
//    src/stereoFrame.cpp:357) has its minimum at the true shift.
#include "gfpl_synth.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uni() { return (double)(next() >> 11) * 0x1.0p-53; }          // [0,1)
    double uni(double a, double b) { return a + (b - a) * uni(); }
    double gauss() {
        double u1 = uni(), u2 = uni();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

uint64_t mix(uint64_t a, uint64_t b) {
    Rng r(a * 0xD1B54A32D192ED03ull ^ (b + 0x8CB92BA72F3D8DD7ull));
    r.next();
    return r.next();
}

struct Pose { double R[9]; double t[3]; };   // T_w<-c : X_w = R X_c + t

void pose_at(const gfpl_synth_params* p, int k, Pose* T, double* ts) {
    if (p->traj && p->n_traj > 0) {
        int kk = std::min(std::max(k, 0), p->n_traj - 1);   // callers refuse k >= n_traj
        const double* r = p->traj + 12 * kk;
        // rebase on the first pose so the sequence starts at identity
        const double* r0 = p->traj;
        double R0[9] = {r0[0], r0[1], r0[2], r0[4], r0[5], r0[6], r0[8], r0[9], r0[10]};
        double t0[3] = {r0[3], r0[7], r0[11]};
        double Rk[9] = {r[0], r[1], r[2], r[4], r[5], r[6], r[8], r[9], r[10]};
        double tk[3] = {r[3], r[7], r[11]};
        // T = T0^-1 Tk
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int m = 0; m < 3; ++m) s += R0[m * 3 + i] * Rk[m * 3 + j];
                T->R[i * 3 + j] = s;
            }
        for (int i = 0; i < 3; ++i) {
            double s = 0;
            for (int m = 0; m < 3; ++m) s += R0[m * 3 + i] * (tk[m] - t0[m]);
            T->t[i] = s;
        }
        *ts = p->traj_t ? p->traj_t[kk] - p->traj_t[0] + 1.0 : 1.0 + k * p->dt;
        return;
    }
    double time = k * p->dt;
    double psi = p->yaw_rate * time;
    double c = std::cos(psi), s = std::sin(psi);
    // rotation about the camera y axis (down): x right, z forward
    double R[9] = {c, 0, s, 0, 1, 0, -s, 0, c};
    std::memcpy(T->R, R, sizeof R);
    // integrate forward velocity along the heading: closed form for constant yaw rate
    if (std::fabs(p->yaw_rate) < 1e-12) {
        T->t[0] = 0; T->t[1] = 0; T->t[2] = p->v_fwd * time;
    } else {
        double w = p->yaw_rate;
        T->t[0] = p->v_fwd * (1.0 - std::cos(psi)) / w;
        T->t[1] = 0;
        T->t[2] = p->v_fwd * std::sin(psi) / w;
    }
    *ts = 1.0 + time;
}

// world -> camera
void w2c(const Pose& T, const double Xw[3], double Xc[3]) {
    double d[3] = {Xw[0] - T.t[0], Xw[1] - T.t[1], Xw[2] - T.t[2]};
    for (int i = 0; i < 3; ++i) Xc[i] = T.R[0 * 3 + i] * d[0] + T.R[1 * 3 + i] * d[1] + T.R[2 * 3 + i] * d[2];
}
void c2w(const Pose& T, const double Xc[3], double Xw[3]) {
    for (int i = 0; i < 3; ++i)
        Xw[i] = T.R[i * 3 + 0] * Xc[0] + T.R[i * 3 + 1] * Xc[1] + T.R[i * 3 + 2] * Xc[2] + T.t[i];
}

struct Landmark { double X[3]; int octave; uint8_t code[32]; uint64_t key; };
struct Segment  { double S[3], E[3]; uint8_t code[32]; uint64_t key; };

void rand_code(Rng& r, uint8_t* c) {
    for (int i = 0; i < 4; ++i) { uint64_t v = r.next(); std::memcpy(c + 8 * i, &v, 8); }
}
void observe_code(Rng& r, const uint8_t* code, uint8_t* out) {
    for (int i = 0; i < 4; ++i) {
        uint64_t v; std::memcpy(&v, code + 8 * i, 8);
        uint64_t flip = r.next() & r.next() & r.next() & r.next();   // p = 1/16 per bit
        v ^= flip;
        std::memcpy(out + 8 * i, &v, 8);
    }
}

struct World {
    std::vector<Landmark> pts;
    std::vector<Segment> lines;
};

// ORB per-level quotas (src/ORBextractor.cc:433-446), normalised to probabilities
std::vector<double> level_quota(const gfpl_synth_params* p, const gfpl_camera* cam) {
    int nl = cam->n_levels;
    std::vector<double> quota(nl);
    double factor = 1.0 / (double)cam->scale[1 < nl ? 1 : 0];
    double nd = p->n_kp * (1 - factor) / (1 - std::pow(factor, (double)nl));
    double sum = 0;
    for (int l = 0; l < nl - 1; ++l) { quota[l] = std::round(nd); sum += quota[l]; nd *= factor; }
    quota[nl - 1] = std::max(p->n_kp - sum, 0.0);
    double tot = 0; for (double q : quota) tot += q;
    for (double& q : quota) q /= tot;
    return quota;
}

void sample_landmark(Rng& r, const gfpl_synth_params* p, const gfpl_camera* cam, const std::vector<double>& quota,
                     const Pose& T, Landmark& L) {
    const int nl = cam->n_levels;
    const double m = p->margin;
    double u = r.uni(m, cam->width - m), v = r.uni(m, cam->height - m);
    double iz = r.uni(1.0 / p->z_max, 1.0 / p->z_min);   // uniform in inverse depth
    double z = 1.0 / iz;
    double Xc[3] = {(u - cam->cx) * z / cam->fx, (v - cam->cy) * z / cam->fy, z};
    c2w(T, Xc, L.X);
    double a = r.uni(), acc = 0; L.octave = nl - 1;
    for (int l = 0; l < nl; ++l) { acc += quota[l]; if (a < acc) { L.octave = l; break; } }
    rand_code(r, L.code);
    L.key = r.next();
}

void sample_segment(Rng& r, const gfpl_synth_params* p, const gfpl_camera* cam, const Pose& T, Segment& S) {
    const double m = p->margin;
    double u = r.uni(m, cam->width - m), v = r.uni(m, cam->height - m);
    double z = r.uni(p->z_min * 1.5, p->z_max * 0.8);
    double Xc[3] = {(u - cam->cx) * z / cam->fx, (v - cam->cy) * z / cam->fy, z};
    double d[3] = {r.gauss(), r.gauss(), 0.3 * r.gauss()};
    double n = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) + 1e-12;
    double len = r.uni(0.3, 1.5) * z / 4.0;
    double Sc[3], Ec[3];
    for (int k = 0; k < 3; ++k) { Sc[k] = Xc[k] - 0.5 * len * d[k] / n; Ec[k] = Xc[k] + 0.5 * len * d[k] / n; }
    c2w(T, Sc, S.S);
    c2w(T, Ec, S.E);
    rand_code(r, S.code);
    S.key = r.next();
}

// cv::resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR) for 8UC1 (OpenCV's 11-bit fixed-point
// resizeGeneric_: exact horizontal blend, vertical (s + 2^21) >> 22, rows clamped, the xofs border
// rule), level by level as ComputePyramid builds the right pyramid; the same arithmetic as the
// device's k_orb_resize (tests/test_synth.py pins it against the ORB oracle's restatement)
inline int16_t sat_s16(float v) {
    const int r = (int)std::nearbyintf(v);
    return (int16_t)std::min(std::max(r, -32768), 32767);
}
void resize_linear_u8(const uint8_t* s, int sw, int sh, uint8_t* d, int dw, int dh) {
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    std::vector<int> xofs(dw), r0(dw), r1(dw);
    std::vector<int16_t> alpha(2 * (size_t)dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        alpha[2 * dx] = sat_s16((1.f - fx) * 2048);
        alpha[2 * dx + 1] = sat_s16(fx * 2048);
    }
    auto hrow = [&](int y, std::vector<int>& D) {
        const uint8_t* S = s + (size_t)y * sw;
        for (int dx = 0; dx < dw; ++dx) {
            const int sx = xofs[dx];
            D[dx] = dx < xmax ? S[sx] * alpha[2 * dx] + S[sx + 1] * alpha[2 * dx + 1] : S[sx] * 2048;
        }
    };
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = (int)std::floor(fy);
        fy -= sy;
        const int16_t b0 = sat_s16((1.f - fy) * 2048), b1 = sat_s16(fy * 2048);
        auto clip = [&](int y) { return y >= 0 ? (y < sh ? y : sh - 1) : 0; };
        hrow(clip(sy), r0);
        hrow(clip(sy + 1), r1);
        for (int dx = 0; dx < dw; ++dx) {
            const int v = (r0[dx] * b0 + r1[dx] * b1 + (1 << 21)) >> 22;
            d[(size_t)dy * dw + dx] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    }
}

// The world seen at frame k.  respawn == 0: one pool sampled in the first camera's
// frustum, fixed for the whole sequence (it drains as the camera moves on).
// respawn == L > 0: every pool slot lives L frames and is re-sampled in the frustum of
// the camera at its spawn frame, with a per-slot phase, so at any frame the pool's ages
// are spread uniformly over 0..L-1 and the share of visible landmarks (hence the
// true-keypoint count) is stationary.  Slot i at frame k: epoch e = (k + phase_i) / L,
// spawn frame k - (k + phase_i) % L; everything drawn from (seed, seq, slot, epoch).
void build_world(const gfpl_synth_params* p, const gfpl_camera* cam, int seq, int k, World* W) {
    const std::vector<double> quota = level_quota(p, cam);
    W->pts.resize(p->n_world_pts);
    W->lines.resize(p->n_world_lines);
    if (p->respawn <= 0) {
        Rng r(mix(p->seed, 0x1000000ull + (uint64_t)seq));
        Pose T0; double ts;
        pose_at(p, 0, &T0, &ts);
        for (int i = 0; i < p->n_world_pts; ++i) sample_landmark(r, p, cam, quota, T0, W->pts[i]);
        for (int i = 0; i < p->n_world_lines; ++i) sample_segment(r, p, cam, T0, W->lines[i]);
        return;
    }
    const int L = p->respawn;
    std::vector<Pose> spawn(L);   // spawn[a] = pose of frame k - a (trajectories: clamped at frame 0)
    for (int a = 0; a < L; ++a) {
        double ts;
        pose_at(p, k - a, &spawn[a], &ts);   // synthetic motion extends to negative times
    }
    const uint64_t sk = mix(p->seed, 0x5000000ull + (uint64_t)seq);
    for (int kind = 0; kind < 2; ++kind) {
        const int n = kind == 0 ? p->n_world_pts : p->n_world_lines;
        for (int i = 0; i < n; ++i) {
            const uint64_t slot = mix(sk, ((uint64_t)kind << 32) | (uint64_t)i);
            const int phase = (int)(slot % (uint64_t)L);
            const int64_t t = (int64_t)k + phase;
            const uint64_t epoch = (uint64_t)(t / L);
            const int age = (int)(t % L);
            Rng r(mix(slot, epoch));
            if (kind == 0) sample_landmark(r, p, cam, quota, spawn[age], W->pts[i]);
            else sample_segment(r, p, cam, spawn[age], W->lines[i]);
        }
    }
}

inline bool in_img(double u, double v, const gfpl_camera* cam, double m) {
    return u >= m && u <= cam->width - 1 - m && v >= m && v <= cam->height - 1 - m;
}

template <typename T> void shuffle(std::vector<T>& a, Rng& r) {
    for (size_t i = a.size(); i > 1; --i) {
        size_t j = (size_t)(r.next() % i);
        std::swap(a[i - 1], a[j]);
    }
}

}  // namespace

extern "C" void gfpl_synth_default(gfpl_synth_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->n_kp = 2000;
    p->n_kl = 500;
    p->n_world_pts = 2600;
    p->n_world_lines = 700;
    p->dt = 0.05;
    p->v_fwd = 0.5;
    p->yaw_rate = 2.0 * 3.14159265358979 / 180.0;
    p->z_min = 1.0;
    p->z_max = 8.0;
    p->px_noise = 0.3;
    p->distractor_frac = 0.1;
    p->margin = 40;
    p->seed = 0x9E3779B97F4A7C15ull;
}

extern "C" int gfpl_synth_frame_ex(const gfpl_synth_params* p, const gfpl_camera* cam,
                                   int seq, int k, int kp_cap, int kl_cap,
                                   int* n_kp_l, int* n_kp_r, gfpl_keypoint* kp_l, gfpl_keypoint* kp_r,
                                   uint8_t* pdesc_l, uint8_t* pdesc_r,
                                   int* n_kl_l, int* n_kl_r, gfpl_keyline* kl_l, gfpl_keyline* kl_r,
                                   uint8_t* ldesc_l, uint8_t* ldesc_r,
                                   uint8_t* pyr_r, double* time_stamp, double* T_wc_out, int* n_true_out) {
    if (!p || !cam || p->n_kp > kp_cap || p->n_kl > kl_cap || k < 0) return GFPL_E_INVALID;
    if (p->traj && k >= p->n_traj) return GFPL_E_INVALID;   // past the loaded trajectory: no wrap-around
    World W;
    build_world(p, cam, seq, k, &W);
    Pose T; double ts;
    pose_at(p, k, &T, &ts);
    if (time_stamp) *time_stamp = ts;
    if (T_wc_out) {
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) T_wc_out[i * 4 + j] = T.R[i * 3 + j];
            T_wc_out[i * 4 + 3] = T.t[i];
        }
        T_wc_out[12] = T_wc_out[13] = T_wc_out[14] = 0; T_wc_out[15] = 1;
    }
    Rng r(mix(mix(p->seed, 0x2000000ull + (uint64_t)seq), (uint64_t)k));
    const double m = p->margin;
    const double fx = cam->fx, fy = cam->fy, cx = cam->cx, cy = cam->cy, b = cam->b;

    // ---- right pyramid noise (level 0 only when the levels are resized from it)
    const int64_t noise_bytes = p->pyr_from_l0 ? (int64_t)cam->lvl_cols[0] * cam->lvl_rows[0] : cam->pyr_bytes;
    if (p->pyr_from_l0) std::memset(pyr_r + noise_bytes, 0, (size_t)(cam->pyr_bytes - noise_bytes));
    for (int64_t i = 0; i < noise_bytes; i += 8) {
        uint64_t v = r.next();
        int64_t nb = std::min<int64_t>(8, cam->pyr_bytes - i);
        std::memcpy(pyr_r + i, &v, (size_t)nb);
    }

    // ---- points
    struct Obs { double ul, vl, ur, vr; int lm; };
    std::vector<Obs> vis;
    for (int i = 0; i < (int)W.pts.size(); ++i) {
        double Xc[3]; w2c(T, W.pts[i].X, Xc);
        if (Xc[2] < p->z_min * 0.8 || Xc[2] > p->z_max * 1.5) continue;
        double u = cx + fx * Xc[0] / Xc[2], v = cy + fy * Xc[1] / Xc[2];
        double d = fx * b / Xc[2];
        if (!in_img(u, v, cam, m) || !in_img(u - d, v, cam, m)) continue;
        vis.push_back({u, v, u - d, v, i});
    }
    int n_true = (int)std::lround(p->n_kp * (1.0 - p->distractor_frac));
    if ((int)vis.size() > n_true) vis.resize(n_true);
    std::vector<gfpl_keypoint> L, R;
    std::vector<std::array<uint8_t, 32>> DL, DR;
    for (const Obs& o : vis) {
        const Landmark& lm = W.pts[o.lm];
        Rng ro(mix(mix(lm.key, (uint64_t)k), 7));
        gfpl_keypoint a, c;
        // outliers: the observation (both images, and its stamped patch) moves by 3-8 px
        double ox = 0.0, oy = 0.0;
        if (p->outlier_frac > 0.0) {
            Rng rq(mix(mix(lm.key, (uint64_t)k), 13));
            if (rq.uni(0.0, 1.0) < p->outlier_frac) {
                ox = rq.uni(3.0, 8.0) * ((rq.next() >> 63) ? -1.0 : 1.0);
                oy = rq.uni(3.0, 8.0) * ((rq.next() >> 63) ? -1.0 : 1.0);
            }
        }
        a.x = (float)(o.ul + ox + p->px_noise * ro.gauss());
        a.y = (float)(o.vl + oy + p->px_noise * ro.gauss());
        a.octave = lm.octave;
        c.x = (float)(o.ur + ox + p->px_noise * ro.gauss());
        c.y = (float)(o.vr + oy + p->px_noise * ro.gauss());
        c.octave = lm.octave;
        std::array<uint8_t, 32> dl, dr;
        observe_code(ro, lm.code, dl.data());
        observe_code(ro, lm.code, dr.data());
        L.push_back(a); R.push_back(c); DL.push_back(dl); DR.push_back(dr);
        // stamp an 11x11 patch at (uL,vL) and (uR,vL) of the octave level
        int o_ = lm.octave;
        float s = cam->inv_scale[o_];
        int cols = cam->lvl_cols[o_], rows = cam->lvl_rows[o_];
        uint8_t* img = pyr_r + cam->lvl_offset[o_];
        int vv = (int)std::lround((o.vl + oy) * s);
        int ul = (int)std::lround((o.ul + ox) * s), ur = (int)std::lround((o.ur + ox) * s);
        uint8_t patch[121];
        for (int q = 0; q < 121; ++q) patch[q] = (uint8_t)(ro.next() >> 56);
        if (p->pyr_from_l0) {
            // level 0: the patch magnified by the octave's scale S (nearest cell), so the
            // resized level o shows it around the keypoint's level-o position
            const double S = cam->scale[o_], iS = 1.0 / S;
            const int W0 = cam->lvl_cols[0], H0 = cam->lvl_rows[0];
            const double yc = o.vl + oy;
            for (int pass = 0; pass < 2; ++pass) {
                const double xc = (pass == 0 ? o.ul : o.ur) + ox;
                const int x0 = std::max((int)std::floor(xc - 5.5 * S), 0), x1 = std::min((int)std::ceil(xc + 5.5 * S), W0 - 1);
                const int y0 = std::max((int)std::floor(yc - 5.5 * S), 0), y1 = std::min((int)std::ceil(yc + 5.5 * S), H0 - 1);
                int cxs[64];   // the patch column of each level-0 column (separable nearest cell)
                const int nx = std::min(x1 - x0 + 1, 64);
                for (int i = 0; i < nx; ++i)
                    cxs[i] = 5 + std::min(std::max((int)std::lround((x0 + i - xc) * iS), -5), 5);
                for (int yy = y0; yy <= y1; ++yy) {
                    const uint8_t* prow = patch + 11 * (5 + std::min(std::max((int)std::lround((yy - yc) * iS), -5), 5));
                    uint8_t* drow = pyr_r + (int64_t)yy * W0 + x0;
                    for (int i = 0; i < nx; ++i) drow[i] = prow[cxs[i]];
                }
            }
            continue;
        }
        for (int pass = 0; pass < 2; ++pass) {
            int uc = pass == 0 ? ul : ur;
            for (int dy = -5; dy <= 5; ++dy)
                for (int dx = -5; dx <= 5; ++dx) {
                    int yy = vv + dy, xx = uc + dx;
                    if (yy < 0 || yy >= rows || xx < 0 || xx >= cols) continue;
                    img[(int64_t)yy * cols + xx] = patch[(dy + 5) * 11 + dx + 5];
                }
        }
    }
    if (p->pyr_from_l0 == 1)   // levels 1.. as ComputePyramid resizes them, each from the previous
        for (int l = 1; l < cam->n_levels; ++l)
            resize_linear_u8(pyr_r + cam->lvl_offset[l - 1], cam->lvl_cols[l - 1], cam->lvl_rows[l - 1],
                             pyr_r + cam->lvl_offset[l], cam->lvl_cols[l], cam->lvl_rows[l]);
    auto distractor_kp = [&](Rng& rr) {
        gfpl_keypoint a;
        a.x = (float)rr.uni(m, cam->width - 1 - m);
        a.y = (float)rr.uni(m, cam->height - 1 - m);
        a.octave = (int)(rr.next() % (uint64_t)cam->n_levels);
        return a;
    };
    {
        Rng rd(mix(mix(p->seed, 0x3000000ull + (uint64_t)seq), (uint64_t)k));
        while ((int)L.size() < p->n_kp) {
            L.push_back(distractor_kp(rd));
            std::array<uint8_t, 32> d; rand_code(rd, d.data()); DL.push_back(d);
        }
        while ((int)R.size() < p->n_kp) {
            R.push_back(distractor_kp(rd));
            std::array<uint8_t, 32> d; rand_code(rd, d.data()); DR.push_back(d);
        }
    }
    {
        std::vector<int> pl(L.size()), pr(R.size());
        for (size_t i = 0; i < pl.size(); ++i) pl[i] = (int)i;
        for (size_t i = 0; i < pr.size(); ++i) pr[i] = (int)i;
        shuffle(pl, r); shuffle(pr, r);
        for (size_t i = 0; i < pl.size(); ++i) { kp_l[i] = L[pl[i]]; std::memcpy(pdesc_l + 32 * i, DL[pl[i]].data(), 32); }
        for (size_t i = 0; i < pr.size(); ++i) { kp_r[i] = R[pr[i]]; std::memcpy(pdesc_r + 32 * i, DR[pr[i]].data(), 32); }
        *n_kp_l = (int)L.size(); *n_kp_r = (int)R.size();
    }

    if (n_true_out) n_true_out[0] = (int)vis.size();

    // ---- lines
    std::vector<gfpl_keyline> LL, LR;
    std::vector<std::array<uint8_t, 32>> LDL, LDR;
    int n_true_l = (int)std::lround(p->n_kl * (1.0 - p->distractor_frac));
    for (int i = 0; i < (int)W.lines.size() && (int)LL.size() < n_true_l; ++i) {
        const Segment& sg = W.lines[i];
        double Sc[3], Ec[3];
        w2c(T, sg.S, Sc); w2c(T, sg.E, Ec);
        if (Sc[2] < p->z_min || Ec[2] < p->z_min) continue;
        double su = cx + fx * Sc[0] / Sc[2], sv = cy + fy * Sc[1] / Sc[2];
        double eu = cx + fx * Ec[0] / Ec[2], ev = cy + fy * Ec[1] / Ec[2];
        double sd = fx * b / Sc[2], ed = fx * b / Ec[2];
        double mm = 10;
        if (!in_img(su, sv, cam, mm) || !in_img(eu, ev, cam, mm) ||
            !in_img(su - sd, sv, cam, mm) || !in_img(eu - ed, ev, cam, mm)) continue;
        Rng ro(mix(mix(sg.key, (uint64_t)k), 11));
        if (p->outlier_frac > 0.0) {   // outliers: the segment moves by 3-8 px in both images
            Rng rq(mix(mix(sg.key, (uint64_t)k), 17));
            if (rq.uni(0.0, 1.0) < p->outlier_frac) {
                const double ox = rq.uni(3.0, 8.0) * ((rq.next() >> 63) ? -1.0 : 1.0);
                const double oy = rq.uni(3.0, 8.0) * ((rq.next() >> 63) ? -1.0 : 1.0);
                su += ox; eu += ox; sv += oy; ev += oy;
            }
        }
        gfpl_keyline a, c;
        a.sx = (float)(su + p->px_noise * ro.gauss()); a.sy = (float)(sv + p->px_noise * ro.gauss());
        a.ex = (float)(eu + p->px_noise * ro.gauss()); a.ey = (float)(ev + p->px_noise * ro.gauss());
        c.sx = (float)(su - sd + p->px_noise * ro.gauss()); c.sy = (float)(sv + p->px_noise * ro.gauss());
        c.ex = (float)(eu - ed + p->px_noise * ro.gauss()); c.ey = (float)(ev + p->px_noise * ro.gauss());
        a.angle = (float)std::atan2((double)a.ey - a.sy, (double)a.ex - a.sx);
        c.angle = (float)std::atan2((double)c.ey - c.sy, (double)c.ex - c.sx);
        a.octave = 0; c.octave = 0;
        std::array<uint8_t, 32> dl, dr;
        observe_code(ro, sg.code, dl.data());
        observe_code(ro, sg.code, dr.data());
        LL.push_back(a); LR.push_back(c); LDL.push_back(dl); LDR.push_back(dr);
    }
    if (n_true_out) n_true_out[1] = (int)LL.size();
    {
        Rng rd(mix(mix(p->seed, 0x4000000ull + (uint64_t)seq), (uint64_t)k));
        auto distractor_kl = [&](Rng& rr) {
            gfpl_keyline a;
            a.sx = (float)rr.uni(10, cam->width - 11); a.sy = (float)rr.uni(10, cam->height - 11);
            a.ex = (float)rr.uni(10, cam->width - 11); a.ey = (float)rr.uni(10, cam->height - 11);
            a.angle = (float)std::atan2((double)a.ey - a.sy, (double)a.ex - a.sx);
            a.octave = 0;
            return a;
        };
        while ((int)LL.size() < p->n_kl) {
            LL.push_back(distractor_kl(rd));
            std::array<uint8_t, 32> d; rand_code(rd, d.data()); LDL.push_back(d);
        }
        while ((int)LR.size() < p->n_kl) {
            LR.push_back(distractor_kl(rd));
            std::array<uint8_t, 32> d; rand_code(rd, d.data()); LDR.push_back(d);
        }
        std::vector<int> pl(LL.size()), pr(LR.size());
        for (size_t i = 0; i < pl.size(); ++i) pl[i] = (int)i;
        for (size_t i = 0; i < pr.size(); ++i) pr[i] = (int)i;
        shuffle(pl, r); shuffle(pr, r);
        for (size_t i = 0; i < pl.size(); ++i) { kl_l[i] = LL[pl[i]]; std::memcpy(ldesc_l + 32 * i, LDL[pl[i]].data(), 32); }
        for (size_t i = 0; i < pr.size(); ++i) { kl_r[i] = LR[pr[i]]; std::memcpy(ldesc_r + 32 * i, LDR[pr[i]].data(), 32); }
        *n_kl_l = (int)LL.size(); *n_kl_r = (int)LR.size();
    }
    return 0;
}

extern "C" int gfpl_synth_frame(const gfpl_synth_params* p, const gfpl_camera* cam,
                                int seq, int k, int kp_cap, int kl_cap,
                                int* n_kp_l, int* n_kp_r, gfpl_keypoint* kp_l, gfpl_keypoint* kp_r,
                                uint8_t* pdesc_l, uint8_t* pdesc_r,
                                int* n_kl_l, int* n_kl_r, gfpl_keyline* kl_l, gfpl_keyline* kl_r,
                                uint8_t* ldesc_l, uint8_t* ldesc_r,
                                uint8_t* pyr_r, double* time_stamp, double* T_wc_out) {
    return gfpl_synth_frame_ex(p, cam, seq, k, kp_cap, kl_cap, n_kp_l, n_kp_r, kp_l, kp_r, pdesc_l, pdesc_r,
                               n_kl_l, n_kl_r, kl_l, kl_r, ldesc_l, ldesc_r, pyr_r, time_stamp, T_wc_out, nullptr);
}

extern "C" int gfpl_synth_batch(const gfpl_synth_params* p, const gfpl_camera* cam,
                                int s0, int ns, int f0, int nf, int kp_cap, int kl_cap,
                                int* n_kp_l, int* n_kp_r, gfpl_keypoint* kp_l, gfpl_keypoint* kp_r,
                                uint8_t* pdesc_l, uint8_t* pdesc_r,
                                int* n_kl_l, int* n_kl_r, gfpl_keyline* kl_l, gfpl_keyline* kl_r,
                                uint8_t* ldesc_l, uint8_t* ldesc_r,
                                uint8_t* pyr_r, double* time_stamp, int n_threads) {
    int total = ns * nf;
    if (n_threads < 1) n_threads = 1;
    std::vector<int> rc(n_threads, 0);
    auto work = [&](int tid) {
        for (int job = tid; job < total; job += n_threads) {
            int f = job / ns, s = job % ns;
            size_t row = (size_t)f * ns + s;
            int e = gfpl_synth_frame(p, cam, s0 + s, f0 + f, kp_cap, kl_cap,
                                     n_kp_l + row, n_kp_r + row, kp_l + row * kp_cap, kp_r + row * kp_cap,
                                     pdesc_l + row * kp_cap * 32, pdesc_r + row * kp_cap * 32,
                                     n_kl_l + row, n_kl_r + row, kl_l + row * kl_cap, kl_r + row * kl_cap,
                                     ldesc_l + row * kl_cap * 32, ldesc_r + row * kl_cap * 32,
                                     pyr_r + row * cam->pyr_bytes, time_stamp + row, nullptr);
            if (e) rc[tid] = e;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < n_threads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
    for (int e : rc) if (e) return e;
    return 0;
}

// Synthetic grey image for the ORB extraction row: a deterministic
// piecewise-constant scene of overlapping axis-aligned and rotated rectangles and discs
// of random intensity on a smooth gradient, plus mild pixel noise — corners and blobs at
// every scale of a 4-level 1.2 pyramid.  Pure function of (seed, seq_id, frame_idx).
extern "C" int gfpl_synth_image(uint64_t seed, int seq_id, int frame_idx, int width, int height, uint8_t* out) {
    if (!out || width <= 0 || height <= 0) return -1;
    Rng r(mix(seed ^ 0x5A17ull, ((uint64_t)(uint32_t)seq_id << 32) | (uint32_t)frame_idx));
    std::vector<float> img((size_t)width * height);
    const double gx = r.uni(-0.15, 0.15), gy = r.uni(-0.15, 0.15), g0 = r.uni(60, 190);
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) img[(size_t)y * width + x] = (float)(g0 + gx * x + gy * y);
    const int n_shapes = 60 + (int)(r.next() % 40);
    for (int k = 0; k < n_shapes; ++k) {
        const double cx = r.uni(0, width), cy = r.uni(0, height);
        const double sx = r.uni(6, 70), sy = r.uni(6, 70), th = r.uni(0, 3.141592653589793);
        const float val = (float)r.uni(0, 255);
        const bool disc = (r.next() & 3) == 0;
        const double c = std::cos(th), s = std::sin(th);
        const int x0 = std::max(0, (int)(cx - sx - sy - 2)), x1 = std::min(width - 1, (int)(cx + sx + sy + 2));
        const int y0 = std::max(0, (int)(cy - sx - sy - 2)), y1 = std::min(height - 1, (int)(cy + sx + sy + 2));
        for (int y = y0; y <= y1; ++y)
            for (int x = x0; x <= x1; ++x) {
                const double dx = x - cx, dy = y - cy;
                const double u = c * dx + s * dy, v = -s * dx + c * dy;
                const bool in = disc ? (u * u) / (sx * sx) + (v * v) / (sy * sy) <= 1.0 : (std::fabs(u) <= sx && std::fabs(v) <= sy);
                if (in) img[(size_t)y * width + x] = val;
            }
    }
    for (size_t i = 0; i < img.size(); ++i) {
        const double v = img[i] + 2.0 * r.gauss();
        out[i] = (uint8_t)std::min(255.0, std::max(0.0, std::floor(v + 0.5)));
    }
    return 0;
}
