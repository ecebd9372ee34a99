// stvo.cpp — StVO host mirror over the C ABI (see stvo.h).  No compute here:
// every method forwards to libgfpl_hip.so and refreshes the host objects.
#include "stvo.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <unordered_map>

namespace StVO {

Matrix4d operator*(const Matrix4d& a, const Matrix4d& b) {
    Matrix4d c;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = a(i, 0) * b(0, j);
            for (int k = 1; k < 4; ++k) s = s + a(i, k) * b(k, j);
            c(i, j) = s;
        }
    return c;
}

// ---------------------------------------------------------------- Config --
Config::Config() { gfpl_config_default(&c); }

Config& Config::getInstance() {
    static Config inst;
    return inst;
}

gfpl_config Config::abi() {
    Config& s = getInstance();
    gfpl_config o = s.c;
    o.best_lr_matches = s.best_lr_matches ? 1 : 0;
    o.lr_in_parallel = s.lr_in_parallel ? 1 : 0;
    o.use_line_conf_cut = s.use_line_conf_cut ? 1 : 0;
    o.cut_with_max_vol = s.max_vol_line_cut ? 1 : 0;
    return o;
}

// ---------------------------------------------------- PinholeStereoCamera --
PinholeStereoCamera::PinholeStereoCamera(int width, int height, double fx, double fy, double cx, double cy,
                                         double b) {
    const gfpl_config cfg = Config::abi();
    const int rc = gfpl_camera_init(&cam_, width, height, fx, fy, cx, cy, b, &cfg);
    if (rc != GFPL_OK) throw std::runtime_error(std::string("gfpl_camera_init: ") + gfpl_strerror(rc));
}

// ----------------------------------------------------------- StereoFrame --
StereoFrame::StereoFrame(const int& idx_, PinholeStereoCamera* cam_, const double& time_stamp_,
                         std::vector<KeyPoint> points_l_, std::vector<KeyPoint> points_r_,
                         std::vector<Descriptor> pdesc_l_, std::vector<Descriptor> pdesc_r_,
                         std::vector<KeyLine> lines_l_, std::vector<KeyLine> lines_r_,
                         std::vector<Descriptor> ldesc_l_, std::vector<Descriptor> ldesc_r_,
                         std::vector<uint8_t> pyramid_r_)
    : time_stamp(time_stamp_), frame_idx(idx_),
      points_l(std::move(points_l_)), points_r(std::move(points_r_)),
      lines_l(std::move(lines_l_)), lines_r(std::move(lines_r_)),
      pdesc_l(std::move(pdesc_l_)), pdesc_r(std::move(pdesc_r_)),
      ldesc_l(std::move(ldesc_l_)), ldesc_r(std::move(ldesc_r_)),
      pyramid_r(std::move(pyramid_r_)), cam(cam_) {
    if (pdesc_l.size() != points_l.size() || pdesc_r.size() != points_r.size() ||
        ldesc_l.size() != lines_l.size() || ldesc_r.size() != lines_r.size())
        throw std::invalid_argument("StereoFrame: one descriptor row per keypoint / keyline");
    if ((int64_t)pyramid_r.size() > cam->pyramidBytes())
        throw std::invalid_argument("StereoFrame: right pyramid larger than the camera's packed pyramid");
    pyramid_r.resize((size_t)cam->pyramidBytes(), 0);
}

StereoFrame::StereoFrame(const uint8_t* img_l_, const uint8_t* img_r_, const int& idx_, PinholeStereoCamera* cam_,
                         const double& time_stamp_)
    : time_stamp(time_stamp_), frame_idx(idx_), cam(cam_) {
    if (!img_l_ || !img_r_) throw std::invalid_argument("StereoFrame: null image");
    const size_t n = (size_t)cam->getWidth() * cam->getHeight();
    gryImg_l.assign(img_l_, img_l_ + n);
    gryImg_r.assign(img_r_, img_r_ + n);
}

StereoFrame::~StereoFrame() {
    for (auto* p : stereo_pt) delete p;
    for (auto* l : stereo_ls) delete l;
}

int StereoFrame::descriptorDistance(const Descriptor& a, const Descriptor& b) {
    int d = 0;
    for (int i = 0; i < GFPL_DESC_BYTES; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

// ------------------------------------------------------------ BFMatcher --
namespace {
void abi_check(int rc, const char* what) {
    if (rc != GFPL_OK) throw std::runtime_error(std::string(what) + ": " + gfpl_strerror(rc));
}
std::vector<uint8_t> pack_rows(const std::vector<Descriptor>& d) {
    std::vector<uint8_t> o(32 * d.size());
    for (size_t i = 0; i < d.size(); ++i) std::memcpy(&o[32 * i], d[i].data(), 32);
    return o;
}
}  // namespace

BFMatcher::BFMatcher(int normType_, bool crossCheck_, int device) : normType(normType_), crossCheck(crossCheck_) {
    if (normType != NORM_HAMMING && normType != NORM_HAMMING2)
        throw std::invalid_argument("BFMatcher: NORM_HAMMING / NORM_HAMMING2 only (binary descriptors)");
    if (crossCheck) throw std::invalid_argument("BFMatcher: crossCheck = true is not supported (the reference never sets it)");
    abi_check(gfpl_create_async(device, &ctx_), "gfpl_create_async");
}

BFMatcher::~BFMatcher() {
    if (ctx_) gfpl_destroy(ctx_);
}

void BFMatcher::knnMatch(const std::vector<Descriptor>& query, const std::vector<Descriptor>& train,
                         std::vector<std::vector<DMatch>>& matches, int k) const {
    if (k != 2) throw std::invalid_argument("BFMatcher::knnMatch: k = 2 only (every call site of the reference)");
    const int nq = (int)query.size(), nt = (int)train.size();
    matches.assign(nq, std::vector<DMatch>());
    if (nq == 0) return;
    const std::vector<uint8_t> q = pack_rows(query), t = pack_rows(train);
    std::vector<int32_t> idx(2 * (size_t)nq);
    std::vector<float> dist(2 * (size_t)nq);
    abi_check(gfpl_knn2_hamming_host(ctx_, q.data(), nq, t.data(), nt, cell(), idx.data(), dist.data()),
              "gfpl_knn2_hamming_host");
    for (int i = 0; i < nq; ++i) {
        matches[i].push_back(DMatch(i, idx[2 * i], dist[2 * i]));
        matches[i].push_back(DMatch(i, idx[2 * i + 1], dist[2 * i + 1]));
    }
}

void BFMatcher::radiusMatch(const std::vector<Descriptor>& query, const std::vector<Descriptor>& train,
                            std::vector<std::vector<DMatch>>& matches, float maxDistance) const {
    const int nq = (int)query.size(), nt = (int)train.size();
    matches.assign(nq, std::vector<DMatch>());
    if (nq == 0) return;
    const std::vector<uint8_t> q = pack_rows(query), t = pack_rows(train);
    std::vector<int32_t> off(nq + 1);
    // sizes first (ragged rows), then the rows
    int rc = gfpl_radius_hamming_host(ctx_, q.data(), nq, t.data(), nt, cell(), maxDistance, off.data(), 0, nullptr,
                                      nullptr);
    if (rc == GFPL_OK) return;   // no match at all
    if (rc != GFPL_E_CAPACITY) abi_check(rc, "gfpl_radius_hamming_host");
    std::vector<int32_t> idx(off[nq]);
    std::vector<float> dist(off[nq]);
    abi_check(gfpl_radius_hamming_host(ctx_, q.data(), nq, t.data(), nt, cell(), maxDistance, off.data(), off[nq],
                                       idx.data(), dist.data()),
              "gfpl_radius_hamming_host");
    for (int i = 0; i < nq; ++i)
        for (int k = off[i]; k < off[i + 1]; ++k) matches[i].push_back(DMatch(i, idx[k], dist[k]));
}

// ---------------------------------------------- StereoFrame frame members --
PinholeStereoCamera::~PinholeStereoCamera() = default;   // (StereoFrameHandler complete here)

StereoFrameHandler& StereoFrame::engine() {
    std::lock_guard<std::mutex> lk(cam->engine_mu_);
    if (!cam->engine_) cam->engine_.reset(new StereoFrameHandler(cam));
    return *cam->engine_;
}

void StereoFrame::extractInitialStereoFeatures(int /*fast_th*/) { engine().frame_stereo(this, true); }
void StereoFrame::extractStereoFeatures_ORBSLAM(int /*fast_th*/) { engine().frame_stereo(this, false); }
void StereoFrame::estimateStereoUncertainty() { engine().frame_uncertainty(this); }

void StereoFrame::matchPointFeatures(BFMatcher* bfm, const std::vector<Descriptor>& pdesc_1,
                                     const std::vector<Descriptor>& pdesc_2,
                                     std::vector<std::vector<DMatch>>& pmatches_12) {
    bfm->knnMatch(pdesc_1, pdesc_2, pmatches_12, 2);
}
void StereoFrame::matchLineFeatures(BFMatcher* bfm, const std::vector<Descriptor>& ldesc_1,
                                    const std::vector<Descriptor>& ldesc_2,
                                    std::vector<std::vector<DMatch>>& lmatches_12) {
    bfm->knnMatch(ldesc_1, ldesc_2, lmatches_12, 2);
}
void StereoFrame::matchPointFeatures_radius(BFMatcher* bfm, const std::vector<Descriptor>& pdesc_1,
                                            const std::vector<Descriptor>& pdesc_2,
                                            std::vector<std::vector<DMatch>>& pmatches_12) {
    bfm->radiusMatch(pdesc_1, pdesc_2, pmatches_12, (float)Config::pointMatchRadius());
}
void StereoFrame::matchLineFeatures_radius(BFMatcher* bfm, const std::vector<Descriptor>& ldesc_1,
                                           const std::vector<Descriptor>& ldesc_2,
                                           std::vector<std::vector<DMatch>>& lmatches_12) {
    bfm->radiusMatch(ldesc_1, ldesc_2, lmatches_12, (float)Config::lineMatchRadius());
}
void StereoFrame::pointDescriptorMAD(const std::vector<std::vector<DMatch>> matches, double& nn_mad, double& nn12_mad) {
    double o[3];
    engine().frame_stats(0, matches, 1, o);
    nn_mad = o[0];
    nn12_mad = o[1];
}
void StereoFrame::lineDescriptorMAD(const std::vector<std::vector<DMatch>> matches, double& nn_mad, double& nn12_mad) {
    double o[3];
    engine().frame_stats(1, matches, 1, o);
    nn_mad = o[0];
    nn12_mad = o[1];
}
void StereoFrame::pointDescriptorBudgetThres(const std::vector<std::vector<DMatch>> matches, double& thres_budget) {
    double o[3];
    engine().frame_stats(0, matches, Config::maxPointMatchNum(), o);
    thres_budget = o[2];
}
void StereoFrame::lineDescriptorBudgetThres(const std::vector<std::vector<DMatch>> matches, double& thres_budget) {
    double o[3];
    engine().frame_stats(1, matches, Config::maxLineMatchNum(), o);
    thres_budget = o[2];
}

// ---------------------------------------------------- StereoFrameHandler --
struct StereoFrameHandler::HostBuf {
    std::vector<double> pt_pl, pt_pl_obs, pt_disp, pt_P, pt_sigma2;
    std::vector<int32_t> pt_idx, pt_level;
    std::vector<uint8_t> pt_inlier, pdesc;
    std::vector<double> ls_spl, ls_epl, ls_spl_obs, ls_epl_obs, ls_sdisp, ls_edisp, ls_sdisp_obs, ls_edisp_obs,
        ls_angle, ls_sigma2, ls_sP, ls_eP, ls_le, ls_le_obs, ls_covS, ls_covE, ls_cut, ls_invcov;
    std::vector<int32_t> ls_idx, ls_level;
    std::vector<uint8_t> ls_inlier, ldesc;
    gfpl_frame_host fh{};
    gfpl_track_host tr{};
    // input staging (host side of gfpl_upload_frames)
    std::vector<gfpl_keypoint> kp_l, kp_r;
    std::vector<gfpl_keyline> kl_l, kl_r;
    std::vector<uint8_t> in_pdesc_l, in_pdesc_r, in_ldesc_l, in_ldesc_r;

    HostBuf(int P, int L) {
        auto d = [](std::vector<double>& v, size_t n) { v.assign(n, 0.0); return v.data(); };
        auto i = [](std::vector<int32_t>& v, size_t n) { v.assign(n, 0); return v.data(); };
        auto u = [](std::vector<uint8_t>& v, size_t n) { v.assign(n, 0); return v.data(); };
        fh.pt_pl = d(pt_pl, 2 * P); fh.pt_pl_obs = d(pt_pl_obs, 2 * P); fh.pt_disp = d(pt_disp, P);
        fh.pt_P = d(pt_P, 3 * P); fh.pt_sigma2 = d(pt_sigma2, P); fh.pt_idx = i(pt_idx, P);
        fh.pt_level = i(pt_level, P); fh.pt_inlier = u(pt_inlier, P); fh.pdesc = u(pdesc, 32 * (size_t)P);
        fh.ls_spl = d(ls_spl, 2 * L); fh.ls_epl = d(ls_epl, 2 * L); fh.ls_spl_obs = d(ls_spl_obs, 2 * L);
        fh.ls_epl_obs = d(ls_epl_obs, 2 * L); fh.ls_sdisp = d(ls_sdisp, L); fh.ls_edisp = d(ls_edisp, L);
        fh.ls_sdisp_obs = d(ls_sdisp_obs, L); fh.ls_edisp_obs = d(ls_edisp_obs, L); fh.ls_angle = d(ls_angle, L);
        fh.ls_sigma2 = d(ls_sigma2, L); fh.ls_sP = d(ls_sP, 3 * L); fh.ls_eP = d(ls_eP, 3 * L);
        fh.ls_le = d(ls_le, 3 * L); fh.ls_le_obs = d(ls_le_obs, 3 * L); fh.ls_covS = d(ls_covS, 9 * L);
        fh.ls_covE = d(ls_covE, 9 * L); fh.ls_cut = d(ls_cut, 2 * L); fh.ls_invcov = d(ls_invcov, 36 * L);
        fh.ls_idx = i(ls_idx, L); fh.ls_level = i(ls_level, L); fh.ls_inlier = u(ls_inlier, L);
        fh.ldesc = u(ldesc, 32 * (size_t)L);
        kp_l.resize(P); kp_r.resize(P); kl_l.resize(L); kl_r.resize(L);
        in_pdesc_l.resize(32 * (size_t)P); in_pdesc_r.resize(32 * (size_t)P);
        in_ldesc_l.resize(32 * (size_t)L); in_ldesc_r.resize(32 * (size_t)L);
    }
};

void StereoFrameHandler::check(int rc, const char* what) const {
    if (rc != GFPL_OK) throw std::runtime_error(std::string(what) + ": " + gfpl_strerror(rc));
}

StereoFrameHandler::StereoFrameHandler(PinholeStereoCamera* cam_, int device, int kp_cap, int kl_cap)
    : cam(cam_), kp_cap_(kp_cap), kl_cap_(kl_cap) {
    check(gfpl_create(device, nullptr, &ctx_), "gfpl_create");
    check(gfpl_set_camera(ctx_, &cam->abi()), "gfpl_set_camera");
    check(gfpl_set_timing(ctx_, 1), "gfpl_set_timing");   // stage marks for TimeLog
    // one sequence per handler: size its matched lists for the largest budgets the
    // ABI accepts, so a later Config::maxPointMatchNum() / maxLineMatchNum() change
    // (e.g. the gazebo value 1000, src/config.cpp:89) stays within the seqbatch
    cfg_ = Config::abi();
    gfpl_config widest = cfg_;
    widest.max_point_match_num = GFPL_MAX_MATCHED_PT;
    widest.max_line_match_num = GFPL_MAX_MATCHED_LS;
    check(gfpl_set_config(ctx_, &widest), "gfpl_set_config");
    check(gfpl_seqbatch_create(ctx_, 1, kp_cap_, kl_cap_, &sb_), "gfpl_seqbatch_create");
    check(gfpl_set_config(ctx_, &cfg_), "gfpl_set_config");
    buf_ = new HostBuf(kp_cap_, kl_cap_);
}

StereoFrameHandler::~StereoFrameHandler() {
    delete prev_frame;
    delete curr_frame;
    delete buf_;
    if (det_) gfpl_detector_destroy(det_);
    if (sb_) gfpl_seqbatch_destroy(sb_);
    if (ctx_) gfpl_destroy(ctx_);
}

void StereoFrameHandler::sync_config() {
    gfpl_config c = Config::abi();
    c.cut_step = cfg_.cut_step;
    c.cut_rng[0] = cfg_.cut_rng[0];
    c.cut_rng[1] = cfg_.cut_rng[1];
    if (std::memcmp(&c, &cfg_, sizeof c) != 0) {
        check(gfpl_set_config(ctx_, &c), "gfpl_set_config");
        cfg_ = c;
    }
}

void StereoFrameHandler::detect(StereoFrame* f, gfpl_frames* dev) {
    gfpl_detector_params p;
    const gfpl_config c = Config::abi();
    check(gfpl_detector_params_default(&cam->abi(), &c, &p), "gfpl_detector_params_default");
    p.orb.nfeatures = Config::orbNFeatures();
    p.lsd.n_features = Config::lsdNFeatures();
    p.lsd.min_length = Config::minLineLength() * std::min(cam->getWidth(), cam->getHeight());
    if (det_ && std::memcmp(&p, &det_prm_, sizeof p) != 0) {
        check(gfpl_detector_destroy(det_), "gfpl_detector_destroy");
        det_ = nullptr;
    }
    if (!det_) {
        check(gfpl_detector_create(ctx_, &p, 1, kp_cap_, kl_cap_, 2, &det_), "gfpl_detector_create");
        det_prm_ = p;
    }
    check(gfpl_detect_stereo(det_, f->gryImg_l.data(), f->gryImg_r.data(), 1, &f->time_stamp, 1, dev),
          "gfpl_detect_stereo");
}

// points_l / points_r / pdesc_* / lines_* / ldesc_* as detectFeatures leaves them
// (src/stereoFrame.cpp:1128-1227), before the stereo matching reorders pdesc_l / ldesc_l
void StereoFrameHandler::pull_detections(StereoFrame* f, const gfpl_frames& dev) {
    HostBuf& h = *buf_;
    gfpl_detections_host d{};
    d.kp_l = h.kp_l.data(); d.kp_r = h.kp_r.data(); d.kl_l = h.kl_l.data(); d.kl_r = h.kl_r.data();
    d.pdesc_l = h.in_pdesc_l.data(); d.pdesc_r = h.in_pdesc_r.data();
    d.ldesc_l = h.in_ldesc_l.data(); d.ldesc_r = h.in_ldesc_r.data();
    check(gfpl_read_detections(ctx_, &dev, 0, &d), "gfpl_read_detections");
    auto kps = [](const std::vector<gfpl_keypoint>& v, int n, std::vector<KeyPoint>& o) {
        o.resize(n);
        for (int i = 0; i < n; ++i) o[i] = {v[i].x, v[i].y, v[i].octave};
    };
    auto kls = [](const std::vector<gfpl_keyline>& v, int n, std::vector<KeyLine>& o) {
        o.resize(n);
        for (int i = 0; i < n; ++i) o[i] = {v[i].sx, v[i].sy, v[i].ex, v[i].ey, v[i].angle, v[i].octave};
    };
    auto rows = [](const std::vector<uint8_t>& v, int n, std::vector<Descriptor>& o) {
        o.resize(n);
        for (int i = 0; i < n; ++i) std::memcpy(o[i].data(), &v[32 * (size_t)i], 32);
    };
    kps(h.kp_l, d.n_kp_l, f->points_l); kps(h.kp_r, d.n_kp_r, f->points_r);
    kls(h.kl_l, d.n_kl_l, f->lines_l); kls(h.kl_r, d.n_kl_r, f->lines_r);
    rows(h.in_pdesc_l, d.n_kp_l, f->pdesc_l); rows(h.in_pdesc_r, d.n_kp_r, f->pdesc_r);
    rows(h.in_ldesc_l, d.n_kl_l, f->ldesc_l); rows(h.in_ldesc_r, d.n_kl_r, f->ldesc_r);
}

void StereoFrameHandler::upload(StereoFrame* f, gfpl_frames* dev) {
    if (f->hasImages()) {
        detect(f, dev);
        pull_detections(f, *dev);   // (the view stays valid: its buffer set is reused two detections later)
        return;
    }
    HostBuf& h = *buf_;
    const int nkl = (int)f->points_l.size(), nkr = (int)f->points_r.size();
    const int nll = (int)f->lines_l.size(), nlr = (int)f->lines_r.size();
    if (nkl > kp_cap_ || nkr > kp_cap_ || nll > kl_cap_ || nlr > kl_cap_)
        throw std::length_error("StereoFrame larger than the handler's capacity");
    for (int i = 0; i < nkl; ++i) h.kp_l[i] = {f->points_l[i].x, f->points_l[i].y, f->points_l[i].octave};
    for (int i = 0; i < nkr; ++i) h.kp_r[i] = {f->points_r[i].x, f->points_r[i].y, f->points_r[i].octave};
    auto kl = [](const KeyLine& k) {
        return gfpl_keyline{k.startPointX, k.startPointY, k.endPointX, k.endPointY, k.angle, k.octave};
    };
    for (int i = 0; i < nll; ++i) h.kl_l[i] = kl(f->lines_l[i]);
    for (int i = 0; i < nlr; ++i) h.kl_r[i] = kl(f->lines_r[i]);
    auto rows = [](const std::vector<Descriptor>& src, std::vector<uint8_t>& dst) {
        for (size_t i = 0; i < src.size(); ++i) std::memcpy(&dst[32 * i], src[i].data(), 32);
    };
    rows(f->pdesc_l, h.in_pdesc_l); rows(f->pdesc_r, h.in_pdesc_r);
    rows(f->ldesc_l, h.in_ldesc_l); rows(f->ldesc_r, h.in_ldesc_r);
    gfpl_frames in{};
    in.batch = 1; in.kp_cap = kp_cap_; in.kl_cap = kl_cap_;
    in.n_kp_l = &nkl; in.n_kp_r = &nkr; in.n_kl_l = &nll; in.n_kl_r = &nlr;
    in.kp_l = h.kp_l.data(); in.kp_r = h.kp_r.data(); in.kl_l = h.kl_l.data(); in.kl_r = h.kl_r.data();
    in.pdesc_l = h.in_pdesc_l.data(); in.pdesc_r = h.in_pdesc_r.data();
    in.ldesc_l = h.in_ldesc_l.data(); in.ldesc_r = h.in_ldesc_r.data();
    in.pyr_r = f->pyramid_r.data();
    in.time_stamp = &f->time_stamp;
    check(gfpl_upload_frames(sb_, &in, dev), "gfpl_upload_frames");
}

void StereoFrameHandler::pull(int which, StereoFrame* f, bool features, bool pose) {
    HostBuf& h = *buf_;
    check(gfpl_read_frame(sb_, which, 0, &h.fh), "gfpl_read_frame");
    const gfpl_frame_host& o = h.fh;
    if (features) {
        // update in place when the count is unchanged (prev_frame: matched lists and
        // KeyFrames alias these objects), otherwise rebuild
        if ((int)f->stereo_pt.size() != o.n_pt) {
            for (auto* p : f->stereo_pt) delete p;
            f->stereo_pt.clear();
            for (int i = 0; i < o.n_pt; ++i) f->stereo_pt.push_back(new PointFeature());
        }
        if ((int)f->stereo_ls.size() != o.n_ls) {
            for (auto* l : f->stereo_ls) delete l;
            f->stereo_ls.clear();
            for (int i = 0; i < o.n_ls; ++i) f->stereo_ls.push_back(new LineFeature());
        }
        f->pdesc_l.resize(o.n_pt);
        f->ldesc_l.resize(o.n_ls);
        for (int i = 0; i < o.n_pt; ++i) {
            PointFeature& p = *f->stereo_pt[i];
            p.idx = o.pt_idx[i];
            for (int k = 0; k < 2; ++k) { p.pl(k) = o.pt_pl[2 * i + k]; p.pl_obs(k) = o.pt_pl_obs[2 * i + k]; }
            p.disp = o.pt_disp[i];
            for (int k = 0; k < 3; ++k) p.P(k) = o.pt_P[3 * i + k];
            p.inlier = o.pt_inlier[i] != 0;
            p.level = o.pt_level[i];
            p.sigma2 = o.pt_sigma2[i];
            std::memcpy(f->pdesc_l[i].data(), o.pdesc + 32 * (size_t)i, 32);
        }
        for (int i = 0; i < o.n_ls; ++i) {
            LineFeature& l = *f->stereo_ls[i];
            l.idx = o.ls_idx[i];
            for (int k = 0; k < 2; ++k) {
                l.spl(k) = o.ls_spl[2 * i + k]; l.epl(k) = o.ls_epl[2 * i + k];
                l.spl_obs(k) = o.ls_spl_obs[2 * i + k]; l.epl_obs(k) = o.ls_epl_obs[2 * i + k];
                l.cutRatio[k] = o.ls_cut[2 * i + k];
            }
            l.sdisp = o.ls_sdisp[i]; l.edisp = o.ls_edisp[i];
            l.sdisp_obs = o.ls_sdisp_obs[i]; l.edisp_obs = o.ls_edisp_obs[i];
            l.angle = o.ls_angle[i];
            for (int k = 0; k < 3; ++k) {
                l.sP(k) = o.ls_sP[3 * i + k]; l.eP(k) = o.ls_eP[3 * i + k];
                l.le(k) = o.ls_le[3 * i + k]; l.le_obs(k) = o.ls_le_obs[3 * i + k];
            }
            for (int k = 0; k < 9; ++k) { l.covSpt3D.v[k] = o.ls_covS[9 * i + k]; l.covEpt3D.v[k] = o.ls_covE[9 * i + k]; }
            for (int k = 0; k < 36; ++k) l.invCovPose.v[k] = o.ls_invcov[36 * i + k];
            l.inlier = o.ls_inlier[i] != 0;
            l.level = o.ls_level[i];
            l.sigma2 = o.ls_sigma2[i];
            std::memcpy(f->ldesc_l[i].data(), o.ldesc + 32 * (size_t)i, 32);
        }
    }
    if (pose) {
        std::memcpy(f->Tfw.v, o.Tfw, sizeof o.Tfw);
        std::memcpy(f->DT.v, o.DT, sizeof o.DT);
        std::memcpy(f->DT_cov.v, o.DT_cov, sizeof o.DT_cov);
        std::memcpy(f->Tfw_cov.v, o.Tfw_cov, sizeof o.Tfw_cov);
        std::memcpy(f->DT_cov_eig.v, o.DT_cov_eig, sizeof o.DT_cov_eig);
        f->err_norm = o.err_norm;
        f->time_stamp = o.time_stamp;
    }
}

void StereoFrameHandler::pull_track() {
    gfpl_track_host& t = buf_->tr;
    check(gfpl_read_track(sb_, 0, &t), "gfpl_read_track");
    matched_pt.clear();
    matched_ls.clear();
    for (int i = 0; i < t.n_matched_pt; ++i) matched_pt.push_back(prev_frame->stereo_pt.at(t.matched_pt[i]));
    for (int i = 0; i < t.n_matched_ls; ++i) matched_ls.push_back(prev_frame->stereo_ls.at(t.matched_ls[i]));
    n_inliers = t.n_inliers;
    n_inliers_pt = t.n_inliers_pt;
    n_inliers_ls = t.n_inliers_ls;
    numFrameLoss = t.num_frame_loss;
}

void StereoFrameHandler::pull_kf() {
    gfpl_kf_state st;
    check(gfpl_read_kf_state(sb_, 0, &st), "gfpl_read_kf_state");
    numFrameSinceKeyframe = st.num_frame_since_kf;
    prev_f_iskf = st.prev_f_iskf != 0;
    entropy_first_prevKF = st.entropy_first_prevKF;
    for (int i = 0; i < 16; ++i) T_prevKF.v[i] = st.T_prevKF[i];
    for (int i = 0; i < 36; ++i) cov_prevKF_currF.v[i] = st.cov_prevKF_currF[i];
}

bool StereoFrameHandler::needNewKF() {
    if (!curr_frame) throw std::logic_error("needNewKF without a current frame");
    sync_config();
    int32_t flag = 0;
    check(gfpl_need_new_kf(sb_, &flag), "gfpl_need_new_kf");
    pull_kf();
    return flag != 0;
}

void StereoFrameHandler::currFrameIsKF() {
    if (!curr_frame) throw std::logic_error("currFrameIsKF without a current frame");
    const int32_t all = 1;
    check(gfpl_curr_frame_is_kf(sb_, &all), "gfpl_curr_frame_is_kf");
    pull(GFPL_CURR, curr_frame, true, true);   // idx renumbered, Tfw = Tfw_cov = I
    pull_kf();
}

void StereoFrameHandler::initialize(StereoFrame* frame) {
    sync_config();
    gfpl_frames dev{};
    upload(frame, &dev);
    check(gfpl_initialize(sb_, &dev), "gfpl_initialize");
    delete prev_frame;
    delete curr_frame;
    curr_frame = nullptr;
    prev_frame = frame;
    matched_pt.clear();
    matched_ls.clear();
    pull(GFPL_PREV, prev_frame, true, true);
    pull_kf();
}

void StereoFrameHandler::insertStereoPair(StereoFrame* frame) {
    if (!prev_frame) throw std::logic_error("insertStereoPair before initialize");
    sync_config();
    gfpl_frames dev{};
    upload(frame, &dev);
    check(gfpl_insert_stereo_pair(sb_, &dev), "gfpl_insert_stereo_pair");
    delete curr_frame;
    curr_frame = frame;
    pull(GFPL_CURR, curr_frame, true, true);
    pull(GFPL_PREV, prev_frame, true, false);   // pl_obs, *_obs, inlier, cut endpoints, covariances
    pull_track();
    numFrameSinceKeyframe++;   // as gfpl_insert_stereo_pair did on the device (:150)
    // counts of TimeLog (src/stereoFrame.cpp:628,765,1147,1187; src/stereoFrameHandler.cpp:601,684)
    TimeLog& lg = curr_frame->log_;
    lg.num_pt_detect = (double)curr_frame->points_l.size();
    lg.num_ln_detect = (double)curr_frame->lines_l.size();
    lg.num_pt_stereo = (double)curr_frame->stereo_pt.size();
    lg.num_ln_stereo = (double)curr_frame->stereo_ls.size();
    lg.num_pt_cross = (double)matched_pt.size();
    lg.num_ln_cross = (double)matched_ls.size();
}

void StereoFrameHandler::initialize(const uint8_t* img_l, const uint8_t* img_r, const int idx, const double time_stamp) {
    initialize(new StereoFrame(img_l, img_r, idx, cam, time_stamp));
}

void StereoFrameHandler::insertStereoPair(const uint8_t* img_l, const uint8_t* img_r, const int idx,
                                          const double time_stamp) {
    insertStereoPair(new StereoFrame(img_l, img_r, idx, cam, time_stamp));
}

void StereoFrameHandler::stereoMatching(StereoFrame* frame) {
    if (!prev_frame) throw std::logic_error("stereoMatching before initialize");
    sync_config();
    gfpl_frames dev{};
    upload(frame, &dev);
    check(gfpl_stereo_points(sb_, &dev), "gfpl_stereo_points");
    check(gfpl_stereo_lines(sb_, &dev), "gfpl_stereo_lines");
    delete curr_frame;
    curr_frame = frame;
    pull(GFPL_CURR, curr_frame, true, true);
}

void StereoFrameHandler::estimateStereoUncertainty() {
    sync_config();
    check(gfpl_line_uncertainty(sb_), "gfpl_line_uncertainty");
    pull(GFPL_PREV, prev_frame, true, false);
}

void StereoFrameHandler::crossFrameMatching_Hybrid() {
    sync_config();
    check(gfpl_cross_points(sb_), "gfpl_cross_points");
    check(gfpl_cross_lines(sb_), "gfpl_cross_lines");
    pull(GFPL_CURR, curr_frame, true, true);   // predicted Tfw, matched idx
    pull(GFPL_PREV, prev_frame, true, false);
    pull_track();
}

void StereoFrameHandler::estimateProjUncertainty_submodular(const double stepCutRatio, const double rngCutRatio[2]) {
    cfg_.cut_step = stepCutRatio;
    cfg_.cut_rng[0] = rngCutRatio[0];
    cfg_.cut_rng[1] = rngCutRatio[1];
    check(gfpl_set_config(ctx_, &cfg_), "gfpl_set_config");
    sync_config();
    check(gfpl_line_cut(sb_), "gfpl_line_cut");
    pull(GFPL_PREV, prev_frame, true, false);
}

void StereoFrameHandler::optimizePose(Matrix4d DT_ini) {
    if (!prev_frame || !curr_frame) throw std::logic_error("optimizePose without a current frame");
    sync_config();
    if (DT_ini == prev_frame->DT)
        check(gfpl_optimize_pose(sb_), "gfpl_optimize_pose");   // the app's call (Q2)
    else
        check(gfpl_optimize_pose_ini(sb_, DT_ini.data()), "gfpl_optimize_pose_ini");
    pull(GFPL_CURR, curr_frame, false, true);
    pull(GFPL_PREV, prev_frame, true, false);   // outlier flags
    pull_track();
    // stage times of the insertStereoPair + optimizePose pair: [stereo points, stereo lines,
    // cross points (with the prev-frame line uncertainty), cross lines, line cut, pose] in ms
    float ms[7];
    if (gfpl_get_stage_times(ctx_, ms) == GFPL_OK) {
        TimeLog& lg = curr_frame->log_;
        lg.time_pt_stereo = ms[0] * 1e-3;
        lg.time_ln_stereo = ms[1] * 1e-3;
        lg.time_pt_cross = ms[2] * 1e-3;
        lg.time_ln_cross = ms[3] * 1e-3;
        lg.time_ln_cut = ms[4] * 1e-3;
        lg.time_pose_optim = ms[5] * 1e-3;
    }
}

void StereoFrameHandler::updateFrame_ECCV18(const Matrix4d T_base) {
    const Matrix4d T_curr_w = T_base * prev_frame->Tfw;
    updateFrame();
    vec_all_frame_pose.push_back(T_curr_w);
}

void StereoFrameHandler::updateFrame() {
    if (!curr_frame) throw std::logic_error("updateFrame without a current frame");
    check(gfpl_update_frame(sb_), "gfpl_update_frame");
    delete prev_frame;
    prev_frame = curr_frame;
    curr_frame = nullptr;
    matched_pt.clear();
    matched_ls.clear();
}

void StereoFrameHandler::push_frame(int which, StereoFrame* f) {
    HostBuf& h = *buf_;
    if (!f) return;
    gfpl_frame_host& o = h.fh;
    o.n_pt = (int)f->stereo_pt.size();
    o.n_ls = (int)f->stereo_ls.size();
    if (o.n_pt > kp_cap_ || o.n_ls > kl_cap_) throw std::length_error("pushState: capacity");
    for (int i = 0; i < o.n_pt; ++i) {
        const PointFeature& p = *f->stereo_pt[i];
        o.pt_idx[i] = p.idx;
        for (int k = 0; k < 2; ++k) { o.pt_pl[2 * i + k] = p.pl(k); o.pt_pl_obs[2 * i + k] = p.pl_obs(k); }
        o.pt_disp[i] = p.disp;
        for (int k = 0; k < 3; ++k) o.pt_P[3 * i + k] = p.P(k);
        o.pt_inlier[i] = p.inlier ? 1 : 0;
        o.pt_level[i] = p.level;
        o.pt_sigma2[i] = p.sigma2;
        std::memcpy(o.pdesc + 32 * (size_t)i, f->pdesc_l.at(i).data(), 32);
    }
    for (int i = 0; i < o.n_ls; ++i) {
        const LineFeature& l = *f->stereo_ls[i];
        o.ls_idx[i] = l.idx;
        for (int k = 0; k < 2; ++k) {
            o.ls_spl[2 * i + k] = l.spl(k); o.ls_epl[2 * i + k] = l.epl(k);
            o.ls_spl_obs[2 * i + k] = l.spl_obs(k); o.ls_epl_obs[2 * i + k] = l.epl_obs(k);
            o.ls_cut[2 * i + k] = l.cutRatio[k];
        }
        o.ls_sdisp[i] = l.sdisp; o.ls_edisp[i] = l.edisp;
        o.ls_sdisp_obs[i] = l.sdisp_obs; o.ls_edisp_obs[i] = l.edisp_obs;
        o.ls_angle[i] = l.angle;
        for (int k = 0; k < 3; ++k) {
            o.ls_sP[3 * i + k] = l.sP(k); o.ls_eP[3 * i + k] = l.eP(k);
            o.ls_le[3 * i + k] = l.le(k); o.ls_le_obs[3 * i + k] = l.le_obs(k);
        }
        for (int k = 0; k < 9; ++k) { o.ls_covS[9 * i + k] = l.covSpt3D.v[k]; o.ls_covE[9 * i + k] = l.covEpt3D.v[k]; }
        for (int k = 0; k < 36; ++k) o.ls_invcov[36 * i + k] = l.invCovPose.v[k];
        o.ls_inlier[i] = l.inlier ? 1 : 0;
        o.ls_level[i] = l.level;
        o.ls_sigma2[i] = l.sigma2;
        std::memcpy(o.ldesc + 32 * (size_t)i, f->ldesc_l.at(i).data(), 32);
    }
    std::memcpy(o.Tfw, f->Tfw.v, sizeof o.Tfw);
    std::memcpy(o.DT, f->DT.v, sizeof o.DT);
    std::memcpy(o.DT_cov, f->DT_cov.v, sizeof o.DT_cov);
    std::memcpy(o.Tfw_cov, f->Tfw_cov.v, sizeof o.Tfw_cov);
    std::memcpy(o.DT_cov_eig, f->DT_cov_eig.v, sizeof o.DT_cov_eig);
    o.err_norm = f->err_norm;
    o.time_stamp = f->time_stamp;
    check(gfpl_write_frame(sb_, which, 0, &o), "gfpl_write_frame");
}

void StereoFrameHandler::pushState() {
    HostBuf& h = *buf_;
    push_frame(GFPL_PREV, prev_frame);
    push_frame(GFPL_CURR, curr_frame);
    if (prev_frame) {
        std::unordered_map<const void*, int> pi, li;
        for (size_t i = 0; i < prev_frame->stereo_pt.size(); ++i) pi[prev_frame->stereo_pt[i]] = (int)i;
        for (size_t i = 0; i < prev_frame->stereo_ls.size(); ++i) li[prev_frame->stereo_ls[i]] = (int)i;
        gfpl_track_host& t = h.tr;
        t.n_matched_pt = 0;
        for (auto* p : matched_pt) t.matched_pt[t.n_matched_pt++] = pi.at(p);
        t.n_matched_ls = 0;
        for (auto* l : matched_ls) t.matched_ls[t.n_matched_ls++] = li.at(l);
        t.n_inliers = n_inliers; t.n_inliers_pt = n_inliers_pt; t.n_inliers_ls = n_inliers_ls;
        t.num_frame_loss = numFrameLoss;
        check(gfpl_write_track(sb_, 0, &t), "gfpl_write_track");
    }
}

// ------------------------------------------------------------ frame engine --
// The frame-level members of StereoFrame run on a per-camera handler that never owns the frame:
// its seqbatch is initialised once with an empty frame, so the stage entry points run
void StereoFrameHandler::engine_ready() {
    if (engine_init_) return;
    StereoFrame empty(0, cam, 0.0, {}, {}, {}, {}, {}, {}, {}, {}, {});
    gfpl_frames dev{};
    upload(&empty, &dev);
    check(gfpl_initialize(sb_, &dev), "gfpl_initialize");
    engine_init_ = true;
}

void StereoFrameHandler::frame_stereo(StereoFrame* f, bool initial) {
    std::lock_guard<std::mutex> lk(engine_mu_);
    sync_config();
    engine_ready();
    gfpl_frames dev{};
    upload(f, &dev);   // (an image frame is detected here: points_* / lines_* / *desc_* filled)
    if (initial) {
        check(gfpl_initialize(sb_, &dev), "gfpl_initialize");   // extractInitialStereoFeatures (the init frame)
        pull(GFPL_PREV, f, true, false);
    } else {
        check(gfpl_stereo_points(sb_, &dev), "gfpl_stereo_points");
        check(gfpl_stereo_lines(sb_, &dev), "gfpl_stereo_lines");
        pull(GFPL_CURR, f, true, false);
    }
}

void StereoFrameHandler::frame_uncertainty(StereoFrame* f) {
    std::lock_guard<std::mutex> lk(engine_mu_);
    sync_config();
    engine_ready();
    push_frame(GFPL_PREV, f);
    check(gfpl_line_uncertainty(sb_), "gfpl_line_uncertainty");   // prev_frame->estimateStereoUncertainty()
    pull(GFPL_PREV, f, true, false);
}

void StereoFrameHandler::frame_stats(int kind, const std::vector<std::vector<DMatch>>& m, int max_num, double* out3) {
    std::vector<float> d0(m.size()), d1(m.size());
    for (size_t i = 0; i < m.size(); ++i) {
        if (m[i].size() < 2) throw std::invalid_argument("descriptor MAD: every knn row needs two matches");
        d0[i] = m[i][0].distance;
        d1[i] = m[i][1].distance;
    }
    std::lock_guard<std::mutex> lk(engine_mu_);
    check(gfpl_match_stats_host(ctx_, kind, d0.data(), d1.data(), (int)m.size(), max_num, out3),
          "gfpl_match_stats_host");
}

}  // namespace StVO
