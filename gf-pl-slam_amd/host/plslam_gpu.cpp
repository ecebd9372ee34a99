// plslam_gpu.cpp — the per-frame loop of app/plslam_mod.cpp:318-515 over the
// StVO host mirror, GPU only: on a directory of rectified grey stereo images
// (--images: detection on the GPU, the reference's insertStereoPair(img_l, img_r,
// idx, ts) signature) or on synthetic stereo detections (gfpl_synth).
//
//   plslam_gpu [--camera vga|euroc|kitti|stress] [--frames N] [--seq S] [--out PREFIX] [--json]
//              [--images DIR] [--orb-features N]
//
// --images DIR reads DIR/left/%06d.pgm and DIR/right/%06d.pgm (binary 8-bit PGM of the
// camera's size; the reference's app reads its dataset through cv::imread) for frames
// 0..N-1 (stopping at the first missing pair) and the time stamps from DIR/times.txt
// (one per line; absent: 0.05 s per frame).
//
// Per frame: initialize (frame 0) or insertStereoPair -> optimizePose(prev_frame->DT)
// -> numFrameLoss check -> needNewKF / currFrameIsKF -> updateFrame_ECCV18(T_base),
// then the lines of the reference's three text outputs, in its formats:
//  PREFIX_AllFrameTrajectory.txt (app/plslam_mod.cpp:288-293, 480-493): fixed,
//      setprecision(7), " tx ty tz qx qy qz qw" of the logged pose, quaternion of R^T;
//  PREFIX_Log.txt (:296-301, 494-513): the just-processed frame's TimeLog, timestamp
//      setprecision(6), times [s] setprecision(7), counts setprecision(0);
//  PREFIX_KeyFrameTrajectory.txt (:538-566), written at the end: "ts tx ty tz qx qy qz qw"
//      of every keyframe's T_kf_w, timestamp setprecision(6), the rest setprecision(7),
//      quaternion of R (not transposed).
// Mapping (local BA, loop closure) is out of scope: the keyframe chain is
// MapHandler::addKeyFrame's composition T_kf_w = prev_kf->T_kf_w * curr_kf->T_kf_w
// (src/mapHandler.cpp:126-127) without the later BA refinements.  --json prints one
// line per frame with the pose bits, for the parity test against the CPU oracle.
#include <cctype>
#include <cmath>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "../synth/gfpl_synth.h"
#include "stvo.h"

using namespace StVO;

// Eigen::Quaterniond(const Matrix3d&) (Eigen/src/Geometry/Quaternion.h, quaternionbase_assign_impl)
// as used by toQuaternion (src/auxiliar.cpp:38-50): x, y, z, w
static std::vector<float> toQuaternion(const Matrix3d& M) {
    double q[4];   // x y z w
    const double t = (M(0, 0) + M(1, 1)) + M(2, 2);
    if (t > 0.0) {
        double s = std::sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (M(2, 1) - M(1, 2)) * s;
        q[1] = (M(0, 2) - M(2, 0)) * s;
        q[2] = (M(1, 0) - M(0, 1)) * s;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(((M(i, i) - M(j, j)) - M(k, k)) + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (M(k, j) - M(j, k)) * s;
        q[j] = (M(j, i) + M(i, j)) * s;
        q[k] = (M(k, i) + M(i, k)) * s;
    }
    return {(float)q[0], (float)q[1], (float)q[2], (float)q[3]};
}

struct CamDef { const char* name; int w, h; double fx, fy, cx, cy, b; };
static const CamDef kCams[] = {
    {"vga", 640, 480, 554.25626, 554.25626, 320.0, 240.0, 0.1},                       // config/gazebo_params.yaml
    {"euroc", 752, 480, 458.654, 457.296, 367.215, 248.375, 0.110077842},             // config/euroc_params.yaml
    {"kitti", 1241, 376, 718.856, 718.856, 607.1928, 185.2157, 0.537165719},          // config/kitti/kitti00-02.yaml
    {"stress", 1920, 1080, 1662.76878, 1662.76878, 960.0, 540.0, 0.1},                // gazebo x3
};

static StereoFrame* make_frame(const gfpl_synth_params& sp, PinholeStereoCamera* cam, int seq, int k, int kp_cap,
                               int kl_cap) {
    int nkl, nkr, nll, nlr;
    double ts;
    std::vector<gfpl_keypoint> kl(kp_cap), kr(kp_cap);
    std::vector<gfpl_keyline> ll(kl_cap), lr(kl_cap);
    std::vector<uint8_t> pdl(32 * (size_t)kp_cap), pdr(32 * (size_t)kp_cap), ldl(32 * (size_t)kl_cap),
        ldr(32 * (size_t)kl_cap), pyr((size_t)cam->pyramidBytes());
    if (gfpl_synth_frame(&sp, &cam->abi(), seq, k, kp_cap, kl_cap, &nkl, &nkr, kl.data(), kr.data(), pdl.data(),
                         pdr.data(), &nll, &nlr, ll.data(), lr.data(), ldl.data(), ldr.data(), pyr.data(), &ts,
                         nullptr) != 0)
        throw std::runtime_error("gfpl_synth_frame failed");
    auto kps = [](const std::vector<gfpl_keypoint>& v, int n) {
        std::vector<KeyPoint> o(n);
        for (int i = 0; i < n; ++i) o[i] = {v[i].x, v[i].y, v[i].octave};
        return o;
    };
    auto kls = [](const std::vector<gfpl_keyline>& v, int n) {
        std::vector<KeyLine> o(n);
        for (int i = 0; i < n; ++i) o[i] = {v[i].sx, v[i].sy, v[i].ex, v[i].ey, v[i].angle, v[i].octave};
        return o;
    };
    auto rows = [](const std::vector<uint8_t>& v, int n) {
        std::vector<Descriptor> o(n);
        for (int i = 0; i < n; ++i) std::memcpy(o[i].data(), &v[32 * (size_t)i], 32);
        return o;
    };
    return new StereoFrame(k, cam, ts, kps(kl, nkl), kps(kr, nkr), rows(pdl, nkl), rows(pdr, nkr), kls(ll, nll),
                           kls(lr, nlr), rows(ldl, nll), rows(ldr, nlr), std::move(pyr));
}

// binary PGM (P5, maxval 255): the pixels, or empty if the file is missing or malformed
static std::vector<uint8_t> read_pgm(const std::string& path, int w, int h) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return {};
    std::string magic;
    int W = 0, H = 0, maxval = 0;
    f >> magic;
    auto skip = [&]() {   // whitespace and comments between header fields
        while (f && (std::isspace(f.peek()) || f.peek() == '#')) {
            if (f.peek() == '#') { std::string line; std::getline(f, line); }
            else f.get();
        }
    };
    skip(); f >> W; skip(); f >> H; skip(); f >> maxval;
    if (magic != "P5" || maxval != 255 || !f) return {};
    f.get();   // the single whitespace before the raster
    if (W != w || H != h) throw std::runtime_error(path + ": image size differs from the camera's");
    std::vector<uint8_t> px((size_t)w * h);
    f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size());
    if (!f) return {};
    return px;
}

static std::string frame_name(const std::string& dir, const char* side, int k) {
    char b[32];
    std::snprintf(b, sizeof b, "%06d.pgm", k);
    return dir + "/" + side + "/" + b;
}

static int run(int argc, char** argv) {
    std::string camname = "vga", out, images;
    int frames = 10, seq = 0, orb_features = 0;
    bool json = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) throw std::invalid_argument("missing value for " + a);
            return argv[++i];
        };
        if (a == "--camera") camname = next();
        else if (a == "--frames") frames = std::stoi(next());
        else if (a == "--seq") seq = std::stoi(next());
        else if (a == "--out") out = next();
        else if (a == "--json") json = true;
        else if (a == "--images") images = next();
        else if (a == "--orb-features") orb_features = std::stoi(next());
        else { std::cerr << "unknown option " << a << "\n"; return 2; }
    }
    const CamDef* cd = nullptr;
    for (const auto& c : kCams)
        if (camname == c.name) cd = &c;
    if (!cd) { std::cerr << "unknown camera " << camname << "\n"; return 2; }
    PinholeStereoCamera cam(cd->w, cd->h, cd->fx, cd->fy, cd->cx, cd->cy, cd->b);
    gfpl_synth_params sp;
    gfpl_synth_default(&sp);
    if (camname == "kitti") { sp.dt = 0.1; sp.v_fwd = 8.0; sp.z_min = 4.0; sp.z_max = 40.0; }
    const int kp_cap = images.empty() ? 2048 : 2320, kl_cap = images.empty() ? 512 : 320;
    if (orb_features > 0) Config::orbNFeatures() = orb_features;
    std::vector<double> times;
    if (!images.empty()) {
        std::ifstream ft(images + "/times.txt");
        for (double t; ft >> t;) times.push_back(t);
    }

    std::ofstream fAllFrameTrack, fLog;
    if (!out.empty()) {
        fAllFrameTrack.open(out + "_AllFrameTrajectory.txt");
        fAllFrameTrack << std::fixed;
        fAllFrameTrack << "#TimeStamp Tx Ty Tz Qx Qy Qz Qw" << std::endl;
        fLog.open(out + "_Log.txt");
        fLog << std::fixed;
        fLog << "#TimeStamp Tx Ty Tz Qx Qy Qz Qw" << std::endl;   // the reference's header, as written
    }
    struct KfRow { double time_stamp; Matrix4d T_kf_w; };
    std::vector<KfRow> keyframes;   // MapHandler::map_keyframes (first KF: frame 0, T_kf_w = I)
    StereoFrameHandler* StVO = new StereoFrameHandler(&cam, 0, kp_cap, kl_cap);
    Matrix4d T_kf_w = Matrix4d::Identity();   // the last keyframe's world pose (first KF: frame 0)
    int n_kf = 1;
    for (int k = 0; k < frames; ++k) {
        StereoFrame* f = nullptr;
        if (images.empty()) {
            f = make_frame(sp, &cam, seq, k, kp_cap, kl_cap);
        } else {
            const std::vector<uint8_t> L = read_pgm(frame_name(images, "left", k), cd->w, cd->h);
            const std::vector<uint8_t> R = read_pgm(frame_name(images, "right", k), cd->w, cd->h);
            if (L.empty() || R.empty()) break;
            const double ts = k < (int)times.size() ? times[k] : 0.05 * k;
            f = new StereoFrame(L.data(), R.data(), k, &cam, ts);   // = insertStereoPair(img_l, img_r, k, ts)
        }
        if (k == 0) {
            StVO->initialize(f);
            keyframes.push_back({StVO->prev_frame->time_stamp, T_kf_w});
            continue;
        }
        const auto t_track = std::chrono::steady_clock::now();
        StVO->insertStereoPair(f);
        const int mpt = (int)StVO->matched_pt.size(), mls = (int)StVO->matched_ls.size();
        StVO->optimizePose(StVO->prev_frame->DT);
        // app/plslam_mod.cpp:388-413 (wall time here: the work runs on the GPU)
        StVO->curr_frame->log_.frame_time_stamp = StVO->curr_frame->time_stamp;
        StVO->curr_frame->log_.time_track =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_track).count();
        if (StVO->numFrameLoss > 10) {   // Config::maxNumFrameLoss() (src/config.cpp)
            std::cerr << "Early termination due to track loss!" << std::endl;
            break;
        }
        const Matrix4d T_base = T_kf_w;   // prev_kf->T_kf_w, read before the KF decision
        bool is_kf = false;
        if (StVO->needNewKF()) {
            is_kf = true;
            T_kf_w = T_kf_w * StVO->curr_frame->Tfw;   // KeyFrame(curr_frame) + addKeyFrame
            StVO->currFrameIsKF();
            keyframes.push_back({StVO->curr_frame->time_stamp, T_kf_w});
            ++n_kf;
        }
        if (json) {
            const StereoFrame* c = StVO->curr_frame;
            std::printf("{\"frame\": %d, \"n_pt\": %zu, \"n_ls\": %zu, \"matched_pt\": %d, \"matched_ls\": %d, "
                        "\"n_inliers\": %d, \"num_frame_loss\": %d, \"err_norm\": %.17g, \"kf\": %d, "
                        "\"time_stamp\": %.17g, \"DT\": [",
                        k, c->stereo_pt.size(), c->stereo_ls.size(), mpt, mls, StVO->n_inliers, StVO->numFrameLoss,
                        c->err_norm, is_kf ? 1 : 0, c->time_stamp);
            for (int i = 0; i < 16; ++i) std::printf("%s%.17g", i ? ", " : "", c->DT.v[i]);
            std::printf("], \"Tfw\": [");
            for (int i = 0; i < 16; ++i) std::printf("%s%.17g", i ? ", " : "", c->Tfw.v[i]);
            std::printf("]}\n");
        }
        StVO->updateFrame_ECCV18(T_base);
        if (!out.empty() && !StVO->vec_all_frame_pose.empty()) {
            const Matrix4d& Tfw = StVO->vec_all_frame_pose.back();
            Matrix3d R;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R(i, j) = Tfw(j, i);   // Tfw.block(0,0,3,3).transpose()
            const std::vector<float> q = toQuaternion(R);
            fAllFrameTrack << std::setprecision(7) << " " << Tfw(0, 3) << " " << Tfw(1, 3) << " " << Tfw(2, 3) << " "
                           << q[0] << " " << q[1] << " " << q[2] << " " << q[3] << std::endl;
        }
        if (!out.empty()) {
            const TimeLog& lg = StVO->prev_frame->log_;   // the frame just processed
            fLog << std::setprecision(6) << lg.frame_time_stamp << " " << std::setprecision(7) << lg.time_track << " "
                 << lg.time_pt_extract << " " << lg.time_ln_detect << " " << lg.time_ln_descri << " " << lg.time_pt_stereo
                 << " " << lg.time_ln_stereo << " " << lg.time_pt_cross << " " << lg.time_ln_cross << " "
                 << lg.time_ln_cut << " " << lg.time_pose_optim << " " << std::setprecision(0) << lg.num_pt_detect << " "
                 << lg.num_ln_detect << " " << lg.num_pt_stereo << " " << lg.num_ln_stereo << " " << lg.num_pt_cross
                 << " " << lg.num_ln_cross << std::endl;
        }
    }
    if (!out.empty()) {
        std::ofstream fKeyFrameTrack(out + "_KeyFrameTrajectory.txt");
        fKeyFrameTrack << std::fixed;
        fKeyFrameTrack << "#TimeStamp Tx Ty Tz Qx Qy Qz Qw" << std::endl;
        for (const KfRow& kf : keyframes) {
            Matrix3d R;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R(i, j) = kf.T_kf_w(i, j);   // T_kf_w.block(0,0,3,3)
            const std::vector<float> q = toQuaternion(R);
            fKeyFrameTrack << std::setprecision(6) << kf.time_stamp << std::setprecision(7) << " " << kf.T_kf_w(0, 3)
                           << " " << kf.T_kf_w(1, 3) << " " << kf.T_kf_w(2, 3) << " " << q[0] << " " << q[1] << " "
                           << q[2] << " " << q[3] << std::endl;
        }
    }
    if (!json) std::cerr << "keyframes: " << n_kf << std::endl;
    delete StVO;
    return 0;
}

int main(int argc, char** argv) {
    try {
        return run(argc, argv);
    } catch (const std::exception& e) {
        std::cerr << "plslam_gpu: " << e.what() << std::endl;
        return 1;
    }
}
