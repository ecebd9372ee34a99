// stvo.h — C++ host mirror of the reference's tracking API (namespace StVO) over
// the MI355X C ABI (include/gfpl.h).
//
// The reference's per-frame path lives behind StVO::StereoFrame and
// StVO::StereoFrameHandler (include/stereoFrame.h:89-260,
// include/stereoFrameHandler.h:38-174 of SimonsRoad/gf-pl-slam).  This header
// keeps the names, public members and call order a caller such as
// app/plslam_mod.cpp:375-477, KeyFrame (src/keyFrame.cpp:26-58) or MapHandler
// relies on, with these deliberate differences:
//  * a StereoFrame is built either from a grey stereo pair, as the reference's
//    StereoFrame(img_l, img_r, idx, cam, ts) (detection then runs on the GPU,
//    gfpl_detector: ORB, LSD, LBD), or from injected keypoints, keylines,
//    descriptors and the right ORB pyramid (the reference's own simulator does the
//    same through public members, src/simulate_line_cut.cpp:62-212);
//  * images are raw 8-bit grey rows of the camera's width x height (cv::Mat
//    CV_8UC1 data); colour conversion is the caller's;
//  * Eigen / OpenCV are not available: Vector*/Matrix* are small row-major value
//    types with the same element access (operator()), KeyPoint/KeyLine carry the
//    fields the path reads;
//  * the handler owns its frames and features (the reference leaks features);
//  * every compute call runs on the GPU through the C ABI; there is no CPU path.
//    After each call the host objects are refreshed from HBM so the public
//    members read exactly like the reference's (matched_pt / matched_ls point into
//    prev_frame->stereo_pt / stereo_ls, mutated in place).
#pragma once
#include <array>
#include <cfloat>
#include <cstdint>
#include <list>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/gfpl.h"

namespace StVO {

// ------------------------------------------------------------ value types --
template <int R, int C>
struct Mat {
    double v[R * C] = {};
    double& operator()(int i, int j) { return v[i * C + j]; }
    double operator()(int i, int j) const { return v[i * C + j]; }
    double& operator()(int i) { return v[i]; }
    double operator()(int i) const { return v[i]; }
    double* data() { return v; }
    const double* data() const { return v; }
    static Mat Identity() {
        Mat m;
        for (int i = 0; i < (R < C ? R : C); ++i) m(i, i) = 1.0;
        return m;
    }
    static Mat Zero() { return Mat(); }
    bool operator==(const Mat& o) const {
        for (int i = 0; i < R * C; ++i)
            if (v[i] != o.v[i]) return false;
        return true;
    }
};
using Vector2d = Mat<2, 1>;
using Vector3d = Mat<3, 1>;
using Vector6d = Mat<6, 1>;
using Matrix3d = Mat<3, 3>;
using Matrix4d = Mat<4, 4>;
using Matrix6d = Mat<6, 6>;
Matrix4d operator*(const Matrix4d& a, const Matrix4d& b);

// cv::KeyPoint / line_descriptor::KeyLine subsets read by the path
struct KeyPoint {
    float x = 0, y = 0;   // pt
    int octave = 0;
};
struct KeyLine {
    float startPointX = 0, startPointY = 0, endPointX = 0, endPointY = 0, angle = 0;
    int octave = 0;
};
using Descriptor = std::array<uint8_t, GFPL_DESC_BYTES>;   // one row of pdesc_* / ldesc_*

// cv::DMatch (the fields the reference's matchers fill and its callers read)
struct DMatch {
    int queryIdx = -1, trainIdx = -1, imgIdx = -1;
    float distance = FLT_MAX;
    DMatch() = default;
    DMatch(int q, int t, float d) : queryIdx(q), trainIdx(t), imgIdx(0), distance(d) {}
    bool operator<(const DMatch& o) const { return distance < o.distance; }
};
// cv::NormTypes the path uses (OpenCV's values)
enum NormTypes { NORM_HAMMING = 6, NORM_HAMMING2 = 7 };

// cv::BFMatcher subset the reference builds (`new BFMatcher(NORM_HAMMING[2], false)`,
// src/stereoFrame.cpp:176,636, src/mapHandler.cpp:213,345,551,679): knnMatch with k = 2
// (gfpl_knn2_hamming_host: i8 MFMA, the OpenCV tie rule) and radiusMatch
// (gfpl_radius_hamming_host), both on the GPU over the matcher's own context and stream.
// Thread-safe: MapHandler runs two matches on one matcher from two std::async tasks.
// Not supported (std::invalid_argument): crossCheck = true, k != 2 (the reference uses
// neither); fewer than 2 train rows throws (GFPL_E_TOO_FEW_TRAIN: the reference then reads
// a missing second neighbour, ledger U4).
class BFMatcher {
public:
    explicit BFMatcher(int normType = NORM_HAMMING, bool crossCheck = false, int device = 0);
    ~BFMatcher();
    BFMatcher(const BFMatcher&) = delete;
    BFMatcher& operator=(const BFMatcher&) = delete;
    void knnMatch(const std::vector<Descriptor>& query, const std::vector<Descriptor>& train,
                  std::vector<std::vector<DMatch>>& matches, int k) const;
    void radiusMatch(const std::vector<Descriptor>& query, const std::vector<Descriptor>& train,
                     std::vector<std::vector<DMatch>>& matches, float maxDistance) const;
    const int normType;
    const bool crossCheck;

private:
    int cell() const { return normType == NORM_HAMMING2 ? 2 : 1; }
    gfpl_ctx* ctx_ = nullptr;
};

// ---------------------------------------------------------------- Config --
// The path's subset of Config (include/config.h:28-141, defaults src/config.cpp:26-154),
// same static accessor names.  Changes take effect at the next handler call.
class Config {
public:
    static Config& getInstance();
    static bool& bestLRMatches() { return getInstance().best_lr_matches; }
    static bool& lrInParallel() { return getInstance().lr_in_parallel; }
    static bool& useLineConfCut() { return getInstance().use_line_conf_cut; }
    static bool& cutWithMaxVol() { return getInstance().max_vol_line_cut; }
    static double& ratioDispSTD() { return getInstance().c.ratio_disp_std; }
    static double& ratioDispSTDHor() { return getInstance().c.ratio_disp_std_hor; }
    static int& maxLineMatchNum() { return getInstance().c.max_line_match_num; }
    static int& maxPointMatchNum() { return getInstance().c.max_point_match_num; }
    static double& maxDistEpip() { return getInstance().c.max_dist_epip; }
    static double& lineMatchRadius() { return getInstance().line_match_radius; }   // src/config.cpp:111
    static double& minDisp() { return getInstance().c.min_disp; }
    static double& maxRatio12P() { return getInstance().c.max_ratio_12_p; }
    static double& pointMatchRadius() { return getInstance().c.point_match_radius; }
    static double& stereoOverlapTh() { return getInstance().c.stereo_overlap_th; }
    static double& lineHorizTh() { return getInstance().c.line_horiz_th; }
    static double& descThL() { return getInstance().c.desc_th_l; }
    static double& lineCovTh() { return getInstance().c.line_cov_th; }
    static double& homogTh() { return getInstance().c.homog_th; }
    static int& minFeatures() { return getInstance().c.min_features; }
    static int& maxIters() { return getInstance().c.max_iters; }
    static int& maxItersRef() { return getInstance().c.max_iters_ref; }
    static double& minError() { return getInstance().c.min_error; }
    static double& minErrorChange() { return getInstance().c.min_error_change; }
    static double& inlierK() { return getInstance().c.inlier_k; }
    static double& motionStepThres() { return getInstance().c.motion_step_th; }
    static double& orbScaleFactor() { return getInstance().c.orb_scale_factor; }
    static int& orbNLevels() { return getInstance().c.orb_n_levels; }
    static double& lsdScale() { return getInstance().c.lsd_scale; }
    // detection (src/config.cpp:107,134,143): used by the image-input calls
    static int& orbNFeatures() { return getInstance().orb_nfeatures; }
    static int& lsdNFeatures() { return getInstance().lsd_nfeatures; }
    static double& minLineLength() { return getInstance().min_line_length; }
    static double& minEntropyRatio() { return getInstance().c.min_entropy_ratio; }
    static int& maxKFNumFrames() { return getInstance().c.max_kf_num_frames; }
    // the C-ABI view (bools folded in)
    static gfpl_config abi();

private:
    Config();
    gfpl_config c{};
    bool best_lr_matches = true, lr_in_parallel = true, use_line_conf_cut = true, max_vol_line_cut = true;
    int orb_nfeatures = 1000, lsd_nfeatures = 300;
    double min_line_length = 0.025;
    double line_match_radius = 80.0;
};

// ---------------------------------------------------- PinholeStereoCamera --
// include/pinholeStereoCamera.h:37-103 (rectified, distortion-free subset).
class StereoFrameHandler;

class PinholeStereoCamera {
public:
    PinholeStereoCamera(int width, int height, double fx, double fy, double cx, double cy, double b);
    // a copy is a new camera: it gets its own frame engine (StereoFrame's frame-level members)
    PinholeStereoCamera(const PinholeStereoCamera& o) : cam_(o.cam_) {}
    PinholeStereoCamera& operator=(const PinholeStereoCamera& o) {
        if (this != &o) { cam_ = o.cam_; engine_.reset(); }
        return *this;
    }
    ~PinholeStereoCamera();
    int getWidth() const { return cam_.width; }
    int getHeight() const { return cam_.height; }
    double getFx() const { return cam_.fx; }
    double getFy() const { return cam_.fy; }
    double getCx() const { return cam_.cx; }
    double getCy() const { return cam_.cy; }
    double getB() const { return cam_.b; }
    // ORB pyramid geometry the right pyramid must follow (levels consecutive)
    int64_t pyramidBytes() const { return cam_.pyr_bytes; }
    const gfpl_camera& abi() const { return cam_; }

private:
    friend class StereoFrame;
    gfpl_camera cam_{};
    // the GPU engine behind StereoFrame's frame-level members on this camera (one sequence),
    // created on first use and destroyed with the camera (not in a static destructor)
    mutable std::unique_ptr<StereoFrameHandler> engine_;
    mutable std::mutex engine_mu_;
};

// -------------------------------------------------------------- features --
// include/stereoFeatures.h:36-124
class PointFeature {
public:
    int idx = -1;
    Vector2d pl, pl_obs;
    double disp = 0;
    Vector3d P;
    bool inlier = true;
    int level = 0;
    double sigma2 = 1.0;
    bool frame_matched = false;
};

class LineFeature {
public:
    int idx = -1;
    Vector2d spl, epl, spl_obs, epl_obs;
    double sdisp = 0, edisp = 0, angle = 0, sdisp_obs = 0, edisp_obs = 0;
    Vector3d sP, eP;
    Vector3d le, le_obs;
    bool inlier = true;
    int level = 0;
    double sigma2 = 1.0;
    bool frame_matched = false;
    Matrix3d covSpt3D, covEpt3D;
    double cutRatio[2] = {0, 0};
    Matrix6d invCovPose;
};

// -------------------------------------------------------------- TimeLog --
// include/stereoFrame.h:66-86: per-frame time costs [s] and counts, written out by the
// app as PREFIX_Log.txt (app/plslam_mod.cpp:494-513).  The handler fills the stage
// times from the device's HIP-event stage marks (gfpl_get_stage_times) and the counts;
// the app fills frame_time_stamp and time_track.  Detection is injected,
// so time_pt_extract / time_ln_detect / time_ln_descri stay 0.
struct TimeLog {
    double frame_time_stamp = 0;
    double time_track = 0;
    double time_pt_extract = 0;
    double time_ln_detect = 0;
    double time_ln_descri = 0;
    double time_pt_stereo = 0;
    double time_ln_stereo = 0;
    double time_pt_cross = 0;
    double time_ln_cross = 0;
    double time_ln_cut = 0;
    double time_pose_optim = 0;
    double num_pt_detect = 0;
    double num_ln_detect = 0;
    double num_pt_stereo = 0;
    double num_ln_stereo = 0;
    double num_pt_cross = 0;
    double num_ln_cross = 0;
};

class StereoFrameHandler;

// ----------------------------------------------------------- StereoFrame --
// include/stereoFrame.h:89-260.  Built from a grey stereo pair (the handler
// detects it on the GPU and fills points_* / lines_* / *desc_* as
// detectFeatures does) or from injected detections; after the handler matched
// it, stereo_pt / stereo_ls and the reordered pdesc_l / ldesc_l hold the stereo
// features exactly as extractStereoFeatures_ORBSLAM leaves them.
class StereoFrame {
public:
    // StereoFrame(img_l, img_r, idx, cam, time_stamp) (src/stereoFrame.cpp:46-60): the two
    // grey images (cam width x height bytes each) are copied; detection runs when the
    // handler takes the frame
    StereoFrame(const uint8_t* img_l_, const uint8_t* img_r_, const int& idx_, PinholeStereoCamera* cam_,
                const double& time_stamp_);
    StereoFrame(const int& idx_, PinholeStereoCamera* cam_, const double& time_stamp_,
                std::vector<KeyPoint> points_l_, std::vector<KeyPoint> points_r_,
                std::vector<Descriptor> pdesc_l_, std::vector<Descriptor> pdesc_r_,
                std::vector<KeyLine> lines_l_, std::vector<KeyLine> lines_r_,
                std::vector<Descriptor> ldesc_l_, std::vector<Descriptor> ldesc_r_,
                std::vector<uint8_t> pyramid_r_);
    ~StereoFrame();
    StereoFrame(const StereoFrame&) = delete;
    StereoFrame& operator=(const StereoFrame&) = delete;

    double time_stamp;
    int frame_idx;
    Matrix4d Tfw = Matrix4d::Identity();
    Matrix4d DT = Matrix4d::Identity();
    Matrix6d Tfw_cov = Matrix6d::Identity();
    Vector6d Tfw_cov_eig;
    Matrix6d DT_cov;
    Vector6d DT_cov_eig;
    double err_norm = 0;
    TimeLog log_;

    std::vector<PointFeature*> stereo_pt;
    std::vector<LineFeature*> stereo_ls;

    std::vector<KeyPoint> points_l, points_r;
    std::vector<KeyLine> lines_l, lines_r;
    std::vector<Descriptor> pdesc_l, pdesc_r, ldesc_l, ldesc_r;
    std::vector<uint8_t> pyramid_r;   // right ORB pyramid, levels packed (cam->pyramidBytes()); empty
                                      // for an image frame (its pyramid stays on the device)
    std::vector<uint8_t> gryImg_l, gryImg_r;   // image frames: the grey pair (else empty)
    bool hasImages() const { return !gryImg_l.empty(); }

    PinholeStereoCamera* cam;

    // Hamming distance of two 32-byte rows (include/stereoFrame.h:185-201)
    static int descriptorDistance(const Descriptor& a, const Descriptor& b);

    // --- the frame-level members the reference's callers use (include/stereoFrame.h:104-148) ---
    // Detection + stereo matching of this frame on the GPU (src/stereoFrame.cpp:148-336 /
    // 411-768): an image frame is detected first (ORB, LSD, LBD); stereo_pt / stereo_ls and the
    // reordered pdesc_l / ldesc_l are filled as the reference leaves them.  The pose members are
    // untouched.  fast_th is accepted and unused, as in the reference (its use is commented out,
    // src/stereoFrame.cpp:1131-1145).  Runs on the camera's frame engine (a one-sequence GPU
    // tracker per PinholeStereoCamera, created on first use, one call at a time).
    void extractInitialStereoFeatures(int fast_th = 20);
    void extractStereoFeatures_ORBSLAM(int fast_th = 20);
    // covSpt3D / covEpt3D of every stereo line (src/stereoFrame.cpp:1448-1484), on the GPU
    void estimateStereoUncertainty();
    // BFMatcher::knnMatch(k = 2) / radiusMatch (Config::pointMatchRadius / lineMatchRadius)
    // wrappers (src/stereoFrame.cpp:1229-1257), as MapHandler calls them through std::async
    void matchPointFeatures(BFMatcher* bfm, const std::vector<Descriptor>& pdesc_1,
                            const std::vector<Descriptor>& pdesc_2, std::vector<std::vector<DMatch>>& pmatches_12);
    void matchLineFeatures(BFMatcher* bfm, const std::vector<Descriptor>& ldesc_1,
                           const std::vector<Descriptor>& ldesc_2, std::vector<std::vector<DMatch>>& lmatches_12);
    void matchPointFeatures_radius(BFMatcher* bfm, const std::vector<Descriptor>& pdesc_1,
                                   const std::vector<Descriptor>& pdesc_2,
                                   std::vector<std::vector<DMatch>>& pmatches_12);
    void matchLineFeatures_radius(BFMatcher* bfm, const std::vector<Descriptor>& ldesc_1,
                                  const std::vector<Descriptor>& ldesc_2,
                                  std::vector<std::vector<DMatch>>& lmatches_12);
    // statistics of a knn-2 list (src/stereoFrame.cpp:1259-1341; gfpl_match_stats_host: ledger U1,
    // U12); every row must hold two matches (GFPL_E_INVALID on an empty list, as the reference
    // reads element size/2 of it)
    void pointDescriptorMAD(const std::vector<std::vector<DMatch>> matches, double& nn_mad, double& nn12_mad);
    void lineDescriptorMAD(const std::vector<std::vector<DMatch>> matches, double& nn_mad, double& nn12_mad);
    void pointDescriptorBudgetThres(const std::vector<std::vector<DMatch>> matches, double& thres_budget);
    void lineDescriptorBudgetThres(const std::vector<std::vector<DMatch>> matches, double& thres_budget);

private:
    StereoFrameHandler& engine();
};

// ---------------------------------------------------- StereoFrameHandler --
// include/stereoFrameHandler.h:38-174; one handler = one sequence.
class StereoFrameHandler {
public:
    explicit StereoFrameHandler(PinholeStereoCamera* cam_, int device = 0, int kp_cap = 8192, int kl_cap = 2048);
    ~StereoFrameHandler();
    StereoFrameHandler(const StereoFrameHandler&) = delete;
    StereoFrameHandler& operator=(const StereoFrameHandler&) = delete;

    // src/stereoFrameHandler.cpp:45-81 (takes ownership of the frame)
    void initialize(StereoFrame* frame);
    // src/stereoFrameHandler.cpp:83-151 (takes ownership of the frame)
    void insertStereoPair(StereoFrame* frame);
    // the reference's image signatures (include/stereoFrameHandler.h:48-53, called at
    // app/plslam_mod.cpp:377,387): a StereoFrame of the grey pair, detected on the GPU
    void initialize(const uint8_t* img_l, const uint8_t* img_r, const int idx, const double time_stamp);
    void insertStereoPair(const uint8_t* img_l, const uint8_t* img_r, const int idx, const double time_stamp);
    // src/stereoFrameHandler.cpp:1939-2030; the app calls optimizePose(prev_frame->DT)
    void optimizePose(Matrix4d DT_ini);
    // src/stereoFrameHandler.cpp:864-922 (prev <- curr; logs T_base * old prev Tfw)
    void updateFrame_ECCV18(const Matrix4d T_base);
    void updateFrame();
    // src/stereoFrameHandler.cpp:2309-2349 / 2351-2379 (app/plslam_mod.cpp:436-447)
    bool needNewKF();
    void currFrameIsKF();

    // stage entry points of insertStereoPair, for callers that drive them one by one
    void stereoMatching(StereoFrame* frame);                     // extractStereoFeatures_ORBSLAM minus detection
    void estimateStereoUncertainty();                             // prev_frame->estimateStereoUncertainty()
    void crossFrameMatching_Hybrid();                             // includes predictFramePose()
    void estimateProjUncertainty_submodular(const double stepCutRatio, const double rngCutRatio[2]);

    // write host-side edits of prev_frame / curr_frame / matched lists back to HBM
    void pushState();

    std::list<PointFeature*> matched_pt;
    std::list<LineFeature*> matched_ls;
    StereoFrame* prev_frame = nullptr;
    StereoFrame* curr_frame = nullptr;
    PinholeStereoCamera* cam;
    int n_inliers = 0, n_inliers_pt = 0, n_inliers_ls = 0;
    int numFrameLoss = 0;
    std::vector<Matrix4d> vec_all_frame_pose;
    // SLAM variables for the KF decision (include/stereoFrameHandler.h:147-153),
    // refreshed from HBM after every call that changes them
    int numFrameSinceKeyframe = 0;
    bool prev_f_iskf = true;
    double entropy_first_prevKF = 0.0;
    Matrix4d T_prevKF = Matrix4d::Identity();
    Matrix6d cov_prevKF_currF;

private:
    friend class StereoFrame;   // frame-level members run on a per-camera handler (the frame engine)
    void frame_stereo(StereoFrame* f, bool initial);
    void frame_uncertainty(StereoFrame* f);
    void frame_stats(int kind, const std::vector<std::vector<DMatch>>& m, int max_num, double* out3);
    void engine_ready();
    void push_frame(int which, StereoFrame* f);
    std::mutex engine_mu_;
    bool engine_init_ = false;
    void sync_config();
    void upload(StereoFrame* f, gfpl_frames* dev);   // detects an image frame, uploads an injected one
    void detect(StereoFrame* f, gfpl_frames* dev);
    void pull_detections(StereoFrame* f, const gfpl_frames& dev);
    void pull(int which, StereoFrame* f, bool features, bool pose);
    void pull_track();
    void pull_kf();
    void check(int rc, const char* what) const;

    gfpl_ctx* ctx_ = nullptr;
    gfpl_seqbatch* sb_ = nullptr;
    gfpl_detector* det_ = nullptr;   // created at the first image frame (and when the detection config changes)
    gfpl_detector_params det_prm_{};
    int kp_cap_, kl_cap_;
    gfpl_config cfg_{};
    struct HostBuf;   // gfpl_frame_host backing store
    HostBuf* buf_ = nullptr;
};

}  // namespace StVO
