/*
 * gfpl.h — C ABI of the MI355X-native GF-PL-SLAM tracking hot path.
 *
 * The reference has no FFI: its hot path is the C++ member functions of
 * StVO::StereoFrame / StVO::StereoFrameHandler (include/stereoFrame.h:89-260,
 * include/stereoFrameHandler.h:38-174 of SimonsRoad/gf-pl-slam).  Each entry
 * point below names the reference method it replaces; INTEGRATION.md shows the
 * one-line call a maintainer puts into that method body.
 *
 * Conventions
 *  - extern "C", plain pointers and sizes, no C++ / torch types.
 *  - Every function returns int: 0 = GFPL_OK, negative = GFPL_E_*.
 *  - A gfpl_ctx is bound to one HIP device and is not re-entrant; one context
 *    per host thread.  Work is enqueued on the stream passed to gfpl_create
 *    (hipStream_t as void*, NULL = default stream) and is asynchronous unless
 *    the function says it synchronises.
 *  - A gfpl_seqbatch holds B independent stereo sequences (one StereoFrameHandler
 *    each) resident in HBM: prev/curr frame state, matched lists and pose.
 *  - Input frames (gfpl_frames) are DEVICE pointers laid out [B][cap] per
 *    sequence (counts per sequence in n_*).  The right image pyramid is packed
 *    per sequence as consecutive levels of gfpl_camera.lvl_rows x lvl_cols bytes.
 *  - Matrices are row-major double.
 */
#ifndef GFPL_H
#define GFPL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GFPL_ABI_VERSION 6   /* 6: STEP_REC 24 (gfpl_debug_step_records writes B x 24 int64), cut_proof 0-3 */

#define GFPL_DESC_BYTES 32          /* ORB rBRIEF / binarised LBD: 256 bit        */
#define GFPL_MAX_LEVELS 8           /* ORB pyramid levels supported              */
#define GFPL_MAX_IMAGE_DIM 2047     /* pyramid level width / height limit        */
#define GFPL_MAX_MATCHED_PT 2048    /* capacity of matched_pt (cap from config)   */
#define GFPL_MAX_MATCHED_LS 1024    /* capacity of matched_ls (cap from config)   */
#define GFPL_PYR_TAIL 64            /* slack after each packed pyramid (bytes)    */

/* error codes */
#define GFPL_OK                   0
#define GFPL_E_INVALID          (-1)   /* bad argument / NULL pointer            */
#define GFPL_E_HIP              (-2)   /* HIP runtime error                     */
#define GFPL_E_NO_DEVICE        (-3)   /* no HIP device / extension not built   */
#define GFPL_E_TOO_FEW_TRAIN    (-4)   /* knn-2 with < 2 train rows (ref UB, U4) */
#define GFPL_E_CAPACITY         (-5)   /* counts exceed the seqbatch capacity    */
#define GFPL_E_STATE            (-6)   /* call order violated (e.g. insert before initialize) */
#define GFPL_E_UNSUPPORTED      (-7)   /* config flag combination not on the path */

/* which frame of a sequence */
#define GFPL_PREV 0
#define GFPL_CURR 1

/* Hamming cell size: 1 = cv::NORM_HAMMING, 2 = cv::NORM_HAMMING2 */
#define GFPL_HAMMING  1
#define GFPL_HAMMING2 2

/* ------------------------------------------------------------------------ */
/* Camera: PinholeStereoCamera (include/pinholeStereoCamera.h:37-103) plus the
 * ORB scale tables of ORBextractor (src/ORBextractor.cc:410-431) and the
 * right-pyramid geometry of ORBextractor::ComputePyramid (:1107-1132).     */
typedef struct gfpl_camera {
    int    width, height;
    double fx, fy, cx, cy, b;
    int    n_levels;                          /* Config::orbNLevels            */
    float  scale[GFPL_MAX_LEVELS];            /* mvScaleFactors                */
    float  inv_scale[GFPL_MAX_LEVELS];        /* mvInvScaleFactors             */
    int    lvl_cols[GFPL_MAX_LEVELS];         /* cvRound(W * inv_scale)        */
    int    lvl_rows[GFPL_MAX_LEVELS];         /* cvRound(H * inv_scale)        */
    int64_t lvl_offset[GFPL_MAX_LEVELS];      /* byte offset of level in packed pyramid */
    int64_t pyr_bytes;                        /* bytes of one packed pyramid: sum of the
                                                 levels + >= GFPL_PYR_TAIL, a multiple of 4
                                                 (gfpl_camera_init: of 256)               */
    double sigma2_pt[GFPL_MAX_LEVELS];        /* PointFeature::sigma2 per level (src/stereoFeatures.cpp:41-47) */
    double sigma2_ln[GFPL_MAX_LEVELS];        /* LineFeature::sigma2 per level  (src/stereoFeatures.cpp:96-101) */
} gfpl_camera;

/* Config values used by the path (src/config.cpp:77-153).  Mutable like the
 * reference's Config::xxx() accessors: fill with gfpl_config_default() and
 * override fields before gfpl_set_config.                                  */
typedef struct gfpl_config {
    int    best_lr_matches;      /* :81  true  (only true is implemented)      */
    int    lr_in_parallel;       /* :79  true  (radius branch of cross points) */
    int    use_line_conf_cut;    /* :83  true                                   */
    int    cut_with_max_vol;     /* :86  true  (only true is implemented)      */
    double ratio_disp_std;       /* :84  0.15                                   */
    double ratio_disp_std_hor;   /* :85  0.9                                    */
    int    max_line_match_num;   /* :94  300                                    */
    int    max_point_match_num;  /* :95  500                                    */
    double max_dist_epip;        /* :101 2.0                                    */
    double min_disp;             /* :102 1.0                                    */
    double max_ratio_12_p;       /* :103 0.9                                    */
    double point_match_radius;   /* :104 50.0                                   */
    double stereo_overlap_th;    /* :106 0.5                                    */
    double line_horiz_th;        /* :108 0.1                                    */
    double desc_th_l;            /* :109 0.1                                    */
    double line_cov_th;          /* :110 10.0                                   */
    double homog_th;             /* :121 1e-7                                   */
    int    min_features;         /* :122 10                                     */
    int    max_iters;            /* :124 5                                      */
    int    max_iters_ref;        /* :125 10                                     */
    double min_error;            /* :126 1e-7                                   */
    double min_error_change;     /* :127 1e-7                                   */
    double inlier_k;             /* :128 2.0                                    */
    double motion_step_th;       /* :129 10                                     */
    double orb_scale_factor;     /* :135 1.2                                    */
    int    orb_n_levels;         /* :136 4                                      */
    double lsd_scale;            /* :145 1                                      */
    double cut_step;             /* stepCutRatio 0.05 (src/stereoFrameHandler.cpp:135) */
    double cut_rng[2];           /* rngCutRatio {0,1} (src/stereoFrameHandler.cpp:134)  */
    double proj_gate_px;         /* rng_included 10.0 (src/stereoFrameHandler.cpp:534)  */
    double min_entropy_ratio;    /* :34  0.90  (needNewKF)                      */
    int    max_kf_num_frames;    /* :35  50    (needNewKF)                      */
    double cut_certify;          /* (new) 1e-9: relative margin of the certified line-cut
                                    search; 0 = every neighbour evaluated with
                                    the reference's LLT; nonzero values below 1e-10 are rejected */
    int    cut_proof;            /* (new) what ties a margined line-cut decision to the
                                    reference's own logdet:
                                    0 measured: the comparison operands' measured agreement
                                      with the reference's (not a proof);
                                    1 proven after the fact: the measured search records its
                                      decisions, k_cut_verify proves them with the per-step
                                      agreement bound; a sequence not proven is redone by the
                                      eager-proven search;
                                    2 eager-proven: every step of the search carries the bound;
                                    3 (test hook) as 1, but every sequence is redone eagerly.
                                    A step no bound covers takes the reference's evaluation. */
} gfpl_config;

/* cv::KeyPoint subset used by the path */
typedef struct gfpl_keypoint { float x, y; int octave; } gfpl_keypoint;
/* ORB_SLAM2::ORBextractor parameters (src/ORBextractor.cc:410-470), as the path builds it
 * (src/stereoFrame.cpp:33-36): Config::orbNFeatures, orbScaleFactor, orbNLevels, 20, 7 */
typedef struct gfpl_orb_params {
    int   nfeatures;      /* Config::orbNFeatures (src/config.cpp:134; 2000 in BASELINE cfg 2) */
    float scale_factor;   /* Config::orbScaleFactor 1.2 */
    int   nlevels;        /* Config::orbNLevels 4 */
    int   ini_th_fast;    /* iniThFAST 20 */
    int   min_th_fast;    /* minThFAST 7 */
} gfpl_orb_params;
/* line_descriptor::KeyLine subset (3rdparty/line_descriptor/include/line_descriptor/descriptor_custom.hpp:105-170) */
typedef struct gfpl_keyline { float sx, sy, ex, ey, angle; int octave; } gfpl_keyline;

typedef struct gfpl_event gfpl_event;   /* stream-ordering event (gfpl_event_*) */

/* One batch of input stereo frames (detections already done — detection is out
 * of scope).  All pointers are DEVICE pointers.     */
typedef struct gfpl_frames {
    int batch;                         /* B                                   */
    int kp_cap, kl_cap;                /* row capacity per sequence           */
    const int*           n_kp_l;       /* [B]  points_l.size()                */
    const int*           n_kp_r;       /* [B]  points_r.size()                */
    const gfpl_keypoint* kp_l;         /* [B*kp_cap]                          */
    const gfpl_keypoint* kp_r;         /* [B*kp_cap]                          */
    const uint8_t*       pdesc_l;      /* [B*kp_cap*32]                       */
    const uint8_t*       pdesc_r;      /* [B*kp_cap*32]                       */
    const int*           n_kl_l;       /* [B]  lines_l.size()                 */
    const int*           n_kl_r;       /* [B]                                 */
    const gfpl_keyline*  kl_l;         /* [B*kl_cap]                          */
    const gfpl_keyline*  kl_r;         /* [B*kl_cap]                          */
    const uint8_t*       ldesc_l;      /* [B*kl_cap*32]                       */
    const uint8_t*       ldesc_r;      /* [B*kl_cap*32]                       */
    const uint8_t*       pyr_r;        /* [B*cam.pyr_bytes] right ORB pyramid (4-byte aligned) */
    const double*        time_stamp;   /* [B]                                 */
    /* optional stream ordering with a producer on another context (e.g. the detectors):
     * a tracker call that reads these frames makes its stream wait for `ready` first and
     * records `consumed` once its reads are enqueued.  NULL (zero-initialised): none.   */
    gfpl_event*          ready;
    gfpl_event*          consumed;
} gfpl_frames;

/* Host view of one frame's state (StereoFrame public members the path
 * produces, include/stereoFrame.h:205-259; feature records
 * include/stereoFeatures.h:36-124).  Arrays are caller-allocated with the
 * capacity given to the seqbatch (points: kp_cap, lines: kl_cap).  The CPU
 * oracle fills the same struct, so parity tests compare field by field.   */
typedef struct gfpl_frame_host {
    int n_pt, n_ls;
    /* stereo_pt */
    double*  pt_pl;        /* [cap*2]  pl                    */
    double*  pt_pl_obs;    /* [cap*2]  pl_obs                */
    double*  pt_disp;      /* [cap]                          */
    double*  pt_P;         /* [cap*3]                        */
    double*  pt_sigma2;    /* [cap]                          */
    int32_t* pt_idx;       /* [cap]                          */
    int32_t* pt_level;     /* [cap]                          */
    uint8_t* pt_inlier;    /* [cap]                          */
    uint8_t* pdesc;        /* [cap*32]  pdesc_l (reordered)  */
    /* stereo_ls */
    double*  ls_spl;       /* [cap*2] */
    double*  ls_epl;       /* [cap*2] */
    double*  ls_spl_obs;   /* [cap*2] */
    double*  ls_epl_obs;   /* [cap*2] */
    double*  ls_sdisp;     /* [cap]   */
    double*  ls_edisp;     /* [cap]   */
    double*  ls_sdisp_obs; /* [cap]   */
    double*  ls_edisp_obs; /* [cap]   */
    double*  ls_angle;     /* [cap]   */
    double*  ls_sigma2;    /* [cap]   */
    double*  ls_sP;        /* [cap*3] */
    double*  ls_eP;        /* [cap*3] */
    double*  ls_le;        /* [cap*3] */
    double*  ls_le_obs;    /* [cap*3] */
    double*  ls_covS;      /* [cap*9] covSpt3D */
    double*  ls_covE;      /* [cap*9] covEpt3D */
    double*  ls_cut;       /* [cap*2] cutRatio */
    double*  ls_invcov;    /* [cap*36] invCovPose */
    int32_t* ls_idx;       /* [cap] */
    int32_t* ls_level;     /* [cap] */
    uint8_t* ls_inlier;    /* [cap] */
    uint8_t* ldesc;        /* [cap*32] ldesc_l (reordered) */
    /* pose */
    double Tfw[16], DT[16], DT_cov[36], Tfw_cov[36], DT_cov_eig[6];
    double err_norm, time_stamp;
} gfpl_frame_host;

/* StereoFrameHandler tracking results of the last step
 * (include/stereoFrameHandler.h:120-161). matched_* hold indices into
 * prev_frame->stereo_pt / stereo_ls in list order (duplicates allowed for
 * points).                                                */
typedef struct gfpl_track_host {
    int n_matched_pt;
    int n_matched_ls;
    int32_t matched_pt[GFPL_MAX_MATCHED_PT];
    int32_t matched_ls[GFPL_MAX_MATCHED_LS];
    int n_inliers, n_inliers_pt, n_inliers_ls;
    int num_frame_loss;
} gfpl_track_host;

/* Keyframe-decision state of one StereoFrameHandler (include/stereoFrameHandler.h:147-153). */
typedef struct gfpl_kf_state {
    double T_prevKF[16];          /* row-major                                   */
    double cov_prevKF_currF[36];
    double entropy_first_prevKF;
    double entropy_ratio;         /* of the last gfpl_need_new_kf               */
    int    prev_f_iskf;
    int    num_frame_since_kf;    /* numFrameSinceKeyframe                       */
    int    need_new_kf;           /* decision of the last gfpl_need_new_kf       */
} gfpl_kf_state;

typedef struct gfpl_ctx gfpl_ctx;
typedef struct gfpl_seqbatch gfpl_seqbatch;

/* ---------------------------------------------------------------- setup -- */
int  gfpl_abi_version(void);
/* Config::Config() defaults (src/config.cpp:26-154). */
int  gfpl_config_default(gfpl_config* cfg);
/* Fill the derived tables of a camera (scale tables, pyramid geometry,
 * sigma2 tables) from the intrinsics, image size and ORB pyramid params.   */
int  gfpl_camera_init(gfpl_camera* cam, int width, int height, double fx, double fy,
                      double cx, double cy, double b, const gfpl_config* cfg);

/* context: device + stream + camera + config (replaces the Config singleton
 * src/config.cpp:158-162 and the PinholeStereoCamera* each frame holds).   */
int  gfpl_create(int device, void* hip_stream, gfpl_ctx** out);
/* A context on its own non-blocking stream (created here, destroyed with the context):
 * for a caller without a HIP runtime that wants, e.g., detection and tracking on two
 * contexts ordered by gfpl_event_* instead of one serial stream.                      */
int  gfpl_create_async(int device, gfpl_ctx** out);
/* the hipStream_t (as void*) the context enqueues on */
void* gfpl_get_stream(const gfpl_ctx* ctx);

/* Stream-ordering events between contexts (all asynchronous but synchronize):
 * record on a context's stream, make another context's stream wait for it.           */
int  gfpl_event_create(gfpl_ctx* ctx, gfpl_event** out);
int  gfpl_event_destroy(gfpl_event* ev);
int  gfpl_event_record(gfpl_event* ev, gfpl_ctx* ctx);
int  gfpl_event_wait(gfpl_ctx* ctx, gfpl_event* ev);
int  gfpl_event_synchronize(gfpl_event* ev);
/* how often the event was recorded so far (gfpl_event_record, or by a tracker call as a
 * gfpl_frames.consumed event): a producer reusing buffers checks its views were read.  */
int  gfpl_event_record_count(const gfpl_event* ev, int64_t* count);
/* GFPL_E_STATE while seqbatches or ORB / LBD / LSD objects created on the context
 * are still alive (they use its stream; ORB also reads its camera).           */
int  gfpl_destroy(gfpl_ctx* ctx);
/* GFPL_E_STATE while seqbatches or detector objects of the context live (their pyramid
 * builders and ORB / LSD geometry are laid out for the camera they were created on).
 * GFPL_E_INVALID for bad level tables.                                                 */
int  gfpl_set_camera(gfpl_ctx* ctx, const gfpl_camera* cam);
/* max_point_match_num / max_line_match_num size the matched lists and the cut /
 * pose scratch of a seqbatch when it is created; while any seqbatch of the
 * context lives, a config with a larger budget than its capacity is refused with
 * GFPL_E_CAPACITY (lower budgets are accepted).  Other fields (e.g. cut_proof) may
 * change between steps: each step reads the config current at its launch.     */
int  gfpl_set_config(gfpl_ctx* ctx, const gfpl_config* cfg);
int  gfpl_get_camera(const gfpl_ctx* ctx, gfpl_camera* cam);
int  gfpl_get_config(const gfpl_ctx* ctx, gfpl_config* cfg);
int  gfpl_synchronize(gfpl_ctx* ctx);
/* Copy `bytes` of DEVICE memory (e.g. a field of a gfpl_frames view) to HOST memory after the
 * context's stream drained, for FFI callers without a HIP runtime of their own.  Synchronises. */
int  gfpl_copy_to_host(gfpl_ctx* ctx, void* host_dst, const void* device_src, size_t bytes);

/* B independent sequences (B StereoFrameHandler objects) resident in HBM.
 * kp_cap <= 8192 keypoints and kl_cap <= 2048 keylines per side (config 5:
 * 8000 ORB + 2000 LBD); larger values return GFPL_E_INVALID.               */
int  gfpl_seqbatch_create(gfpl_ctx* ctx, int batch, int kp_cap, int kl_cap, gfpl_seqbatch** out);
int  gfpl_seqbatch_destroy(gfpl_seqbatch* sb);
/* bytes of device memory held by the seqbatch (state + workspace) */
int64_t gfpl_seqbatch_bytes(const gfpl_seqbatch* sb);

/* -------------------------------------------------- tracker entry points -- */
/* StereoFrameHandler::initialize (src/stereoFrameHandler.cpp:45-81) with the
 * detections injected: StereoFrame::extractInitialStereoFeatures matching part
 * (src/stereoFrame.cpp:173-336); Tfw = Tfw_cov = DT = I.                      */
int  gfpl_initialize(gfpl_seqbatch* sb, const gfpl_frames* in);
/* StereoFrameHandler::insertStereoPair (src/stereoFrameHandler.cpp:83-151):
 * stereo matching of the new frame, predictFramePose, prev-frame line
 * uncertainty, crossFrameMatching_Hybrid, estimateProjUncertainty_submodular. */
int  gfpl_insert_stereo_pair(gfpl_seqbatch* sb, const gfpl_frames* in);
/* StereoFrameHandler::optimizePose(prev_frame->DT) (src/stereoFrameHandler.cpp:1939-2030,
 * called as at app/plslam_mod.cpp:408).                                       */
int  gfpl_optimize_pose(gfpl_seqbatch* sb);
/* StereoFrameHandler::optimizePose(Matrix4d DT_ini) with an explicit initial guess per
 * sequence: dt_ini = HOST array [B*16] row-major (NULL = prev_frame->DT).  Synchronises. */
int  gfpl_optimize_pose_ini(gfpl_seqbatch* sb, const double* dt_ini);
/* Copy one batch of HOST input frames (host->* are host pointers, same layout)
 * into staging buffer 0 of the seqbatch and return its device view in *dev
 * (valid until the next upload into that buffer).  Synchronous; for FFI callers
 * without a HIP runtime of their own.  The rate through this path includes PCIe. */
int  gfpl_upload_frames(gfpl_seqbatch* sb, const gfpl_frames* host, gfpl_frames* dev);
/* Stream-ordered upload, no host synchronisation: copy the host->batch sequences of
 * a HOST input batch (pinned memory for an asynchronous DMA) into sequences
 * [s0, s0 + host->batch) of staging buffer `slot` (0 or 1; each holds one input
 * frame of all B sequences, allocated on first use) on the seqbatch's own copy
 * stream.  The copy waits for the last tracker call that read the slot, and every
 * tracker call that reads the slot (gfpl_staged_frames view) waits for the copies
 * enqueued before it — so uploading frame k+1 into one slot overlaps the step on
 * frame k in the other.  *ticket (nullable) names the copy for gfpl_upload_wait;
 * the host memory must stay unchanged until then.                              */
int  gfpl_upload_frames_async(gfpl_seqbatch* sb, const gfpl_frames* host, int s0, int slot, int64_t* ticket);
/* The same with only level 0 of each right pyramid on the host: host->pyr_r holds the
 * level-0 images (lvl_cols[0] x lvl_rows[0] bytes) of the host->batch sequences, l0_stride
 * bytes apart; after the copy the device builds levels 1.. of the staged pyramids as
 * ORBextractor::ComputePyramid does (cv::resize INTER_LINEAR of the level above,
 * src/ORBextractor.cc:1107-1132; the ORB extractor's k_orb_resize), on the copy stream —
 * about half the bytes over PCIe at VGA.                                                   */
int  gfpl_upload_frames_l0_async(gfpl_seqbatch* sb, const gfpl_frames* host, int s0, int slot,
                                 int64_t l0_stride, int64_t* ticket);
/* Block the host until the copy `ticket` (and every copy enqueued before it) is done. */
int  gfpl_upload_wait(gfpl_seqbatch* sb, int64_t ticket);
/* Device view (all B sequences) of staging buffer `slot` (GFPL_E_INVALID before its first upload). */
int  gfpl_staged_frames(gfpl_seqbatch* sb, int slot, gfpl_frames* dev);
/* StereoFrameHandler::updateFrame_ECCV18 state swap (src/stereoFrameHandler.cpp:864-922):
 * prev <- curr, matched lists cleared.  (FAST-threshold adaptation is out of scope;
 * the T_base trajectory log lives in the host mirror, gf-pl-slam_amd/host/stvo.h.) */
int  gfpl_update_frame(gfpl_seqbatch* sb);
/* StereoFrameHandler::needNewKF (src/stereoFrameHandler.cpp:2309-2349) for every
 * sequence on its curr frame (after optimize_pose, as app/plslam_mod.cpp:436):
 * entropy of the covariance accumulated since the last keyframe vs the first one.
 * flags: HOST [B] (synchronises) or NULL; 1 = new keyframe needed.  The decision
 * and the ratio are kept in the sequence's gfpl_kf_state either way.          */
int  gfpl_need_new_kf(gfpl_seqbatch* sb, int32_t* flags);
/* StereoFrameHandler::currFrameIsKF (src/stereoFrameHandler.cpp:2351-2379) for the
 * sequences whose mask entry is nonzero (HOST [B], synchronises; NULL = the last
 * gfpl_need_new_kf decisions, asynchronous): numFrameSinceKeyframe = 0, curr idx
 * renumbered, curr Tfw = Tfw_cov = I, T_prevKF = I, cov_prevKF_currF = 0.     */
int  gfpl_curr_frame_is_kf(gfpl_seqbatch* sb, const int32_t* mask);
int  gfpl_read_kf_state(gfpl_seqbatch* sb, int seq, gfpl_kf_state* out);
/* insert_stereo_pair + optimize_pose + update_frame, one batched step.       */
int  gfpl_frame_step(gfpl_seqbatch* sb, const gfpl_frames* in);

/* ------------------------------------------------------- stage entry points */
/* StereoFrame::extractStereoFeatures_ORBSLAM point branch (src/stereoFrame.cpp:453-630)
 * incl. subPixelStereoRefine_ORBSLAM (:340-404) -> curr stereo_pt, pdesc_l.   */
int  gfpl_stereo_points(gfpl_seqbatch* sb, const gfpl_frames* in);
/* ... line branch (src/stereoFrame.cpp:633-767) -> curr stereo_ls, ldesc_l,
 * plus the covariances estimateStereoUncertainty (:1448-1484) will need.      */
int  gfpl_stereo_lines(gfpl_seqbatch* sb, const gfpl_frames* in);
/* StereoFrame::estimateStereoUncertainty on the PREV frame (src/stereoFrame.cpp:1448-1484). */
int  gfpl_line_uncertainty(gfpl_seqbatch* sb);
/* predictFramePose + crossFrameMatching_Hybrid points (src/stereoFrameHandler.cpp:153-157,451-603) */
int  gfpl_cross_points(gfpl_seqbatch* sb);
/* crossFrameMatching_Hybrid lines (src/stereoFrameHandler.cpp:605-695)       */
int  gfpl_cross_lines(gfpl_seqbatch* sb);
/* estimateProjUncertainty_submodular(0.05,{0,1}) (src/stereoFrameHandler.cpp:1618-1764) */
int  gfpl_line_cut(gfpl_seqbatch* sb);

/* cv::BFMatcher::knnMatch(k=2) with NORM_HAMMING / NORM_HAMMING2 on device
 * buffers (call sites src/stereoFrame.cpp:183-197,256-272,636-656;
 * src/stereoFrameHandler.cpp:617-633).  q: nq x 32 B, t: nt x 32 B (device).
 * out_idx[2*nq], out_dist[2*nq] (device; distance as float like cv::DMatch).
 * Returns GFPL_E_TOO_FEW_TRAIN when nt < 2 (reference UB).        */
int  gfpl_knn2_hamming(gfpl_ctx* ctx, const uint8_t* q, int nq, const uint8_t* t, int nt,
                       int cell, int32_t* out_idx, float* out_dist);
/* The same on HOST buffers (copied in and out; synchronous): StereoFrame::matchPointFeatures /
 * matchLineFeatures (src/stereoFrame.cpp:1229-1241), which MapHandler calls from two std::async
 * tasks (src/mapHandler.cpp:223-226,355-356,558-559,686-687).  Thread-safe per context.      */
int  gfpl_knn2_hamming_host(gfpl_ctx* ctx, const uint8_t* q, int nq, const uint8_t* t, int nt,
                            int cell, int32_t* out_idx, float* out_dist);
/* cv::BFMatcher::radiusMatch with NORM_HAMMING (cell 1) / NORM_HAMMING2 (cell 2):
 * StereoFrame::matchPointFeatures_radius / matchLineFeatures_radius (src/stereoFrame.cpp:
 * 1243-1257).  Row i holds every train row j with distance <= max_dist (ledger T1), sorted by
 * distance, equal distances in train order (T2); rows are ragged: row i is
 * [row_off[i], row_off[i+1]) of out_idx / out_dist (row_off has nq + 1 entries, always
 * filled).  When row_off[nq] > cap nothing else is written and GFPL_E_CAPACITY is returned
 * (call again with cap >= row_off[nq]).  _host: HOST buffers, synchronous; the device form
 * takes DEVICE q / t / row_off / out_* and returns after the rows are written.              */
int  gfpl_radius_hamming(gfpl_ctx* ctx, const uint8_t* q, int nq, const uint8_t* t, int nt, int cell,
                         float max_dist, int32_t* row_off, int cap, int32_t* out_idx, float* out_dist);
int  gfpl_radius_hamming_host(gfpl_ctx* ctx, const uint8_t* q, int nq, const uint8_t* t, int nt, int cell,
                              float max_dist, int32_t* row_off, int cap, int32_t* out_idx, float* out_dist);
/* Statistics of a knn-2 match list, HOST d0[n] / d1[n] = the best / second distances of each
 * row (vector<vector<DMatch>> rows [0] / [1]): kind 0 pointDescriptorMAD + pointDescriptor-
 * BudgetThres, kind 1 lineDescriptorMAD + lineDescriptorBudgetThres (src/stereoFrame.cpp:
 * 1259-1341).  out[0] nn_mad, out[1] nn12_mad, out[2] thres_budget for max_num (the
 * Config::max*MatchNum the reference reads).  nn_dist_median is the reference's
 * uninitialised value pinned to 0.0 (ledger U1); NaN ratios order above +inf (U12).
 * GFPL_E_INVALID for n < 1 or max_num < 1 (the reference indexes element -1).  Synchronous.   */
int  gfpl_match_stats_host(gfpl_ctx* ctx, int kind, const float* d0, const float* d1, int n, int max_num,
                           double* out);

/* --------------------------------------------- ORB extraction (§8(f)1) ---- */
/* ORB_SLAM2::ORBextractor (src/ORBextractor.cc:410-470 constructor, :1043-1105
 * operator()) as StereoFrame builds it (src/stereoFrame.cpp:33-36), over a batch of
 * grey images on the device.  The extractor owns its workspace for images of
 * width x height (64..2047 px) and up to max_images per call; kp_cap bounds the
 * keypoints returned per image.  Arithmetic of the OpenCV calls pinned as the CPU
 * oracle's ledger O1-O7.                                          */
typedef struct gfpl_orb gfpl_orb;
int  gfpl_orb_create(gfpl_ctx* ctx, int width, int height, const gfpl_orb_params* prm,
                     int max_images, int kp_cap, gfpl_orb** out);
int  gfpl_orb_destroy(gfpl_orb* orb);
/* bytes of one image's packed level images (the gfpl_frames.pyr_r layout) */
int  gfpl_orb_pyramid_bytes(const gfpl_orb* orb, int64_t* bytes);
/* operator()(image, noArray(), keypoints, descriptors) for n images, all pointers
 * DEVICE: images [n][height][width] u8; per image i, rows [i*kp_cap, +n_kp[i]) of
 * kps / desc (32 B) / angle (degrees) / response (FAST score) hold the keypoints
 * in the reference's order (level by level, DistributeOctTree node order),
 * coordinates scaled to level 0.  angle, response, pyramid may be NULL; pyramid
 * receives each image's level images at pyr_stride bytes apart.  When the context has
 * a camera of this image size and pyr_stride is its pyr_bytes (the tracker's
 * gfpl_frames.pyr_r), the extractor's level geometry must be the camera's
 * (GFPL_E_INVALID otherwise).  Synchronises; GFPL_E_CAPACITY when an internal or
 * kp_cap capacity was exceeded.                                                */
int  gfpl_orb_extract(gfpl_orb* orb, const uint8_t* images, int n, gfpl_keypoint* kps,
                      uint8_t* desc, int* n_kp, float* angle, float* response,
                      uint8_t* pyramid, int64_t pyr_stride);
/* The same, stream-ordered: returns after enqueueing on the context's stream (argument
 * errors are still returned at once); the capacity status of every async call since the
 * last status is returned by gfpl_orb_status (which waits for the last of them).      */
int  gfpl_orb_extract_async(gfpl_orb* orb, const uint8_t* images, int n, gfpl_keypoint* kps,
                            uint8_t* desc, int* n_kp, float* angle, float* response,
                            uint8_t* pyramid, int64_t pyr_stride);
int  gfpl_orb_status(gfpl_orb* orb);

/* ---------------------------------------- LBD descriptors (§8(f)2 part) ---- */
/* line_descriptor::BinaryDescriptor::compute(image, keylines, descriptors)
 * (3rdparty/line_descriptor/src/binary_descriptor_custom.cpp:539-687, computeLBD :1026-1372)
 * as StereoFrame::detectLineFeatures calls it (src/stereoFrame.cpp:1194,1220): keylines of
 * octave 0 (Config::lsdOctaveNum = 1; another octave returns GFPL_E_UNSUPPORTED), images of
 * width x height (8..8192 px), up to max_images per call, kl_cap keylines per image.
 * Arithmetic pinned as the CPU oracle's ledger L1-L5.                        */
typedef struct gfpl_lbd gfpl_lbd;
int  gfpl_lbd_create(gfpl_ctx* ctx, int width, int height, int max_images, int kl_cap, gfpl_lbd** out);
int  gfpl_lbd_destroy(gfpl_lbd* lbd);
/* all pointers DEVICE: images [n][height][width] u8, keylines [n][kl_cap] (sx sy ex ey angle
 * octave, LSDDetectorC's fields), n_kl [n]; desc [n][kl_cap][32] receives row i of image j's
 * 32-byte LBD for keyline i < n_kl[j].  Synchronises; GFPL_E_CAPACITY when some n_kl[j] >
 * kl_cap (the first kl_cap are described), GFPL_E_UNSUPPORTED for a keyline of octave != 0. */
int  gfpl_lbd_compute(gfpl_lbd* lbd, const uint8_t* images, int n, const gfpl_keyline* keylines,
                      const int* n_kl, uint8_t* desc);
/* stream-ordered form; gfpl_lbd_status reports (and waits for) the async calls since the last */
int  gfpl_lbd_compute_async(gfpl_lbd* lbd, const uint8_t* images, int n, const gfpl_keyline* keylines,
                            const int* n_kl, uint8_t* desc);
int  gfpl_lbd_status(gfpl_lbd* lbd);
/* test hook of ledger L1-L2: the Gaussian-blurred image's Sobel derivatives of one DEVICE image,
 * grad [height][width] (DEVICE) = dx (low 16 bits) | dy (high 16 bits).  Synchronises.      */
int  gfpl_lbd_gradients(gfpl_lbd* lbd, const uint8_t* image, uint32_t* grad);

/* ---------------------------------------- LSD line detection (§8(f)2) ---- */
/* line_descriptor::LSDDetectorC::detect(image, keylines, scale, numOctaves, opts)
 * (3rdparty/line_descriptor/src/LSDDetector_custom.cpp:218-316) as
 * StereoFrame::detectLineFeatures calls it (src/stereoFrame.cpp:1160-1186): one octave,
 * cv::createLineSegmentDetector(opts...) ->detect (OpenCV 3.4.1 lsd.cpp, LSD_REFINE_STD,
 * scale 1), the keylines' extremes clamped, segments not longer than min_length dropped,
 * then, when more than n_features remain and n_features != 0, std::sort by response
 * (include/auxiliar.h:149-154) and the first n_features kept (:1177-1185).  Arithmetic
 * pinned as the CPU oracle's ledger S1-S7 (oracle/gfpl_lsd_oracle.cpp).   */
typedef struct gfpl_lsd_params {
    int    refine;        /* Config::lsdRefine 1 (= LSD_REFINE_STD; only value supported)  */
    double scale;         /* Config::lsdScale 1 (only value supported)                     */
    double quant;         /* Config::lsdQuant 2.0                                          */
    double ang_th;        /* Config::lsdAngTh 22.5                                         */
    double density_th;    /* Config::lsdDensityTh 0.6                                      */
    int    n_bins;        /* Config::lsdNBins 1024                                         */
    double min_length;    /* Config::minLineLength * min(W, H) (src/stereoFrame.cpp:151)   */
    int    n_features;    /* Config::lsdNFeatures 300 (0 = keep all)                       */
} gfpl_lsd_params;
typedef struct gfpl_lsd gfpl_lsd;
/* images up to 2048 x 2048 (and >= 8 x 8), up to max_images per call; kl_cap keylines out
 * per image; seg_cap raw segments per image (GFPL_E_CAPACITY beyond).                       */
int  gfpl_lsd_create(gfpl_ctx* ctx, const gfpl_lsd_params* prm, int width, int height, int max_images,
                     int kl_cap, int seg_cap, gfpl_lsd** out);
int  gfpl_lsd_destroy(gfpl_lsd* lsd);
/* all pointers DEVICE: images [n][height][width] u8; keylines [n][kl_cap] receives image j's
 * keylines (sx sy ex ey angle octave) in the reference's output order, n_kl [n] their count,
 * response [n][kl_cap] (nullable) KeyLine::response.  Keylines beyond kl_cap are an error
 * (GFPL_E_CAPACITY).  Synchronises.                                                        */
int  gfpl_lsd_detect(gfpl_lsd* lsd, const uint8_t* images, int n, gfpl_keyline* keylines, int* n_kl,
                     float* response);
/* stream-ordered form; gfpl_lsd_status reports (and waits for) the async calls since the last */
int  gfpl_lsd_detect_async(gfpl_lsd* lsd, const uint8_t* images, int n, gfpl_keyline* keylines, int* n_kl,
                           float* response);
int  gfpl_lsd_status(gfpl_lsd* lsd);
/* test hook of ledger S2: std::sort(a, a + n, key(x) > key(y)) with key = the high 32 bits of
 * each element, on DEVICE memory (n <= (width-1)(height-1)); the permutation the seed order
 * and the response sort use.  Synchronises.                                                 */
int  gfpl_lsd_sort_desc(gfpl_lsd* lsd, uint64_t* a, int n);

/* ------------------------------- stereo detection from images (§8(f)1-2) ---- */
/* The detection half of StereoFrame(img_l, img_r, idx, cam, ts) as
 * StereoFrameHandler::initialize / insertStereoPair(const Mat& img_l, const Mat& img_r,
 * int idx, double ts) run it (include/stereoFrameHandler.h:48-53, src/stereoFrame.cpp:
 * 148-172, 411-450, 1128-1227; called at app/plslam_mod.cpp:377,387): ORB of both images
 * (the right one's pyramid kept for the sub-pixel refinement), LSD of both with the
 * lsdNFeatures response cut, LBD of both — for B stereo frames, into device buffers a
 * gfpl_frames view points at, so gfpl_initialize / gfpl_insert_stereo_pair / gfpl_frame_step
 * read them without a copy.  The detector runs on two streams of its own; the view's
 * `ready` event orders the tracker call after the detection and its `consumed` event
 * (recorded by that tracker call) orders the next detection into the same buffer set
 * (`sets` of them, used in turn) after the read.                                        */
typedef struct gfpl_detector_params {
    gfpl_orb_params orb;   /* Config::orbNFeatures / orbScaleFactor / orbNLevels, 20, 7     */
    gfpl_lsd_params lsd;   /* the LSDOptions + lsdNFeatures + min line length              */
    int seg_cap;           /* raw LSD segments per image (GFPL_E_CAPACITY beyond), 4096     */
} gfpl_detector_params;
typedef struct gfpl_detector gfpl_detector;
/* the reference's Config defaults (src/config.cpp:107,134-152) for this camera; cfg NULL =
 * gfpl_config_default.  (BASELINE cfg 2 runs orb.nfeatures = 2000.)                      */
int  gfpl_detector_params_default(const gfpl_camera* cam, const gfpl_config* cfg, gfpl_detector_params* prm);
/* On a context with a camera (GFPL_E_STATE otherwise); images are the camera's size, up
 * to max_batch stereo frames per call; kp_cap / kl_cap rows per image (as the seqbatch's);
 * sets 1..4 buffer sets.  The context cannot be destroyed while the detector lives.      */
int  gfpl_detector_create(gfpl_ctx* ctx, const gfpl_detector_params* prm, int max_batch, int kp_cap,
                          int kl_cap, int sets, gfpl_detector** out);
int  gfpl_detector_destroy(gfpl_detector* det);
/* Stream-ordered detection of n stereo frames: img_l / img_r DEVICE [n][H][W] u8 and
 * time_stamp DEVICE [n], produced on the context's stream (the detection waits for it).
 * *out is the view of the next buffer set (valid until that set is detected into again).
 * GFPL_E_STATE when the set's previous view was never read by a tracker call (nor
 * released with gfpl_detector_discard): at most `sets` views may be outstanding.
 * The inputs are copied on the detector's stream and the context's stream is made to wait
 * for that copy, so the caller may overwrite img_l / img_r / time_stamp with work it
 * enqueues on the context's stream after this call returns.                            */
int  gfpl_detect_stereo_async(gfpl_detector* det, const uint8_t* img_l, const uint8_t* img_r, int n,
                              const double* time_stamp, gfpl_frames* out);
/* The same from HOST images / time stamps (copied before it returns; the detection
 * itself stays asynchronous).                                                            */
int  gfpl_detect_stereo_host(gfpl_detector* det, const uint8_t* img_l, const uint8_t* img_r, int n,
                             const double* time_stamp, gfpl_frames* out);
/* capacity / octave errors of the detections since the last status (waits for them) */
int  gfpl_detector_status(gfpl_detector* det);
/* detect (host_pointers: the _host form) + status: returns after the detection finished */
int  gfpl_detect_stereo(gfpl_detector* det, const uint8_t* img_l, const uint8_t* img_r, int n,
                        const double* time_stamp, int host_pointers, gfpl_frames* out);
/* release a view no tracker call will read (its set may then be detected into again) */
int  gfpl_detector_discard(gfpl_detector* det, const gfpl_frames* view);

/* Host copy of one sequence's detections of a DEVICE gfpl_frames view (the
 * points_l / points_r / pdesc_* / lines_* / ldesc_* members of the reference's StereoFrame
 * after detection).  Arrays are caller-allocated at the view's kp_cap / kl_cap (a NULL
 * array is skipped); waits for the view's `ready` event.                               */
typedef struct gfpl_detections_host {
    int n_kp_l, n_kp_r, n_kl_l, n_kl_r;
    gfpl_keypoint* kp_l;  gfpl_keypoint* kp_r;
    uint8_t* pdesc_l;     uint8_t* pdesc_r;   /* [cap][32] */
    gfpl_keyline* kl_l;   gfpl_keyline* kl_r;
    uint8_t* ldesc_l;     uint8_t* ldesc_r;   /* [cap][32] */
} gfpl_detections_host;
int  gfpl_read_detections(gfpl_ctx* ctx, const gfpl_frames* view, int seq, gfpl_detections_host* out);

/* ------------------------------------------------- keyframe consumers ---- */
/* One keyframe's stereo features as KeyFrame::stereo_frame exposes them
 * (src/keyFrame.cpp:26-58, include/stereoFrame.h public members): row i of
 * every point array is stereo_pt[i] and row i of pdesc its left descriptor
 * (pdesc_l); likewise stereo_ls[i] / ldesc_l.  gfpl_kf_common_matches reads
 * the arrays from DEVICE memory (e.g. a gfpl_frame_host uploaded by the
 * caller, or a frame slot it copied out); T_kf_w is a host 4x4 row-major pose. */
typedef struct gfpl_kf_view {
    int            n_pt;
    const uint8_t* pdesc;       /* [n_pt][32]                                  */
    const double*  P;           /* [n_pt][3]  stereo_pt[i]->P                  */
    const double*  pl;          /* [n_pt][2]  stereo_pt[i]->pl                 */
    const double*  pt_sigma2;   /* [n_pt]     stereo_pt[i]->sigma2             */
    int            n_ls;
    const uint8_t* ldesc;       /* [n_ls][32]                                  */
    const double*  sP;          /* [n_ls][3]                                   */
    const double*  eP;          /* [n_ls][3]                                   */
    const double*  le;          /* [n_ls][3]                                   */
    const double*  ls_sigma2;   /* [n_ls]                                      */
    double         T_kf_w[16];  /* KeyFrame::T_kf_w (host)                     */
} gfpl_kf_view;

/* MapHandler::lookForCommonMatches, keyframe-pair stage (src/mapHandler.cpp:
 * 199-470, has_refinement = false as in the reference): DT = inverse_se3(kf1
 * T_kf_w) * kf0 T_kf_w; points: knn-2 NORM_HAMMING kf0->kf1 and kf1->kf0,
 * mutual best, d0/d1 <= max_ratio_12_p, |proj(DT P0) - pl1| * sqrt(sigma2_0) <
 * sqrt(7.815); lines: knn-2 NORM_HAMMING both ways, mutual, d1 - d0 >
 * lineDescriptorMAD(matches_12).nn12 * desc_th_l, |(le0 . proj(DT sP0),
 * le0 . proj(DT eP0))| * sqrt(sigma2_0) < sqrt(7.815).  The accepted (kf0 row,
 * kf1 row) pairs are written in kf0 row order to pt_pairs [2 * kf0->n_pt] and
 * ls_pairs [2 * kf0->n_ls] (device) and their counts to *n_pt_pairs /
 * *n_ls_pairs (host; the call synchronises).  The landmark bookkeeping that
 * follows each accepted pair (MapPoint / MapLine creation, observations,
 * full_graph) stays with the caller, which walks the pairs in the returned
 * order exactly as the reference's loop does.  A kind with fewer than two rows
 * on either keyframe yields no pairs (the reference reads a missing second
 * neighbour: ledger U4).                                                      */
int  gfpl_kf_common_matches(gfpl_ctx* ctx, const gfpl_kf_view* kf0, const gfpl_kf_view* kf1,
                            int32_t* pt_pairs, int* n_pt_pairs, int32_t* ls_pairs, int* n_ls_pairs);

/* The local map as lookForCommonMatches' second stage reads it (src/mapHandler.cpp:
 * 472-772): the map points / lines the caller keeps as local and not yet observed
 * by kf1 (`local && kf_obs_list.back() != kf1_idx`), in map order, with their
 * median descriptor (med_desc.row(0)) and 3D geometry (point3D; line3D = sP, eP).
 * Device pointers.                                                              */
typedef struct gfpl_map_view {
    int            n_pt;
    const uint8_t* pdesc;       /* [n_pt][32]                                  */
    const double*  P;           /* [n_pt][3]  point3D (world)                  */
    int            n_ls;
    const uint8_t* ldesc;       /* [n_ls][32]                                  */
    const double*  L;           /* [n_ls][6]  line3D (world sP, eP)            */
} gfpl_map_view;

/* lookForCommonMatches, local-map stage (src/mapHandler.cpp:472-772): with
 * Twf = inverse_se3(kf1 T_kf_w), the map rows whose projection lies inside the
 * image in front of the camera (:479-490 points, :615-632 lines, both endpoints)
 * are matched against kf1's UNMATCHED features (the caller passes kf1 compacted
 * to its idx == -1 rows, :495-505 / :637-647): knn-2 NORM_HAMMING both ways,
 * mutual best; points: d0/d1 <= max_ratio_12_p, Pf.z > 0 and |proj(Pf) - pl| <
 * max_kf_epip_p; lines: d1 - d0 > lineDescriptorMAD.nn12 * desc_th_l, both
 * endpoints in front and the SIGNED line residuals le . proj(endpoint) both <
 * max_kf_epip_l (the reference compares them without abs).  Pairs (map row in
 * the caller's map_view, kf1 row) in the reference's loop order; counts on the
 * host (synchronises).  Config::maxKFEpipP / maxKFEpipL default to 1.0
 * (src/config.cpp:42-43).  Fewer than two rows on a side: no pairs (U4).      */
int  gfpl_kf_local_map_matches(gfpl_ctx* ctx, const gfpl_map_view* map, const gfpl_kf_view* kf1,
                               double max_kf_epip_p, double max_kf_epip_l,
                               int32_t* pt_pairs, int* n_pt_pairs, int32_t* ls_pairs, int* n_ls_pairs);

/* ----------------------------------------------------- state transfer ----- */
/* Copy one sequence's frame state device -> host (synchronises).            */
int  gfpl_read_frame(gfpl_seqbatch* sb, int which, int seq, gfpl_frame_host* out);
/* Copy a host frame state into one sequence (synchronises).  Used to start a
 * stage from a given state (e.g. the oracle's), like the reference's
 * simulators build frames through the public members (src/simulate_line_cut.cpp:62-212). */
int  gfpl_write_frame(gfpl_seqbatch* sb, int which, int seq, const gfpl_frame_host* in);
int  gfpl_read_track(gfpl_seqbatch* sb, int seq, gfpl_track_host* out);
int  gfpl_write_track(gfpl_seqbatch* sb, int seq, const gfpl_track_host* in);
/* The track of the step before the last gfpl_update_frame / gfpl_frame_step: the
 * matched lists it cleared (matched_pt.clear(), src/stereoFrameHandler.cpp:889-890)
 * as they stood, and the inlier counters.  Valid until the next insert; lets a
 * caller that drives gfpl_frame_step inspect each step without splitting it.  */
int  gfpl_read_last_track(gfpl_seqbatch* sb, int seq, gfpl_track_host* out);

/* ----------------------------------------------------- instrumentation ---- */
/* Per-stage device time of the last gfpl_frame_step (HIP events on the
 * context stream), ms: [stereo_points, stereo_lines, cross_points,
 * cross_lines, line_cut, pose, total].  Enable with gfpl_set_timing(ctx,1). */
int  gfpl_set_timing(gfpl_ctx* ctx, int enable);
int  gfpl_get_stage_times(gfpl_ctx* ctx, float* ms7);
/* Algorithmic bytes of the last step (SURVEY.md §8(d) formula, from runtime
 * counts, summed over the batch).  Synchronises.                           */
int  gfpl_last_step_bytes(gfpl_seqbatch* sb, int64_t* bytes);
/* ... per stage: [stereo_points, stereo_lines, cross_points, cross_lines,
 * line_cut, pose, total] (DESIGN.md §Roofline gives each stage's formula). */
int  gfpl_last_step_stage_bytes(gfpl_seqbatch* sb, int64_t* bytes7);
/* The counts those bytes are priced on, summed over the batch: [N_o (keypoints, both
 * sides), N_k (keylines, both sides), M_o (left keypoints reaching the sub-pixel SAD),
 * S_p (stereo points of the new frame), S_l (its stereo lines), M_p (matched_pt), M_l
 * (matched_ls), n_inliers] of the last insert.  Synchronises.                   */
int  gfpl_last_step_counts(gfpl_seqbatch* sb, int64_t* counts8);
/* More of the last step, summed over the batch: [line-cut greedy steps, steps the
 * certified search evaluated with the reference's own arithmetic (the exact fallback,
 * DESIGN.md §3), n_inliers after optimize_pose (removeOutliers; until it runs, the
 * insert's list sizes), searched lines whose agreement bound was unusable —
 * every step of such a line is exact].  Synchronises.                                */
int  gfpl_last_step_track_counts(gfpl_seqbatch* sb, int64_t* counts4);
/* Proven line cut (cut_proof 1) of the last step, summed over the batch: [sequences whose
 * recorded search k_cut_verify could not prove (their line cut was redone by the eager-proven
 * search), margined steps proven after the fact, the reference's endpoint variances evaluated
 * for them, lines with margined steps].  Zeros in the other modes.  Synchronises.        */
int  gfpl_last_step_cut_proof(gfpl_seqbatch* sb, int64_t* counts4);
/* Diagnostics: the line-cut records of sequence b's first n_lines matched lines of the last
 * insert (80 doubles each: comparison data, bounds, r = 0 info, the agreement bound as
 * k_cut_search formed it — DESIGN.md §3; layout in k_cut.hip).  Synchronises.      */
int  gfpl_debug_cut_records(gfpl_seqbatch* sb, int b, double* out, int n_lines);
/* Every sequence's record of the last step: B x 24 int64 — stage bytes [0..7], the counts of
 * gfpl_last_step_counts [8..15], line-cut steps / exact steps [16..17], inliers after the pose
 * [18], lines without a usable bound [19] (layout: STEP_REC in gfpl_state.hpp).  Synchronises. */
int  gfpl_debug_step_records(gfpl_seqbatch* sb, int64_t* out);
/* B x 8 int64 of diagnostic slots: the clocks instrumented builds of the library write (e.g.
 * -DGFPL_SP_CLOCK: k_stereo_points' phase boundaries); in every build, after a measured-mode step
 * with the 8-sequence-per-wave line-cut search, slots 6 / 7 hold that search wave's HW_ID / XCC_ID
 * (its SIMD and wave slot: the progress exchange's partner check).  Synchronises.               */
int  gfpl_debug_clocks(gfpl_seqbatch* sb, int64_t* out);
/* Per-kernel view of the dominant stages (timing enabled, line cut on):
 * ms4 = device ms of [k_cut_prep, k_cut_search, k_cut_finish, k_pose] of the last
 * step (HIP events on the context stream); bytes4 = algorithmic bytes of the same
 * kernels, summed over the batch (each kernel's own inputs read once and
 * outputs written once; 0 for the cut kernels when the step ran no line cut).  */
int  gfpl_get_kernel_times(gfpl_ctx* ctx, float* ms4);
int  gfpl_last_step_kernel_bytes(gfpl_seqbatch* sb, int64_t* bytes4);

const char* gfpl_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* GFPL_H */
