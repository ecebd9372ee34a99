/*
 * gfpl_oracle.h — CPU ORACLE for the GF-PL-SLAM tracking hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product path (libgfpl_hip.so) never links,
 * loads or calls it.
 *
 * It is a plain C++ restatement of the reference's algorithm
 * (SimonsRoad/gf-pl-slam; every function cites the file:line it follows) with
 * the semantics ledger of SURVEY.md §8(c) pinned explicitly (U1-U7, Q1-Q15,
 * T1) plus the numeric pins listed in DESIGN.md §"Oracle":
 *   N1  all floating point without contraction (-ffp-contract=off);
 *   N2  Eigen expression trees are evaluated in their left-to-right order,
 *       inner products k-sequential, sums over lists sequential in list order;
 *   N3  log / sin / cos are the fdlibm algorithms (e_log.c, k_sin.c, k_cos.c,
 *       e_rem_pio2.c medium branch) evaluated with + - * / only, because the
 *       reference's own values come from Eigen packet math / libm and are not
 *       reproducible across machines;
 *   N4  SelfAdjointEigenSolver -> cyclic Jacobi; LDLT -> Eigen 3.3
 *       ldlt_inplace<Lower> with pivoting + pseudo-inverse D solve;
 *       inverse() of 6x6 -> partial-pivot LU; of 4x4 -> cofactor expansion.
 *
 * Parity status: the reference cannot be compiled in this image (OpenCV 3.4.1,
 * Eigen3, g2o, Boost, yaml-cpp absent) and has no Python
 * implementation and no usable golden vectors.  This oracle is pinned by
 * hand-derived known answers (tests/test_oracle_known_answers.py) and the
 * golden fixtures it generated (tests/golden/, make_golden.py).
 */
#ifndef GFPL_ORACLE_H
#define GFPL_ORACLE_H
#include "../include/gfpl.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gfplo_handler gfplo_handler;

gfplo_handler* gfplo_create(const gfpl_camera* cam, const gfpl_config* cfg);
void gfplo_destroy(gfplo_handler* h);

/* StereoFrameHandler::initialize (src/stereoFrameHandler.cpp:45-81); in = host
 * frames batch, row `seq` is used. */
int gfplo_initialize(gfplo_handler* h, const gfpl_frames* in, int seq);
/* insertStereoPair (src/stereoFrameHandler.cpp:83-151) */
int gfplo_insert_stereo_pair(gfplo_handler* h, const gfpl_frames* in, int seq);
/* optimizePose(prev_frame->DT) (src/stereoFrameHandler.cpp:1939-2030) */
int gfplo_optimize_pose(gfplo_handler* h);
int gfplo_optimize_pose_ini(gfplo_handler* h, const double* DT_ini);
/* updateFrame_ECCV18 swap (src/stereoFrameHandler.cpp:864-922) */
int gfplo_update_frame(gfplo_handler* h);
/* needNewKF / currFrameIsKF (src/stereoFrameHandler.cpp:2309-2379) */
int gfplo_need_new_kf(gfplo_handler* h, int* flag);
int gfplo_curr_frame_is_kf(gfplo_handler* h);
int gfplo_read_kf_state(gfplo_handler* h, gfpl_kf_state* out);

/* ORB_SLAM2::ORBextractor::operator() (src/ORBextractor.cc:1043-1105) on one grey image
 * (gfpl_orb_oracle.cpp; ledger O1-O7): keypoints (x, y, octave) in the reference's output
 * order, their angle / FAST response, 32-byte descriptors; pyramid (nullable) receives the
 * level images packed consecutively (the right pyramid of gfpl_frames). */
int gfplo_orb_extract(const gfpl_orb_params* prm, const uint8_t* image, int width, int height, int kp_cap,
                      gfpl_keypoint* kps, float* angle, float* response, uint8_t* desc, int* n_kp,
                      uint8_t* pyramid);
int gfplo_orb_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh);   /* O1 */
int gfplo_orb_blur(const uint8_t* src, int w, int h, uint8_t* dst);                       /* O2 */
/* O3: FAST(img, kps, threshold, nonmax) on a whole image; xy_score[3*i] = x, y, response */
int gfplo_orb_fast(const uint8_t* img, int w, int h, int threshold, int cap, float* xy_score);
float gfplo_fast_atan2(float y, float x);                                                 /* O4 */

/* line_descriptor::BinaryDescriptor::compute(image, keylines, descriptors)
 * (3rdparty/line_descriptor/src/binary_descriptor_custom.cpp:539-687, computeLBD :1026-1372) for
 * octave-0 keylines (gfpl_lbd_oracle.cpp; ledger L1-L5): desc [n][32] (nullable), desc_f [n][72]
 * the float LBD vector before binarisation (nullable). */
int gfplo_lbd_compute(const uint8_t* image, int width, int height, const gfpl_keyline* kl, int n,
                      uint8_t* desc, float* desc_f);
/* the Gaussian-blurred image (L1) and its 16-bit Sobel derivatives (L2); outputs nullable */
int gfplo_lbd_gradients(const uint8_t* image, int width, int height, uint8_t* blur, int16_t* dx, int16_t* dy);
/* gaussCoefL_[21], gaussCoefG_[63] as the float values computeLBD uses (L4) */
int gfplo_lbd_coefs(float* coef_l, float* coef_g);
/* LSDDetectorC's numOfPixels of a keyline (cv::LineIterator count, 8-connectivity) */
int gfplo_lbd_num_pixels(const gfpl_keyline* kl, int width, int height);

/* line_descriptor::LSDDetectorC::detect as StereoFrame::detectLineFeatures calls it
 * (3rdparty/line_descriptor/src/LSDDetector_custom.cpp:218-316, src/stereoFrame.cpp:1160-1186;
 * gfpl_lsd_oracle.cpp, ledger S1-S7) on one grey image: keylines (nullable) in the reference's
 * output order, response (nullable), n_kl; segs (nullable) [seg_cap][4] the raw LSD segments
 * (after the 0.5 offset, before checkLineExtremes), n_seg their count (nullable). */
int gfplo_lsd_detect(const gfpl_lsd_params* prm, const uint8_t* image, int width, int height, int kl_cap,
                     gfpl_keyline* kls, float* response, int* n_kl, float* segs, int seg_cap, int* n_seg);
/* flsd's per-image constants (S5): prec, rho = quant / sin(prec), min_reg_size */
int gfplo_lsd_constants(const gfpl_lsd_params* prm, int width, int height, double* prec, double* rho,
                        int* min_reg_size);
double gfplo_atan2(double y, double x);                                                  /* S4 */
/* S2: std::sort(a, a + n) by descending high 32 bits (the library's introsort) */
int gfplo_sort_desc(uint64_t* a, int n);

/* MapHandler::lookForCommonMatches keyframe-pair stage (src/mapHandler.cpp:
 * 199-470); same contract as gfpl_kf_common_matches but every pointer of the
 * views and outputs is HOST memory. */
int gfplo_kf_common_matches(const gfpl_camera* cam, const gfpl_config* cfg, const gfpl_kf_view* kf0,
                            const gfpl_kf_view* kf1, int32_t* pt_pairs, int* n_pt_pairs, int32_t* ls_pairs,
                            int* n_ls_pairs);

/* lookForCommonMatches local-map stage (src/mapHandler.cpp:472-772); contract of
 * gfpl_kf_local_map_matches with HOST pointers. */
int gfplo_kf_local_map_matches(const gfpl_camera* cam, const gfpl_config* cfg, const gfpl_map_view* map,
                               const gfpl_kf_view* kf1, double max_kf_epip_p, double max_kf_epip_l,
                               int32_t* pt_pairs, int* n_pt_pairs, int32_t* ls_pairs, int* n_ls_pairs);

/* stage-level entry points (same split as include/gfpl.h) */
int gfplo_begin_frame(gfplo_handler* h, const gfpl_frames* in, int seq);   /* new curr_frame */
int gfplo_stereo_points(gfplo_handler* h);
int gfplo_stereo_lines(gfplo_handler* h);
int gfplo_line_uncertainty(gfplo_handler* h);
int gfplo_cross_points(gfplo_handler* h);   /* includes predictFramePose */
int gfplo_cross_lines(gfplo_handler* h);
int gfplo_line_cut(gfplo_handler* h);

int gfplo_read_frame(gfplo_handler* h, int which, gfpl_frame_host* out);
int gfplo_write_frame(gfplo_handler* h, int which, const gfpl_frame_host* in);
int gfplo_read_track(gfplo_handler* h, gfpl_track_host* out);
int gfplo_write_track(gfplo_handler* h, const gfpl_track_host* in);

/* primitives (known-answer tests) */
int    gfplo_hamming(const uint8_t* a, const uint8_t* b, int cell);
int    gfplo_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell,
                  int32_t* out_idx, float* out_dist);
double gfplo_log(double x);
double gfplo_sin(double x);
double gfplo_cos(double x);
double gfplo_logdet6(const double* M36);
int    gfplo_ldlt_solve6(const double* H36, const double* g6, double* x6);
int    gfplo_inverse6(const double* A36, double* out36);
/* Matrix6d::determinant (PartialPivLU, diagonal product left to right) */
double gfplo_det6(const double* A36);
int    gfplo_inverse4(const double* A16, double* out16);
int    gfplo_eig_sym(const double* A, int n, double* w);
int    gfplo_expmap_se3(const double* x6, double* T16);
int    gfplo_inverse_se3(const double* T16, double* out16);

#ifdef __cplusplus
}
#endif
#endif
