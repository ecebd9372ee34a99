// gfpl_state.hpp — HBM layout of B resident sequences (one StereoFrameHandler
// each) and the parameter block every kernel receives by value.
//
// Layout: structure-of-arrays per frame slot, [B][cap][k] per field, so lane i
// of a wave touches feature i of one sequence (coalesced 8/16/24-B rows).
// Two frame slots ping-pong between prev and curr (updateFrame_ECCV18 is a
// pointer swap, src/stereoFrameHandler.cpp:910-912).
#pragma once
#include <stdint.h>

#include "../../include/gfpl.h"
#include "gfpl_device.hpp"

namespace gfpl {

struct DevPoints {            // StVO::PointFeature (include/stereoFeatures.h:36-60)
    double* pl;      // [B*cap*2]
    double* pl_obs;  // [B*cap*2]
    double* disp;    // [B*cap]
    double* P;       // [B*cap*3]
    double* sigma2;  // [B*cap]
    int32_t* idx;    // [B*cap]
    int32_t* level;  // [B*cap]
    uint8_t* inlier; // [B*cap]
    uint8_t* desc;   // [B*cap*32]  pdesc_l
    int32_t* n;      // [B]
};

struct DevLines {             // StVO::LineFeature (include/stereoFeatures.h:62-124)
    double *spl, *epl, *spl_obs, *epl_obs;        // [B*cap*2]
    double *sdisp, *edisp, *sdisp_obs, *edisp_obs; // [B*cap]
    double *angle, *sigma2;                        // [B*cap]
    double *sP, *eP, *le, *le_obs;                 // [B*cap*3]
    double *covS, *covE;                           // [B*cap*9]
    double *cut;                                   // [B*cap*2]
    double *invcov;                                // [B*cap*36]
    int32_t *idx, *level;                          // [B*cap]
    uint8_t *inlier;                               // [B*cap]
    uint8_t *desc;                                 // [B*cap*32]  ldesc_l
    int32_t* n;                                    // [B]
};

struct DevPose {
    double *Tfw, *DT;            // [B*16]
    double *DT_cov, *Tfw_cov;    // [B*36]
    double *DT_cov_eig;          // [B*6]
    double *err_norm, *time_stamp; // [B]
};

struct DevFrame {
    DevPoints pt;
    DevLines ls;
    DevPose pose;
};

struct DevTrack {
    int32_t* matched_pt;   // [B*mpt_cap]
    int32_t* n_matched_pt; // [B]
    int32_t* matched_ls;   // [B*mls_cap]
    int32_t* n_matched_ls; // [B]
    int32_t* n_inliers;    // [B]
    int32_t* n_inliers_pt; // [B]
    int32_t* n_inliers_ls; // [B]
    int32_t* num_frame_loss; // [B]
    // keyframe decision (needNewKF / currFrameIsKF, include/stereoFrameHandler.h:147-153)
    double* kf_T;          // [B*16] T_prevKF
    double* kf_cov;        // [B*36] cov_prevKF_currF
    double* kf_entropy0;   // [B] entropy_first_prevKF
    double* kf_ratio;      // [B] entropy ratio of the last decision
    int32_t* kf_prev_iskf; // [B] prev_f_iskf
    int32_t* kf_nsince;    // [B] numFrameSinceKeyframe
    int32_t* kf_flag;      // [B] last needNewKF decision
};

#define STEP_REC 24   // int64 per sequence in DevScratch::bytes: [0..5] stage bytes, [6] total, [7] k_cut_search,
                      // [8..15] counts N_o N_k M_o S_p' S_l' M_p M_l n_inliers (gfpl_last_step_counts),
                      // [16] line-cut search steps, [17] of them evaluated exactly (k_cut_search),
                      // [18] n_inliers after optimize_pose (k_pose_finish), [19] lines whose agreement bound
                      // was unusable (k_cut_search: R0 <= 0 or a term not finite; their steps are exact),
                      // proven mode (k_cut_verify): [20] 1 if the recorded search was not proven (the
                      // eager-proven search redid it), [21] margined steps verified, [22] the reference's
                      // endpoint variances evaluated, [23] lines with margined steps
#define CUT_PATH 64   // proven mode: recorded search steps per line (k_cut_search -> k_cut_verify)
#define CUT_DTL 4     // proven mode: detail-list entries per sequence (a sequence past them is redone eagerly)
#define CUT_VMAX 14   // proven mode: doubles per line of k_cut_vref's maxima [0..5] and k_cut_ebound's operand bounds (14 floats at [6..13]) (DevScratch::cut_vmax)
#define CUT_P_STAY 8  //   step byte: no neighbour beat the centre (the line ends), else the move j (0-7)
#define CUT_P_EXACT 16 //  step byte flag: the step was decided by the reference's arithmetic (exact round)
#define CUT_KS 22     // proven line cut: ratio keys per side (KParams::cut_keys)
#define CUT_FAST 56   // doubles of per-line comparison data (k_cut.hip, PD_*): polynomials, flags, error bounds
#define CUT_REC 80    // doubles of a per-line cut record: comparison data | r = 0 info (21) | pad (640 B)

struct DevScratch {
    double* cut_rec;  // [B*mls_cap*CUT_REC] per matched line: P(t) coefficients of both cut endpoints, v'(t)
                      // coefficients, geometry flag, list index of the next line | lower-triangle r = 0 info
    int32_t* knn;     // [B*6*kcap] initial-frame knn results (idx0, d0, d1, ...)
    double* proj;     // [B*kcap*2] cross-points projections (aliases knn: init never overlaps)
    int64_t* bytes;   // [B*STEP_REC] algorithmic bytes of the last step per stage | feature counts
    int32_t* n_subpix; // [B] left keypoints that reached the sub-pixel SAD (M_o)
    double* cut_sum;   // [B*24] invCov_sum (lower triangle) after the r=0 pass
    double* cut_dtinv; // [B*16] DT_inv of the line cut
    double* cut_vtab;  // [B*mls_cap*2*CUT_KS] proven line cut: the reference's scaled endpoint variance
                       // per matched line, side and ratio key (k_cut_vtab)
    double* pose_DT;   // [B*16] GN result before the final bookkeeping
    double* pose_H;    // [B*36] last evaluated H
    double* pose_err;  // [B]
    int32_t* pose_ok;  // [B] 1: stage-2 result usable
    double* pose_in;   // [B*(6*mpt_cap + 10*mls_cap)] gathered GN inputs, one AoS record per list
                       // entry (points 6 doubles, then lines 10), list order
    double* pose_act;  // [B*(6*mpt_cap + 10*mls_cap)] the active entries' records, compacted in list
                       // order per GN run (unused while every entry is active)
                        // (k_pose: points in the low, lines in the high 16 bits)
    double* pose_dtini; // [B*16] staging of gfpl_optimize_pose_ini's DT_ini
    int32_t* kf_mask;  // [B] staging of gfpl_curr_frame_is_kf's mask
    double* cross_tinv; // [B*16] inverse of the predicted curr.Tfw (k_predict_pose -> k_cross_points)
    int64_t* dbg;       // [B*8] diagnostic clocks (only builds with -DGFPL_SP_CLOCK write them)
    int32_t* cut_prog;  // [1 << 17] k_cut_search: lines done per (XCC, SE, SH, CU, SIMD, wave slot)
    uint8_t* cut_path;  // [B*mls_cap*CUT_PATH] proven mode: every line's recorded search steps
    int32_t* cut_flag;  // [B] proven mode: 1 = the recorded search was not proven (redo it eagerly)
    int32_t* cut_offl;  // [1 + B*mls_cap] proven mode: count, then the lines (b * mls_cap + m) k_cut_vref left to k_cut_vref_off
    int32_t* cut_dtln;  // [1 + CUT_DTL * B] proven mode: count, then the lines k_cut_verify left to k_cut_verify_detail
    double* cut_dtl;    // [CUT_DTL * B * 32] their payload: S_full at the line's start (21), the bound terms (9)
    double* cut_vmax;   // [B*mls_cap*CUT_VMAX] proven mode (k_cut_vref -> k_cut_verify): per line, over the ratios
                        // its margined steps compared, max 1 / v' and max r_v / v' per side, the margined
                        // steps, and the ratios whose v' comparison failed
};

// Everything a kernel needs, passed by value (kernarg segment).
struct KParams {
    DevCam cam;
    gfpl_config cfg;
    DevFrame prev, curr;
    DevTrack tr;
    DevScratch scr;
    gfpl_frames in;       // device pointers of the current input batch
    int B, kp_cap, kl_cap, mpt_cap, mls_cap;
    const double* dt_ini; // [B*16] explicit GN initial guesses (optimizePose(DT_ini)); null: prev.DT
    // derived constants, formed on the host so the kernels read them as scalars (kernel
    // arguments live in SGPRs; the same values formed on the device sit in VGPRs, which the
    // register allocator spills under pressure)
    float sp_maxD, sp_mbf;   // k_stereo_points: (float)fx, (float)(fx * b)
    double cut_tq;           // k_cut_search: cut_certify / 4 - 4u, the budget of d's rounding bound
    // proven line cut: the ratio keys — the bit patterns the greedy search's ratios take: 0, s, 2s, ...
    // as r + s accumulates them (<= rng[1]) and k s - s where its bits differ from (k - 1) s — with
    // their +s / -s links (-1: no key)
    double cut_keys[CUT_KS];
    int cut_nkeys;
    int8_t cut_knxt[CUT_KS], cut_kprv[CUT_KS];
};

}  // namespace gfpl
