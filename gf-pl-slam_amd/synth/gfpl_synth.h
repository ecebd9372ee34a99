/*
 * gfpl_synth.h — deterministic synthetic stereo frames for the tracking path.
 *
 * Detection (ORB / LSD / LBD) is outside the path, so
 * the path's inputs are injected the way the reference's own simulator builds
 * frames through the public API (src/simulate_line_cut.cpp:62-212): keypoints,
 * keylines, 32-byte descriptors and the right ORB pyramid.  Everything is a
 * pure function of (seed, seq_id, frame_idx) via splitmix64, so the CPU oracle
 * and the GPU path consume byte-identical inputs.  Not part of the product path.
 */
#ifndef GFPL_SYNTH_H
#define GFPL_SYNTH_H
#include "../../include/gfpl.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gfpl_synth_params {
    int      n_kp;            /* keypoints per side (Config::orbNFeatures, 2000 at cfg 2) */
    int      n_kl;            /* keylines per side (Config::lsdNFeatures, 500 at cfg 2)   */
    int      n_world_pts;     /* landmark pool per sequence                               */
    int      n_world_lines;   /* 3-D segment pool per sequence                            */
    double   dt;              /* frame period [s]                                         */
    double   v_fwd;           /* forward speed [m/s]                                      */
    double   yaw_rate;        /* [rad/s]                                                   */
    double   z_min, z_max;    /* landmark depth range in the first camera [m]             */
    double   px_noise;        /* keypoint / endpoint jitter sigma [px]                    */
    double   distractor_frac; /* fraction of detections with no landmark                 */
    int      margin;          /* keep detections this many px from the border             */
    uint64_t seed;
    const double* traj;       /* optional [n_traj*12] T_w<-c rows (3x4 row-major); NULL = synthetic motion */
    int      n_traj;
    const double* traj_t;     /* optional [n_traj] timestamps [s]                          */
    int      respawn;         /* 0: one landmark pool per sequence, sampled at frame 0 (it
                                 drains as the camera moves); L > 0: each pool slot is
                                 re-sampled in the current frustum every L frames (per-slot
                                 phase), so the true-keypoint share is stationary          */
    double   outlier_frac;    /* share of true observations displaced by 3-8 px (both images
                                 alike, so stereo still matches) in a frame: the cross-frame
                                 match of such an observation is a pose-optimisation outlier */
    int      pyr_from_l0;     /* right pyramid: 0 = every level drawn and stamped on its own;
                                 1 = level 0 drawn (each keypoint's patch stamped at level 0,
                                 magnified by its octave's scale) and levels 1.. resized from it
                                 as ORBextractor::ComputePyramid does (cv::resize INTER_LINEAR,
                                 src/ORBextractor.cc:1107-1132; the device's k_orb_resize);
                                 2 = level 0 only (the consumer builds the rest, e.g.
                                 gfpl_upload_frames_l0_async)                                */
} gfpl_synth_params;

/* Default parameters for a camera (cfg 2 counts: 2000 ORB + 500 LBD). */
void gfpl_synth_default(gfpl_synth_params* p);

/* Generate frame `frame_idx` of sequence `seq_id` into host buffers sized
 * kp_cap / kl_cap / cam->pyr_bytes.  T_wc_out[16] receives the ground-truth
 * camera-to-world pose (row-major) when non-NULL.  Returns 0 on success.   */
int gfpl_synth_frame(const gfpl_synth_params* p, const gfpl_camera* cam,
                     int seq_id, int frame_idx, int kp_cap, int kl_cap,
                     int* n_kp_l, int* n_kp_r, gfpl_keypoint* kp_l, gfpl_keypoint* kp_r,
                     uint8_t* pdesc_l, uint8_t* pdesc_r,
                     int* n_kl_l, int* n_kl_r, gfpl_keyline* kl_l, gfpl_keyline* kl_r,
                     uint8_t* ldesc_l, uint8_t* ldesc_r,
                     uint8_t* pyr_r, double* time_stamp, double* T_wc_out);

/* gfpl_synth_frame + n_true[2] (when non-NULL): the true (landmark) keypoints and
 * keylines per side in the frame; the rest are distractors.                   */
int gfpl_synth_frame_ex(const gfpl_synth_params* p, const gfpl_camera* cam,
                        int seq_id, int frame_idx, int kp_cap, int kl_cap,
                        int* n_kp_l, int* n_kp_r, gfpl_keypoint* kp_l, gfpl_keypoint* kp_r,
                        uint8_t* pdesc_l, uint8_t* pdesc_r,
                        int* n_kl_l, int* n_kl_r, gfpl_keyline* kl_l, gfpl_keyline* kl_r,
                        uint8_t* ldesc_l, uint8_t* ldesc_r,
                        uint8_t* pyr_r, double* time_stamp, double* T_wc_out, int* n_true);

/* Generate frames [f0, f0+nf) for sequences [s0, s0+ns) into batched host
 * arrays laid out [frame][seq][cap] using up to n_threads threads.          */
int gfpl_synth_batch(const gfpl_synth_params* p, const gfpl_camera* cam,
                     int s0, int ns, int f0, int nf, int kp_cap, int kl_cap,
                     int* n_kp_l, int* n_kp_r, gfpl_keypoint* kp_l, gfpl_keypoint* kp_r,
                     uint8_t* pdesc_l, uint8_t* pdesc_r,
                     int* n_kl_l, int* n_kl_r, gfpl_keyline* kl_l, gfpl_keyline* kl_r,
                     uint8_t* ldesc_l, uint8_t* ldesc_r,
                     uint8_t* pyr_r, double* time_stamp, int n_threads);

/* Synthetic grey image (width x height, row-major) for the ORB extraction row. */
int gfpl_synth_image(uint64_t seed, int seq_id, int frame_idx, int width, int height, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
