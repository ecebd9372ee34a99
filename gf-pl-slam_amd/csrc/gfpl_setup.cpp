// Host-side setup of the C ABI: Config defaults, camera tables, error strings.
#include "../../include/gfpl.h"

#include <cmath>
#include <cstring>

extern "C" int gfpl_abi_version(void) { return GFPL_ABI_VERSION; }

// Config::Config() (src/config.cpp:26-154), the fields the path reads.
extern "C" int gfpl_config_default(gfpl_config* c) {
    if (!c) return GFPL_E_INVALID;
    std::memset(c, 0, sizeof(*c));
    c->best_lr_matches = 1;
    c->lr_in_parallel = 1;
    c->use_line_conf_cut = 1;
    c->cut_with_max_vol = 1;
    c->ratio_disp_std = 0.15;
    c->ratio_disp_std_hor = 0.9;
    c->max_line_match_num = 300;
    c->max_point_match_num = 500;
    c->max_dist_epip = 2.0;
    c->min_disp = 1.0;
    c->max_ratio_12_p = 0.9;
    c->point_match_radius = 50.0;
    c->stereo_overlap_th = 0.5;
    c->line_horiz_th = 0.1;
    c->desc_th_l = 0.1;
    c->line_cov_th = 10.0;
    c->homog_th = 0.0000001;
    c->min_features = 10;
    c->max_iters = 5;
    c->max_iters_ref = 10;
    c->min_error = 0.0000001;
    c->min_error_change = 0.0000001;
    c->inlier_k = 2.0;
    c->motion_step_th = 10;
    c->orb_scale_factor = 1.2;
    c->orb_n_levels = 4;
    c->lsd_scale = 1;
    c->cut_step = 0.05;
    c->cut_rng[0] = 0.0;
    c->cut_rng[1] = 1.0;
    c->proj_gate_px = 10.0;
    c->min_entropy_ratio = 0.90;
    c->max_kf_num_frames = 50;
    c->cut_certify = 1e-9;
    c->cut_proof = 0;
    return GFPL_OK;
}

// Scale tables as ORBextractor's ctor builds them (src/ORBextractor.cc:410-431:
// float ctor argument stored in a double member), pyramid level sizes as
// ComputePyramid (:1107-1114, cvRound((float)cols*invScale)), sigma2 tables as
// the PointFeature / LineFeature ctors (src/stereoFeatures.cpp:41-47,96-101).
extern "C" int gfpl_camera_init(gfpl_camera* cam, int width, int height, double fx, double fy,
                                double cx, double cy, double b, const gfpl_config* cfg) {
    if (!cam || !cfg || width <= 0 || height <= 0) return GFPL_E_INVALID;
    if (cfg->orb_n_levels < 1 || cfg->orb_n_levels > GFPL_MAX_LEVELS) return GFPL_E_INVALID;
    std::memset(cam, 0, sizeof(*cam));
    cam->width = width;
    cam->height = height;
    cam->fx = fx; cam->fy = fy; cam->cx = cx; cam->cy = cy; cam->b = b;
    cam->n_levels = cfg->orb_n_levels;
    const double member = (double)(float)cfg->orb_scale_factor;
    cam->scale[0] = 1.0f;
    for (int i = 1; i < cam->n_levels; ++i) cam->scale[i] = (float)((double)cam->scale[i - 1] * member);
    int64_t off = 0;
    for (int i = 0; i < cam->n_levels; ++i) {
        cam->inv_scale[i] = 1.0f / cam->scale[i];
        cam->lvl_cols[i] = (int)std::lrint((double)((float)width * cam->inv_scale[i]));
        cam->lvl_rows[i] = (int)std::lrint((double)((float)height * cam->inv_scale[i]));
        cam->lvl_offset[i] = off;
        off += (int64_t)cam->lvl_cols[i] * cam->lvl_rows[i];
    }
    // keep every sequence's pyramid 256-byte aligned inside a batch, with a tail of
    // at least GFPL_PYR_TAIL bytes (the SAD window rows are read as aligned dwords)
    cam->pyr_bytes = (off + GFPL_PYR_TAIL + 255) & ~(int64_t)255;
    for (int l = 0; l < GFPL_MAX_LEVELS; ++l) {
        double s = 1.0;
        for (int i = 0; i < l + 1; ++i) s *= cfg->orb_scale_factor;
        cam->sigma2_pt[l] = 1.f / (s * s);
        double t = 1.0;
        for (int i = 0; i < l + 1; ++i) t *= cfg->lsd_scale;
        cam->sigma2_ln[l] = 1.f / (t * t);
    }
    return GFPL_OK;
}

extern "C" const char* gfpl_strerror(int code) {
    switch (code) {
        case GFPL_OK: return "ok";
        case GFPL_E_INVALID: return "invalid argument";
        case GFPL_E_HIP: return "HIP runtime error";
        case GFPL_E_NO_DEVICE: return "no HIP device";
        case GFPL_E_TOO_FEW_TRAIN: return "knn-2 needs at least 2 train descriptors";
        case GFPL_E_CAPACITY: return "feature count exceeds seqbatch capacity";
        case GFPL_E_STATE: return "call order violated";
        case GFPL_E_UNSUPPORTED: return "config flag combination not implemented";
        default: return "unknown error";
    }
}
