// gfpl_abi.hip — the extern "C" boundary (include/gfpl.h): contexts, resident
// sequence batches, stage/step entry points and state transfer.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/gfpl.h"
#include "gfpl_kernels.hpp"

using namespace gfpl;

#define GFPL_NEV 10   // timing marks: 0-6 stages, 7 after k_cut_prep, 8 after k_cut_search, 9 after k_pose

struct gfpl_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;   // gfpl_create_async: the context created (and destroys) its stream
    gfpl_camera cam{};
    gfpl_config cfg{};
    bool has_cam = false, has_cfg = false;
    bool timing = false;
    hipEvent_t ev[GFPL_NEV]{};
    float stage_ms[7]{};
    std::vector<gfpl_seqbatch*> sbs;   // live seqbatches: their match-list capacities bound gfpl_set_config
    // live ORB / LBD / LSD / detector objects: they hold the context's stream and camera; they may be
    // created and destroyed from different host threads
    std::atomic<int> n_detectors{0};
    std::mutex host_mu;   // the host-buffer matchers (gfpl_*_host): one call at a time per context
};

struct gfpl_seqbatch {
    gfpl_ctx* ctx = nullptr;
    int B = 0, kp_cap = 0, kl_cap = 0, mpt_cap = 0, mls_cap = 0;
    void* base = nullptr;
    int64_t bytes = 0;
    DevFrame slot[2];
    int prev_slot = 0;
    bool initialized = false;
    bool has_curr = false;
    DevTrack tr{};
    DevScratch scr{};
    // two device staging buffers of uploaded input batches (gfpl_upload_frames[_async]),
    // filled on a copy stream: a step reading slot s waits for ev_ready[s]; a copy into
    // slot s waits for ev_free[s], recorded after the last call that read it
    void* stage[2] = {nullptr, nullptr};
    size_t stage_bytes[2] = {0, 0};
    gfpl_frames stage_view[2]{};
    hipStream_t copy = nullptr;
    hipEvent_t ev_ready[2]{}, ev_free[2]{};
    bool ready_pending[2] = {false, false}, free_recorded[2] = {false, false};
    hipEvent_t ev_ticket[16]{};   // ticket t of gfpl_upload_frames_async -> ev_ticket[t % 16]
    int64_t n_tickets = 0;
    int32_t* last_n_pt = nullptr;   // [B] list lengths before the last gfpl_update_frame
    int32_t* last_n_ls = nullptr;   // (gfpl_read_last_track)
    PyrBuild* pyrb = nullptr;       // levels 1.. of uploaded level-0 right images (gfpl_upload_frames_l0_async)
    int last_cut_mode = -1;         // cfg.cut_proof the last line cut ran with (-1: none since the last
                                    // insert); gfpl_last_step_cut_proof reports on it, not on the current cfg
};

struct gfpl_event {
    int device = 0;
    hipEvent_t ev = nullptr;
    int64_t records = 0;   // host-side count of records (gfpl_event_record, tracker `consumed` marks)
};

// for the other extern "C" objects built on a context (k_orb.hip)
int gfpl_ctx_device(const gfpl_ctx* c) { return c->device; }
void* gfpl_ctx_stream(const gfpl_ctx* c) { return (void*)c->stream; }
const gfpl_camera* gfpl_ctx_camera(const gfpl_ctx* c) { return c->has_cam ? &c->cam : nullptr; }
int64_t gfpl_event_records(const gfpl_event* e) { return e->records; }
void gfpl_ctx_attach(gfpl_ctx* c) { c->n_detectors.fetch_add(1); }
void gfpl_ctx_detach(gfpl_ctx* c) { c->n_detectors.fetch_sub(1); }


namespace {

#define HIPCHK(x)                                                  \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) {                                     \
            std::fprintf(stderr, "gfpl: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return GFPL_E_HIP;                                      \
        }                                                           \
    } while (0)

// bump allocator over one device allocation (256-B aligned fields)
struct Carver {
    size_t off = 0;
    char* base = nullptr;
    template <typename T>
    T* take(size_t n) {
        off = (off + 255) & ~(size_t)255;
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += n * sizeof(T);
        return p;
    }
};

int debug_fill_byte() {
    const char* e = getenv("GFPL_DEBUG_FILL");
    return e ? (int)(strtol(e, nullptr, 0) & 0xFF) : 0;
}

void carve(Carver& c, gfpl_seqbatch* sb) {
    const size_t B = sb->B, P = (size_t)B * sb->kp_cap, L = (size_t)B * sb->kl_cap;
    for (int s = 0; s < 2; ++s) {
        DevFrame& f = sb->slot[s];
        f.pt.pl = c.take<double>(P * 2); f.pt.pl_obs = c.take<double>(P * 2);
        f.pt.disp = c.take<double>(P); f.pt.P = c.take<double>(P * 3); f.pt.sigma2 = c.take<double>(P);
        f.pt.idx = c.take<int32_t>(P); f.pt.level = c.take<int32_t>(P); f.pt.inlier = c.take<uint8_t>(P);
        f.pt.desc = c.take<uint8_t>(P * 32); f.pt.n = c.take<int32_t>(B);
        f.ls.spl = c.take<double>(L * 2); f.ls.epl = c.take<double>(L * 2);
        f.ls.spl_obs = c.take<double>(L * 2); f.ls.epl_obs = c.take<double>(L * 2);
        f.ls.sdisp = c.take<double>(L); f.ls.edisp = c.take<double>(L);
        f.ls.sdisp_obs = c.take<double>(L); f.ls.edisp_obs = c.take<double>(L);
        f.ls.angle = c.take<double>(L); f.ls.sigma2 = c.take<double>(L);
        f.ls.sP = c.take<double>(L * 3); f.ls.eP = c.take<double>(L * 3);
        f.ls.le = c.take<double>(L * 3); f.ls.le_obs = c.take<double>(L * 3);
        f.ls.covS = c.take<double>(L * 9); f.ls.covE = c.take<double>(L * 9);
        f.ls.cut = c.take<double>(L * 2); f.ls.invcov = c.take<double>(L * 36);
        f.ls.idx = c.take<int32_t>(L); f.ls.level = c.take<int32_t>(L); f.ls.inlier = c.take<uint8_t>(L);
        f.ls.desc = c.take<uint8_t>(L * 32); f.ls.n = c.take<int32_t>(B);
        f.pose.Tfw = c.take<double>(B * 16); f.pose.DT = c.take<double>(B * 16);
        f.pose.DT_cov = c.take<double>(B * 36); f.pose.Tfw_cov = c.take<double>(B * 36);
        f.pose.DT_cov_eig = c.take<double>(B * 6);
        f.pose.err_norm = c.take<double>(B); f.pose.time_stamp = c.take<double>(B);
    }
    sb->tr.matched_pt = c.take<int32_t>(B * sb->mpt_cap);
    sb->tr.n_matched_pt = c.take<int32_t>(B);
    sb->tr.matched_ls = c.take<int32_t>(B * sb->mls_cap);
    sb->tr.n_matched_ls = c.take<int32_t>(B);
    sb->tr.n_inliers = c.take<int32_t>(B);
    sb->tr.n_inliers_pt = c.take<int32_t>(B);
    sb->tr.n_inliers_ls = c.take<int32_t>(B);
    sb->tr.num_frame_loss = c.take<int32_t>(B);
    sb->tr.kf_T = c.take<double>(B * 16);
    sb->tr.kf_cov = c.take<double>(B * 36);
    sb->tr.kf_entropy0 = c.take<double>(B);
    sb->tr.kf_ratio = c.take<double>(B);
    sb->tr.kf_prev_iskf = c.take<int32_t>(B);
    sb->tr.kf_nsince = c.take<int32_t>(B);
    sb->tr.kf_flag = c.take<int32_t>(B);
    sb->scr.cut_rec = c.take<double>(B * sb->mls_cap * CUT_REC);
    sb->scr.knn = c.take<int32_t>(B * 2 * (size_t)sb->kp_cap * 3);
    sb->scr.proj = reinterpret_cast<double*>(sb->scr.knn);
    sb->scr.bytes = c.take<int64_t>(B * STEP_REC);
    sb->scr.n_subpix = c.take<int32_t>(B);
    sb->scr.cut_sum = c.take<double>(B * 24);
    sb->scr.cut_dtinv = c.take<double>(B * 16);
    sb->scr.cut_vtab = c.take<double>(B * sb->mls_cap * 2 * CUT_KS);
    sb->scr.pose_DT = c.take<double>(B * 16);
    sb->scr.pose_H = c.take<double>(B * 36);
    sb->scr.pose_err = c.take<double>(B);
    sb->scr.pose_ok = c.take<int32_t>(B);
    sb->scr.pose_in = c.take<double>(B * (6 * (size_t)sb->mpt_cap + 10 * (size_t)sb->mls_cap));
    sb->scr.pose_act = c.take<double>(B * (6 * (size_t)sb->mpt_cap + 10 * (size_t)sb->mls_cap));
    sb->scr.pose_dtini = c.take<double>(B * 16);
    sb->scr.cross_tinv = c.take<double>(B * 16);
    sb->scr.dbg = c.take<int64_t>(B * 8);
    sb->scr.cut_prog = c.take<int32_t>((size_t)1 << 17);
    sb->scr.cut_path = c.take<uint8_t>(B * sb->mls_cap * CUT_PATH);
    sb->scr.cut_flag = c.take<int32_t>(B);
    sb->scr.cut_vmax = c.take<double>(B * sb->mls_cap * CUT_VMAX);
    sb->scr.cut_offl = c.take<int32_t>(1 + B * sb->mls_cap);
    sb->scr.cut_dtln = c.take<int32_t>(1 + CUT_DTL * B);
    sb->scr.cut_dtl = c.take<double>(CUT_DTL * B * 32);
    sb->scr.kf_mask = c.take<int32_t>(B);
    sb->last_n_pt = c.take<int32_t>(B);
    sb->last_n_ls = c.take<int32_t>(B);
}

DevCam devcam(const gfpl_camera& c) {
    DevCam d;
    d.fx = c.fx; d.fy = c.fy; d.cx = c.cx; d.cy = c.cy; d.b = c.b;
    d.width = c.width; d.height = c.height; d.n_levels = c.n_levels;
    for (int i = 0; i < GFPL_MAX_LEVELS; ++i) {
        d.scale[i] = c.scale[i]; d.inv_scale[i] = c.inv_scale[i];
        d.lvl_cols[i] = c.lvl_cols[i]; d.lvl_rows[i] = c.lvl_rows[i];
        d.lvl_offset[i] = c.lvl_offset[i];
        d.sigma2_pt[i] = c.sigma2_pt[i]; d.sigma2_ln[i] = c.sigma2_ln[i];
    }
    d.pyr_bytes = c.pyr_bytes;
    return d;
}

KParams params(gfpl_seqbatch* sb, const gfpl_frames* in) {
    KParams p;
    std::memset(&p, 0, sizeof p);
    p.cam = devcam(sb->ctx->cam);
    p.cfg = sb->ctx->cfg;
    p.prev = sb->slot[sb->prev_slot];
    p.curr = sb->slot[1 - sb->prev_slot];
    p.tr = sb->tr;
    p.scr = sb->scr;
    if (in) p.in = *in;
    p.B = sb->B; p.kp_cap = sb->kp_cap; p.kl_cap = sb->kl_cap;
    p.mpt_cap = sb->mpt_cap; p.mls_cap = sb->mls_cap;
    // the kernels index matched_pt / matched_ls / cut and pose scratch with the
    // seqbatch's capacities; gfpl_set_config refuses larger budgets while this
    // seqbatch lives, so these clamps never change a result (defence in depth)
    p.cfg.max_point_match_num = std::min(p.cfg.max_point_match_num, sb->mpt_cap);
    p.cfg.max_line_match_num = std::min(p.cfg.max_line_match_num, sb->mls_cap);
    p.sp_maxD = (float)p.cam.fx;
    p.sp_mbf = (float)(p.cam.fx * p.cam.b);
    p.cut_tq = 0.25 * p.cfg.cut_certify - 4.0 * 0x1p-53;
    {   // the proven line cut's ratio keys (same IEEE additions as the search's r + s)
        const double s = p.cfg.cut_step, lo = p.cfg.cut_rng[0], hi = p.cfg.cut_rng[1];
        auto same = [](double x, double y) { return std::memcmp(&x, &y, sizeof x) == 0; };
        int n = 0;
        for (double t = 0.0; n < CUT_KS && t <= hi && s > 0.0; t = t + s) p.cut_keys[n++] = t;
        const int ns = n;
        for (int i = 1; i < ns && n < CUT_KS; ++i) {
            const double e = p.cut_keys[i] - s;
            bool have = false;
            for (int k = 0; k < n; ++k) have = have || same(p.cut_keys[k], e);
            if (!have && e >= lo) p.cut_keys[n++] = e;
        }
        for (int i = 0; i < n; ++i) {
            int up = -1, dn = -1;
            for (int k = 0; k < n; ++k) {
                if (same(p.cut_keys[k], p.cut_keys[i] + s)) up = k;
                if (same(p.cut_keys[k], p.cut_keys[i] - s)) dn = k;
            }
            p.cut_knxt[i] = (int8_t)up;
            p.cut_kprv[i] = (int8_t)dn;
        }
        p.cut_nkeys = n;
    }
    return p;
}

int check_in(gfpl_seqbatch* sb, const gfpl_frames* in) {
    if (!in) return GFPL_E_INVALID;
    if (in->batch != sb->B || in->kp_cap != sb->kp_cap || in->kl_cap != sb->kl_cap) return GFPL_E_INVALID;
    if (!in->n_kp_l || !in->n_kp_r || !in->kp_l || !in->kp_r || !in->pdesc_l || !in->pdesc_r || !in->n_kl_l ||
        !in->n_kl_r || !in->kl_l || !in->kl_r || !in->ldesc_l || !in->ldesc_r || !in->pyr_r || !in->time_stamp)
        return GFPL_E_INVALID;
    // the sub-pixel SAD reads pyramid rows as aligned dwords relative to each sequence's pyramid
    if (((uintptr_t)in->pyr_r & 3) != 0) return GFPL_E_INVALID;
    // producer / consumer events must live on the context's device (as gfpl_event_wait checks)
    if ((in->ready && in->ready->device != sb->ctx->device) || (in->consumed && in->consumed->device != sb->ctx->device))
        return GFPL_E_INVALID;
    return GFPL_OK;
}

// A call that reads `in` from a staging slot waits (on the context stream) for that
// slot's uploads; after enqueueing its work it marks the slot free for the next copy.
// Frames with a producer event (gfpl_frames.ready / consumed) are ordered the same way.
int in_acquire(gfpl_seqbatch* sb, const gfpl_frames* in) {
    if (in->ready && hipStreamWaitEvent(sb->ctx->stream, in->ready->ev, 0) != hipSuccess) return -2;
    for (int s = 0; s < 2; ++s)
        if (sb->stage[s] && in->n_kp_l == sb->stage_view[s].n_kp_l) {
            if (sb->ready_pending[s] && hipStreamWaitEvent(sb->ctx->stream, sb->ev_ready[s], 0) != hipSuccess) return -2;
            return s;
        }
    return -1;
}
int in_release(gfpl_seqbatch* sb, const gfpl_frames* in, int slot) {
    if (in->consumed) {
        if (hipEventRecord(in->consumed->ev, sb->ctx->stream) != hipSuccess) return GFPL_E_HIP;
        ++in->consumed->records;
    }
    if (slot < 0) return GFPL_OK;
    if (hipEventRecord(sb->ev_free[slot], sb->ctx->stream) != hipSuccess) return GFPL_E_HIP;
    sb->free_recorded[slot] = true;
    return GFPL_OK;
}

int cfg_supported(const gfpl_config& c) {
    if (!c.best_lr_matches || !c.lr_in_parallel || !c.cut_with_max_vol) return GFPL_E_UNSUPPORTED;
    if (c.max_point_match_num < 1 || c.max_point_match_num > GFPL_MAX_MATCHED_PT) return GFPL_E_INVALID;
    if (c.max_line_match_num < 1 || c.max_line_match_num > GFPL_MAX_MATCHED_LS) return GFPL_E_INVALID;
    // the certified cut search needs a margin far above its ~1e-13 error
    if (!(c.cut_certify == 0.0 || (c.cut_certify >= 1e-10 && c.cut_certify < 1.0))) return GFPL_E_INVALID;
    if (c.cut_proof < 0 || c.cut_proof > 3) return GFPL_E_INVALID;
    // the search's ratio keys and their +-s links are formed from a positive finite step
    // (params(): with s <= 0 or NaN no key would exist and the proven search would follow
    // zeroed links); the range must be an ordered finite interval
    if (!(std::isfinite(c.cut_step) && c.cut_step > 0.0)) return GFPL_E_INVALID;
    if (!(std::isfinite(c.cut_rng[0]) && std::isfinite(c.cut_rng[1]) && c.cut_rng[0] <= c.cut_rng[1]))
        return GFPL_E_INVALID;
    return GFPL_OK;
}

void tmark(gfpl_ctx* c, int i) {
    if (c->timing) (void)hipEventRecord(c->ev[i], c->stream);
}

}  // namespace

extern "C" {

int gfpl_create(int device, void* stream, gfpl_ctx** out) {
    if (!out) return GFPL_E_INVALID;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return GFPL_E_NO_DEVICE;
    if (device < 0 || device >= n) return GFPL_E_INVALID;
    HIPCHK(hipSetDevice(device));
    gfpl_ctx* c = new gfpl_ctx();
    c->device = device;
    c->stream = (hipStream_t)stream;
    gfpl_config_default(&c->cfg);
    c->has_cfg = true;
    for (int i = 0; i < GFPL_NEV; ++i)
        if (hipEventCreate(&c->ev[i]) != hipSuccess) { delete c; return GFPL_E_HIP; }
    *out = c;
    return GFPL_OK;
}

int gfpl_create_async(int device, gfpl_ctx** out) {
    if (!out) return GFPL_E_INVALID;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return GFPL_E_NO_DEVICE;
    if (device < 0 || device >= n) return GFPL_E_INVALID;
    HIPCHK(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int e = gfpl_create(device, (void*)s, out);
    if (e) { (void)hipStreamDestroy(s); return e; }
    (*out)->own_stream = true;
    return GFPL_OK;
}

int gfpl_destroy(gfpl_ctx* c) {
    if (!c) return GFPL_E_INVALID;
    if (!c->sbs.empty()) return GFPL_E_STATE;   // its seqbatches use the context's stream and config
    if (c->n_detectors.load() != 0) return GFPL_E_STATE;   // so do its ORB / LBD / LSD objects
    for (int i = 0; i < GFPL_NEV; ++i)
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    if (c->own_stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    delete c;
    return GFPL_OK;
}

void* gfpl_get_stream(const gfpl_ctx* c) { return c ? (void*)c->stream : nullptr; }

int gfpl_event_create(gfpl_ctx* c, gfpl_event** out) {
    if (!c || !out) return GFPL_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    gfpl_event* e = new gfpl_event();
    e->device = c->device;
    if (hipEventCreateWithFlags(&e->ev, hipEventDisableTiming) != hipSuccess) { delete e; return GFPL_E_HIP; }
    *out = e;
    return GFPL_OK;
}

int gfpl_event_destroy(gfpl_event* e) {
    if (!e) return GFPL_E_INVALID;
    (void)hipEventDestroy(e->ev);
    delete e;
    return GFPL_OK;
}

int gfpl_copy_to_host(gfpl_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c || (!dst && bytes) || (!src && bytes)) return GFPL_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (bytes) HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return GFPL_OK;
}

int gfpl_event_record_count(const gfpl_event* e, int64_t* count) {
    if (!e || !count) return GFPL_E_INVALID;
    *count = e->records;
    return GFPL_OK;
}

int gfpl_event_record(gfpl_event* e, gfpl_ctx* c) {
    if (!e || !c || e->device != c->device) return GFPL_E_INVALID;
    HIPCHK(hipEventRecord(e->ev, c->stream));
    ++e->records;
    return GFPL_OK;
}

int gfpl_event_wait(gfpl_ctx* c, gfpl_event* e) {
    if (!e || !c || e->device != c->device) return GFPL_E_INVALID;
    HIPCHK(hipStreamWaitEvent(c->stream, e->ev, 0));
    return GFPL_OK;
}

int gfpl_event_synchronize(gfpl_event* e) {
    if (!e) return GFPL_E_INVALID;
    HIPCHK(hipEventSynchronize(e->ev));
    return GFPL_OK;
}

int gfpl_set_camera(gfpl_ctx* c, const gfpl_camera* cam) {
    if (!c || !cam || cam->n_levels < 1 || cam->n_levels > GFPL_MAX_LEVELS) return GFPL_E_INVALID;
    // seqbatches (their device pyramid builder) and detectors (ORB / LSD geometry) are laid out
    // for the camera they were created on
    if (!c->sbs.empty() || c->n_detectors.load() != 0) return GFPL_E_STATE;
    int64_t need = 0;
    for (int i = 0; i < cam->n_levels; ++i) {
        if (cam->lvl_cols[i] < 1 || cam->lvl_rows[i] < 1 || cam->lvl_offset[i] < 0) return GFPL_E_INVALID;
        // k_stereo_points packs window rows / columns into 11-bit fields
        if (cam->lvl_cols[i] > GFPL_MAX_IMAGE_DIM || cam->lvl_rows[i] > GFPL_MAX_IMAGE_DIM) return GFPL_E_INVALID;
        need = std::max<int64_t>(need, cam->lvl_offset[i] + (int64_t)cam->lvl_cols[i] * cam->lvl_rows[i]);
    }
    if (cam->pyr_bytes < need + GFPL_PYR_TAIL) return GFPL_E_INVALID;   // window loads read past the last row
    if (cam->pyr_bytes % 4 != 0) return GFPL_E_INVALID;                 // every sequence's pyramid dword-aligned
    c->cam = *cam;
    c->has_cam = true;
    return GFPL_OK;
}

int gfpl_set_config(gfpl_ctx* c, const gfpl_config* cfg) {
    if (!c || !cfg) return GFPL_E_INVALID;
    int e = cfg_supported(*cfg);
    if (e) return e;
    // match budgets size the lists of every live seqbatch (gfpl_seqbatch_create):
    // a larger budget would index past them
    for (const gfpl_seqbatch* sb : c->sbs)
        if (cfg->max_point_match_num > sb->mpt_cap || cfg->max_line_match_num > sb->mls_cap) return GFPL_E_CAPACITY;
    c->cfg = *cfg;
    c->has_cfg = true;
    return GFPL_OK;
}

int gfpl_get_camera(const gfpl_ctx* c, gfpl_camera* cam) {
    if (!c || !cam || !c->has_cam) return GFPL_E_INVALID;
    *cam = c->cam;
    return GFPL_OK;
}

int gfpl_get_config(const gfpl_ctx* c, gfpl_config* cfg) {
    if (!c || !cfg) return GFPL_E_INVALID;
    *cfg = c->cfg;
    return GFPL_OK;
}

int gfpl_synchronize(gfpl_ctx* c) {
    if (!c) return GFPL_E_INVALID;
    HIPCHK(hipStreamSynchronize(c->stream));
    return GFPL_OK;
}

int gfpl_seqbatch_create(gfpl_ctx* c, int batch, int kp_cap, int kl_cap, gfpl_seqbatch** out) {
    if (!c || !out || batch < 1 || kp_cap < 2 || kl_cap < 2 || kp_cap > 8192 || kl_cap > 2048 || !c->has_cam)
        return GFPL_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    gfpl_seqbatch* sb = new gfpl_seqbatch();
    sb->ctx = c;
    sb->B = batch;
    sb->kp_cap = (kp_cap + 1) & ~1;
    sb->kl_cap = (kl_cap + 1) & ~1;
    sb->mpt_cap = c->cfg.max_point_match_num;
    sb->mls_cap = c->cfg.max_line_match_num;
    Carver dry;
    carve(dry, sb);
    sb->bytes = (int64_t)dry.off;
    if (hipMalloc(&sb->base, dry.off) != hipSuccess) { delete sb; return GFPL_E_HIP; }
    // GFPL_DEBUG_FILL=<byte> (debug): fill the whole allocation — frame slots, track lists, every
    // scratch field — with that byte instead of zeros (0xFF: NaN doubles, -1 ints), so a read of
    // memory no step wrote changes results (tests/test_gpu_parity.py::test_poisoned_scratch_*)
    if (hipMemsetAsync(sb->base, debug_fill_byte(), dry.off, c->stream) != hipSuccess) { (void)hipFree(sb->base); delete sb; return GFPL_E_HIP; }
    Carver real;
    real.base = (char*)sb->base;
    carve(real, sb);
    if (sb->kp_cap != kp_cap || sb->kl_cap != kl_cap) {   // caps must match the input layout
        (void)hipFree(sb->base); delete sb; return GFPL_E_INVALID;
    }
    c->sbs.push_back(sb);
    *out = sb;
    return GFPL_OK;
}

int gfpl_seqbatch_destroy(gfpl_seqbatch* sb) {
    if (!sb) return GFPL_E_INVALID;
    (void)hipStreamSynchronize(sb->ctx->stream);
    auto& v = sb->ctx->sbs;
    v.erase(std::remove(v.begin(), v.end(), sb), v.end());
    if (sb->copy) (void)hipStreamSynchronize(sb->copy);
    if (sb->base) (void)hipFree(sb->base);
    for (int k = 0; k < 2; ++k) {
        if (sb->stage[k]) (void)hipFree(sb->stage[k]);
        if (sb->ev_ready[k]) (void)hipEventDestroy(sb->ev_ready[k]);
        if (sb->ev_free[k]) (void)hipEventDestroy(sb->ev_free[k]);
    }
    for (hipEvent_t e : sb->ev_ticket)
        if (e) (void)hipEventDestroy(e);
    if (sb->copy) (void)hipStreamDestroy(sb->copy);
    pyrbuild_destroy(sb->pyrb);
    delete sb;
    return GFPL_OK;
}

int64_t gfpl_seqbatch_bytes(const gfpl_seqbatch* sb) { return sb ? sb->bytes : 0; }

int gfpl_initialize(gfpl_seqbatch* sb, const gfpl_frames* in) {
    if (!sb) return GFPL_E_INVALID;
    int e = check_in(sb, in);
    if (e) return e;
    const int slot = in_acquire(sb, in);
    if (slot == -2) return GFPL_E_HIP;
    KParams p = params(sb, in);
    p.curr = sb->slot[sb->prev_slot];   // the initial frame becomes prev_frame
    HIPCHK(launch_init(p, sb->ctx->stream));
    sb->initialized = true;
    sb->has_curr = false;
    return in_release(sb, in, slot);
}

int gfpl_stereo_points(gfpl_seqbatch* sb, const gfpl_frames* in) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized) return GFPL_E_STATE;
    int e = check_in(sb, in);
    if (e) return e;
    const int slot = in_acquire(sb, in);
    if (slot == -2) return GFPL_E_HIP;
    HIPCHK(launch_stereo_points(params(sb, in), sb->ctx->stream));
    sb->has_curr = true;
    return in_release(sb, in, slot);
}

int gfpl_stereo_lines(gfpl_seqbatch* sb, const gfpl_frames* in) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized) return GFPL_E_STATE;
    int e = check_in(sb, in);
    if (e) return e;
    const int slot = in_acquire(sb, in);
    if (slot == -2) return GFPL_E_HIP;
    HIPCHK(launch_stereo_lines(params(sb, in), sb->ctx->stream));
    sb->has_curr = true;
    return in_release(sb, in, slot);
}

int gfpl_line_uncertainty(gfpl_seqbatch* sb) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized) return GFPL_E_STATE;
    HIPCHK(launch_line_uncertainty(params(sb, nullptr), sb->ctx->stream));
    return GFPL_OK;
}

int gfpl_cross_points(gfpl_seqbatch* sb) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    HIPCHK(launch_cross_points(params(sb, nullptr), sb->ctx->stream));
    return GFPL_OK;
}

int gfpl_cross_lines(gfpl_seqbatch* sb) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    HIPCHK(launch_cross_lines(params(sb, nullptr), sb->ctx->stream));
    return GFPL_OK;
}

int gfpl_line_cut(gfpl_seqbatch* sb) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    sb->last_cut_mode = sb->ctx->cfg.cut_proof;
    HIPCHK(launch_line_cut(params(sb, nullptr), sb->ctx->stream, nullptr));
    return GFPL_OK;
}

int gfpl_insert_stereo_pair(gfpl_seqbatch* sb, const gfpl_frames* in) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized) return GFPL_E_STATE;
    int e = check_in(sb, in);
    if (e) return e;
    gfpl_ctx* c = sb->ctx;
    const int slot = in_acquire(sb, in);
    if (slot == -2) return GFPL_E_HIP;
    KParams p = params(sb, in);
    tmark(c, 0);
    HIPCHK(launch_stereo_points(p, c->stream));
    tmark(c, 1);
    HIPCHK(launch_stereo_lines(p, c->stream));
    tmark(c, 2);
    // predictFramePose is fused into cross_points (src/stereoFrameHandler.cpp:100)
    if (c->cfg.use_line_conf_cut) HIPCHK(launch_line_uncertainty(p, c->stream));   // :103-106
    HIPCHK(launch_cross_points(p, c->stream));
    tmark(c, 3);
    HIPCHK(launch_cross_lines(p, c->stream));
    tmark(c, 4);
    sb->last_cut_mode = c->cfg.use_line_conf_cut ? c->cfg.cut_proof : -1;
    if (c->cfg.use_line_conf_cut)
        HIPCHK(launch_line_cut(p, c->stream, c->timing ? &c->ev[7] : nullptr));
    HIPCHK(launch_step_bytes(p, c->stream));
    tmark(c, 5);
    sb->has_curr = true;
    return in_release(sb, in, slot);
}

int gfpl_optimize_pose(gfpl_seqbatch* sb) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    HIPCHK(launch_pose(params(sb, nullptr), sb->ctx->stream, sb->ctx->timing ? sb->ctx->ev[9] : nullptr));
    tmark(sb->ctx, 6);
    return GFPL_OK;
}

int gfpl_need_new_kf(gfpl_seqbatch* sb, int32_t* flags) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    HIPCHK(launch_need_kf(params(sb, nullptr), sb->ctx->stream));
    if (flags) {
        HIPCHK(hipMemcpyAsync(flags, sb->tr.kf_flag, sizeof(int32_t) * (size_t)sb->B, hipMemcpyDeviceToHost,
                              sb->ctx->stream));
        HIPCHK(hipStreamSynchronize(sb->ctx->stream));
    }
    return GFPL_OK;
}

int gfpl_curr_frame_is_kf(gfpl_seqbatch* sb, const int32_t* mask) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    const int32_t* dmask = sb->tr.kf_flag;   // NULL: the last needNewKF decisions
    if (mask) {
        HIPCHK(hipMemcpyAsync(sb->scr.kf_mask, mask, sizeof(int32_t) * (size_t)sb->B, hipMemcpyHostToDevice,
                              sb->ctx->stream));
        dmask = sb->scr.kf_mask;
    }
    HIPCHK(launch_curr_frame_is_kf(params(sb, nullptr), dmask, sb->ctx->stream));
    if (mask) HIPCHK(hipStreamSynchronize(sb->ctx->stream));   // the caller's mask may be reused on return
    return GFPL_OK;
}

int gfpl_read_kf_state(gfpl_seqbatch* sb, int seq, gfpl_kf_state* out) {
    if (!sb || !out || seq < 0 || seq >= sb->B) return GFPL_E_INVALID;
    hipStream_t s = sb->ctx->stream;
    const DevTrack& T = sb->tr;
    HIPCHK(hipMemcpyAsync(out->T_prevKF, T.kf_T + 16 * (size_t)seq, sizeof(double) * 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out->cov_prevKF_currF, T.kf_cov + 36 * (size_t)seq, sizeof(double) * 36,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&out->entropy_first_prevKF, T.kf_entropy0 + seq, sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&out->entropy_ratio, T.kf_ratio + seq, sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&out->prev_f_iskf, T.kf_prev_iskf + seq, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&out->num_frame_since_kf, T.kf_nsince + seq, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&out->need_new_kf, T.kf_flag + seq, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return GFPL_OK;
}

int gfpl_optimize_pose_ini(gfpl_seqbatch* sb, const double* dt_ini) {
    if (!sb) return GFPL_E_INVALID;
    if (!dt_ini) return gfpl_optimize_pose(sb);
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    HIPCHK(hipMemcpyAsync(sb->scr.pose_dtini, dt_ini, sizeof(double) * 16 * (size_t)sb->B, hipMemcpyHostToDevice,
                          sb->ctx->stream));
    KParams p = params(sb, nullptr);
    p.dt_ini = sb->scr.pose_dtini;
    HIPCHK(launch_pose(p, sb->ctx->stream, sb->ctx->timing ? sb->ctx->ev[9] : nullptr));
    tmark(sb->ctx, 6);
    HIPCHK(hipStreamSynchronize(sb->ctx->stream));   // the caller's buffer may be reused on return
    return GFPL_OK;
}

}  // extern "C"

namespace {
// device layout of one staged input batch of B sequences (the gfpl_frames [B][cap] layout)
void stage_layout(Carver& c, const gfpl_seqbatch* sb, gfpl_frames& f) {
    const size_t B = sb->B, P = B * sb->kp_cap, L = B * sb->kl_cap;
    const size_t pyr = B * (size_t)sb->ctx->cam.pyr_bytes;
    f.batch = sb->B; f.kp_cap = sb->kp_cap; f.kl_cap = sb->kl_cap;
    f.n_kp_l = c.take<int>(B); f.n_kp_r = c.take<int>(B);
    f.kp_l = c.take<gfpl_keypoint>(P); f.kp_r = c.take<gfpl_keypoint>(P);
    f.pdesc_l = c.take<uint8_t>(P * 32); f.pdesc_r = c.take<uint8_t>(P * 32);
    f.n_kl_l = c.take<int>(B); f.n_kl_r = c.take<int>(B);
    f.kl_l = c.take<gfpl_keyline>(L); f.kl_r = c.take<gfpl_keyline>(L);
    f.ldesc_l = c.take<uint8_t>(L * 32); f.ldesc_r = c.take<uint8_t>(L * 32);
    f.pyr_r = c.take<uint8_t>(pyr); f.time_stamp = c.take<double>(B);
}

int stage_alloc(gfpl_seqbatch* sb, int slot) {
    if (!sb->copy) {
        HIPCHK(hipStreamCreateWithFlags(&sb->copy, hipStreamNonBlocking));
        for (int k = 0; k < 2; ++k) {
            HIPCHK(hipEventCreateWithFlags(&sb->ev_ready[k], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&sb->ev_free[k], hipEventDisableTiming));
        }
        for (hipEvent_t& e : sb->ev_ticket) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (sb->stage[slot]) return GFPL_OK;
    Carver c;
    gfpl_frames f{};
    stage_layout(c, sb, f);   // sizing pass (base == nullptr)
    HIPCHK(hipMalloc(&sb->stage[slot], c.off));
    // (debug fill: on the copy stream, ahead of the uploads — hipMemset is asynchronous to the host and
    // the non-blocking copy stream does not wait for the null stream)
    if (const int fill = debug_fill_byte()) HIPCHK(hipMemsetAsync(sb->stage[slot], fill, c.off, sb->copy));
    sb->stage_bytes[slot] = c.off;
    c.off = 0;
    c.base = (char*)sb->stage[slot];
    stage_layout(c, sb, sb->stage_view[slot]);
    return GFPL_OK;
}
}  // namespace

extern "C" {

namespace {
// both upload forms; l0_stride > 0: host->pyr_r holds level-0 images l0_stride bytes apart and the
// device builds levels 1.. (ORB resize) on the copy stream after the copy
int upload_async(gfpl_seqbatch* sb, const gfpl_frames* host, int s0, int slot, int64_t l0_stride, int64_t* ticket);
}  // namespace

int gfpl_upload_frames_async(gfpl_seqbatch* sb, const gfpl_frames* host, int s0, int slot, int64_t* ticket) {
    return upload_async(sb, host, s0, slot, 0, ticket);
}

int gfpl_upload_frames_l0_async(gfpl_seqbatch* sb, const gfpl_frames* host, int s0, int slot, int64_t l0_stride,
                                int64_t* ticket) {
    if (!sb || !sb->ctx->has_cam) return GFPL_E_INVALID;
    const gfpl_camera& cam = sb->ctx->cam;
    if (l0_stride < (int64_t)cam.lvl_cols[0] * cam.lvl_rows[0]) return GFPL_E_INVALID;
    if (!sb->pyrb) {
        HIPCHK(hipSetDevice(sb->ctx->device));
        const int e = pyrbuild_create(&cam, &sb->pyrb);
        if (e) return e;
    }
    return upload_async(sb, host, s0, slot, l0_stride, ticket);
}

}  // extern "C"

namespace {
int upload_async(gfpl_seqbatch* sb, const gfpl_frames* host, int s0, int slot, int64_t l0_stride, int64_t* ticket) {
    if (!sb || !host || (slot != 0 && slot != 1) || !sb->ctx->has_cam) return GFPL_E_INVALID;
    const int n = host->batch;
    if (n < 1 || s0 < 0 || s0 + n > sb->B || host->kp_cap != sb->kp_cap || host->kl_cap != sb->kl_cap)
        return GFPL_E_INVALID;
    if (!host->n_kp_l || !host->n_kp_r || !host->kp_l || !host->kp_r || !host->pdesc_l || !host->pdesc_r ||
        !host->n_kl_l || !host->n_kl_r || !host->kl_l || !host->kl_r || !host->ldesc_l || !host->ldesc_r ||
        !host->pyr_r || !host->time_stamp)
        return GFPL_E_INVALID;
    int e = stage_alloc(sb, slot);
    if (e) return e;
    const gfpl_frames& d = sb->stage_view[slot];
    hipStream_t s = sb->copy;
    if (sb->free_recorded[slot]) HIPCHK(hipStreamWaitEvent(s, sb->ev_free[slot], 0));
    const size_t N = n, P = N * sb->kp_cap, L = N * sb->kl_cap, S = s0;
    const size_t kp0 = S * sb->kp_cap, kl0 = S * sb->kl_cap, pyr = (size_t)sb->ctx->cam.pyr_bytes;
#define UP(field, off, cnt) \
    HIPCHK(hipMemcpyAsync((void*)(d.field + (off)), host->field, sizeof(*d.field) * (cnt), hipMemcpyHostToDevice, s))
    UP(n_kp_l, S, N); UP(n_kp_r, S, N); UP(kp_l, kp0, P); UP(kp_r, kp0, P);
    UP(pdesc_l, kp0 * 32, P * 32); UP(pdesc_r, kp0 * 32, P * 32);
    UP(n_kl_l, S, N); UP(n_kl_r, S, N); UP(kl_l, kl0, L); UP(kl_r, kl0, L);
    UP(ldesc_l, kl0 * 32, L * 32); UP(ldesc_r, kl0 * 32, L * 32);
    UP(time_stamp, S, N);
    if (l0_stride > 0) {
        const gfpl_camera& cam = sb->ctx->cam;
        const size_t l0 = (size_t)cam.lvl_cols[0] * cam.lvl_rows[0];
        uint8_t* dst = const_cast<uint8_t*>(d.pyr_r) + S * pyr;
        HIPCHK(hipMemcpy2DAsync(dst, pyr, host->pyr_r, (size_t)l0_stride, l0, N, hipMemcpyHostToDevice, s));
        HIPCHK(pyrbuild_run(sb->pyrb, dst, (long long)pyr, n, s));
    } else {
        UP(pyr_r, S * pyr, N * pyr);
    }
#undef UP
    HIPCHK(hipEventRecord(sb->ev_ready[slot], s));
    sb->ready_pending[slot] = true;
    const int64_t t = sb->n_tickets++;
    HIPCHK(hipEventRecord(sb->ev_ticket[t % 16], s));
    if (ticket) *ticket = t;
    return GFPL_OK;
}
}  // namespace

extern "C" {

int gfpl_upload_wait(gfpl_seqbatch* sb, int64_t ticket) {
    if (!sb || ticket < 0 || ticket >= sb->n_tickets) return GFPL_E_INVALID;
    // the event may since have been re-recorded by a newer copy on the same in-order stream:
    // waiting for that one is later than needed, never earlier
    HIPCHK(hipEventSynchronize(sb->ev_ticket[ticket % 16]));
    return GFPL_OK;
}

int gfpl_staged_frames(gfpl_seqbatch* sb, int slot, gfpl_frames* dev) {
    if (!sb || !dev || (slot != 0 && slot != 1) || !sb->stage[slot]) return GFPL_E_INVALID;
    *dev = sb->stage_view[slot];
    return GFPL_OK;
}

int gfpl_upload_frames(gfpl_seqbatch* sb, const gfpl_frames* host, gfpl_frames* dev) {
    if (!sb || !host || !dev) return GFPL_E_INVALID;
    if (host->batch != sb->B) return GFPL_E_INVALID;
    int64_t t = 0;
    int e = gfpl_upload_frames_async(sb, host, 0, 0, &t);
    if (e) return e;
    e = gfpl_upload_wait(sb, t);
    if (e) return e;
    *dev = sb->stage_view[0];
    return GFPL_OK;
}

int gfpl_update_frame(gfpl_seqbatch* sb) {
    if (!sb) return GFPL_E_INVALID;
    if (!sb->initialized || !sb->has_curr) return GFPL_E_STATE;
    // the cleared lists stay readable until the next insert (gfpl_read_last_track)
    HIPCHK(hipMemcpyAsync(sb->last_n_pt, sb->tr.n_matched_pt, sizeof(int32_t) * sb->B, hipMemcpyDeviceToDevice,
                          sb->ctx->stream));
    HIPCHK(hipMemcpyAsync(sb->last_n_ls, sb->tr.n_matched_ls, sizeof(int32_t) * sb->B, hipMemcpyDeviceToDevice,
                          sb->ctx->stream));
    // matched_pt.clear(); matched_ls.clear() (src/stereoFrameHandler.cpp:889-890)
    HIPCHK(hipMemsetAsync(sb->tr.n_matched_pt, 0, sizeof(int32_t) * sb->B, sb->ctx->stream));
    HIPCHK(hipMemsetAsync(sb->tr.n_matched_ls, 0, sizeof(int32_t) * sb->B, sb->ctx->stream));
    sb->prev_slot = 1 - sb->prev_slot;
    sb->has_curr = false;
    return GFPL_OK;
}

int gfpl_frame_step(gfpl_seqbatch* sb, const gfpl_frames* in) {
    int e = gfpl_insert_stereo_pair(sb, in);
    if (e) return e;
    e = gfpl_optimize_pose(sb);
    if (e) return e;
    return gfpl_update_frame(sb);
}

int gfpl_knn2_hamming(gfpl_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, int32_t* idx,
                      float* dist) {
    if (!c || !q || !t || !idx || !dist || nq < 0 || (cell != 1 && cell != 2)) return GFPL_E_INVALID;
    if (nt < 2) return GFPL_E_TOO_FEW_TRAIN;
    if (nq == 0) return GFPL_OK;
    HIPCHK(launch_knn2(q, nq, t, nt, cell, idx, dist, c->stream));
    return GFPL_OK;
}

// ------------------------------------------------- host-facing matchers --
// StereoFrame's matcher members as MapHandler calls them: host buffers in and out, one device
// scratch per call (keyframe rate), serialised per context (two std::async tasks share it).
namespace {
struct Scratch {
    char* p = nullptr;
    ~Scratch() { if (p) (void)hipFree(p); }
};
}  // namespace

int gfpl_knn2_hamming_host(gfpl_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, int32_t* idx,
                           float* dist) {
    if (!c || !q || !t || !idx || !dist || nq < 0 || (cell != 1 && cell != 2)) return GFPL_E_INVALID;
    if (nt < 2) return GFPL_E_TOO_FEW_TRAIN;
    if (nq == 0) return GFPL_OK;
    std::lock_guard<std::mutex> lk(c->host_mu);
    HIPCHK(hipSetDevice(c->device));
    const size_t bq = 32 * (size_t)nq, bt = 32 * (size_t)nt, bo = 2 * (size_t)nq * 4;
    Scratch s;
    HIPCHK(hipMalloc(&s.p, bq + bt + 2 * bo + 64));
    uint8_t* dq = reinterpret_cast<uint8_t*>(s.p);
    uint8_t* dt = dq + bq;
    int32_t* di = reinterpret_cast<int32_t*>(dt + bt);
    float* dd = reinterpret_cast<float*>(di + 2 * (size_t)nq);
    HIPCHK(hipMemcpyAsync(dq, q, bq, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(dt, t, bt, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_knn2(dq, nq, dt, nt, cell, di, dd, c->stream));
    HIPCHK(hipMemcpyAsync(idx, di, bo, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(dist, dd, bo, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GFPL_OK;
}

int gfpl_radius_hamming(gfpl_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, float max_dist,
                        int32_t* row_off, int cap, int32_t* idx, float* dist) {
    if (!c || (!q && nq) || (!t && nt) || !row_off || nq < 0 || nt < 0 || cap < 0 || (cell != 1 && cell != 2) ||
        max_dist != max_dist)
        return GFPL_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    std::vector<int32_t> h(nq + 1, 0);
    if (nq > 0 && nt > 0) {
        HIPCHK(launch_radius_count(q, nq, t, nt, cell, max_dist, row_off + 1, c->stream));
        HIPCHK(hipMemcpyAsync(h.data() + 1, row_off + 1, 4 * (size_t)nq, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    for (int i = 0; i < nq; ++i) h[i + 1] += h[i];
    HIPCHK(hipMemcpyAsync(row_off, h.data(), 4 * (size_t)(nq + 1), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));   // (h is pageable stack memory)
    if (h[nq] > cap) return GFPL_E_CAPACITY;
    if (h[nq] > 0) {
        if (!idx || !dist) return GFPL_E_INVALID;
        HIPCHK(launch_radius_rows(q, nq, t, nt, cell, max_dist, row_off, idx, dist, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return GFPL_OK;
}

int gfpl_radius_hamming_host(gfpl_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, float max_dist,
                             int32_t* row_off, int cap, int32_t* idx, float* dist) {
    if (!c || (!q && nq) || (!t && nt) || !row_off || nq < 0 || nt < 0 || cap < 0 || (cell != 1 && cell != 2) ||
        max_dist != max_dist)
        return GFPL_E_INVALID;
    std::lock_guard<std::mutex> lk(c->host_mu);
    HIPCHK(hipSetDevice(c->device));
    const size_t bq = 32 * (size_t)nq, bt = 32 * (size_t)nt, bo = 4 * ((size_t)nq + 1);
    Scratch s;
    HIPCHK(hipMalloc(&s.p, bq + bt + bo + 64));
    uint8_t* dq = reinterpret_cast<uint8_t*>(s.p);
    uint8_t* dt = dq + bq;
    int32_t* dro = reinterpret_cast<int32_t*>(dt + bt + (16 - (bq + bt) % 16) % 16);
    if (bq) HIPCHK(hipMemcpyAsync(dq, q, bq, hipMemcpyHostToDevice, c->stream));
    if (bt) HIPCHK(hipMemcpyAsync(dt, t, bt, hipMemcpyHostToDevice, c->stream));
    // sizes first (rows are ragged), then the rows into a scratch of exactly that size
    int e = gfpl_radius_hamming(c, dq, nq, dt, nt, cell, max_dist, dro, 0, nullptr, nullptr);
    if (e != GFPL_OK && e != GFPL_E_CAPACITY) return e;
    HIPCHK(hipMemcpy(row_off, dro, bo, hipMemcpyDeviceToHost));
    const int total = row_off[nq];
    if (total > cap) return GFPL_E_CAPACITY;
    if (total == 0) return GFPL_OK;
    if (!idx || !dist) return GFPL_E_INVALID;
    Scratch r;
    HIPCHK(hipMalloc(&r.p, 8 * (size_t)total + 64));
    int32_t* ri = reinterpret_cast<int32_t*>(r.p);
    float* rd = reinterpret_cast<float*>(ri + total);
    HIPCHK(launch_radius_rows(dq, nq, dt, nt, cell, max_dist, dro, ri, rd, c->stream));
    HIPCHK(hipMemcpyAsync(idx, ri, 4 * (size_t)total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(dist, rd, 4 * (size_t)total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GFPL_OK;
}

int gfpl_match_stats_host(gfpl_ctx* c, int kind, const float* d0, const float* d1, int n, int max_num, double* out) {
    if (!c || !d0 || !d1 || !out || n < 1 || max_num < 1 || (kind != 0 && kind != 1)) return GFPL_E_INVALID;
    std::lock_guard<std::mutex> lk(c->host_mu);
    HIPCHK(hipSetDevice(c->device));
    Scratch s;
    HIPCHK(hipMalloc(&s.p, 8 * (size_t)n + 64));
    float* a = reinterpret_cast<float*>(s.p);
    float* b = a + n;
    double* o = reinterpret_cast<double*>(s.p + ((8 * (size_t)n + 7) & ~(size_t)7));
    HIPCHK(hipMemcpyAsync(a, d0, 4 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b, d1, 4 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_match_stats(kind, a, b, n, max_num, o, c->stream));
    HIPCHK(hipMemcpyAsync(out, o, 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GFPL_OK;
}

// MapHandler::lookForCommonMatches keyframe-pair stage (src/mapHandler.cpp:199-470):
// per kind two knn-2 launches (the MFMA k_knn2m of gfpl_knn2_hamming) and one gate
// launch (k_kf.hip); keyframe rate, so the scratch is allocated per call.
int gfpl_kf_common_matches(gfpl_ctx* c, const gfpl_kf_view* k0, const gfpl_kf_view* k1, int32_t* pt_pairs,
                           int* n_pt_pairs, int32_t* ls_pairs, int* n_ls_pairs) {
    if (!c || !k0 || !k1 || !n_pt_pairs || !n_ls_pairs || !c->has_cam) return GFPL_E_INVALID;
    if (k0->n_pt < 0 || k1->n_pt < 0 || k0->n_ls < 0 || k1->n_ls < 0) return GFPL_E_INVALID;
    *n_pt_pairs = 0;
    *n_ls_pairs = 0;
    const bool do_pt = k0->n_pt >= 2 && k1->n_pt >= 2;   // ledger U4
    const bool do_ls = k0->n_ls >= 2 && k1->n_ls >= 2;
    if (do_pt && (!pt_pairs || !k0->pdesc || !k1->pdesc || !k0->P || !k0->pt_sigma2 || !k1->pl))
        return GFPL_E_INVALID;
    if (do_ls && (!ls_pairs || !k0->ldesc || !k1->ldesc || !k0->sP || !k0->eP || !k0->le || !k0->ls_sigma2))
        return GFPL_E_INVALID;
    if (!do_pt && !do_ls) return GFPL_OK;
    const size_t npt = do_pt ? (size_t)k0->n_pt + k1->n_pt : 0, nls = do_ls ? (size_t)k0->n_ls + k1->n_ls : 0;
    const size_t bytes = 2 * (npt + nls) * (sizeof(int32_t) + sizeof(float)) + 64;
    char* scr = nullptr;
    HIPCHK(hipMalloc(&scr, bytes));
    int32_t* idx = reinterpret_cast<int32_t*>(scr);
    float* dist = reinterpret_cast<float*>(idx + 2 * (npt + nls));
    int* cnt = reinterpret_cast<int*>(dist + 2 * (npt + nls));
    hipError_t e = hipSuccess;
    gfpl::KfGate g;
    std::memset(&g, 0, sizeof g);
    g.cam = devcam(c->cam);
    for (int i = 0; i < 16; ++i) { g.T0[i] = k0->T_kf_w[i]; g.T1[i] = k1->T_kf_w[i]; }
    g.max_ratio_12_p = c->cfg.max_ratio_12_p;
    g.desc_th_l = c->cfg.desc_th_l;
    int counts[2] = {0, 0};
    size_t o = 0;
    for (int kind = 0; kind < 2 && e == hipSuccess; ++kind) {
        if (kind == 0 ? !do_pt : !do_ls) continue;
        const int n0 = kind == 0 ? k0->n_pt : k0->n_ls, n1 = kind == 0 ? k1->n_pt : k1->n_ls;
        const uint8_t* d0 = kind == 0 ? k0->pdesc : k0->ldesc;
        const uint8_t* d1 = kind == 0 ? k1->pdesc : k1->ldesc;
        int32_t* i12 = idx + 2 * o;
        float* f12 = dist + 2 * o;
        int32_t* i21 = i12 + 2 * n0;
        float* f21 = f12 + 2 * n0;
        o += (size_t)n0 + n1;
        e = launch_knn2(d0, n0, d1, n1, 1, i12, f12, c->stream);   // NORM_HAMMING (:213 / :343)
        if (e == hipSuccess) e = launch_knn2(d1, n1, d0, n0, 1, i21, f21, c->stream);
        g.lines = kind;
        g.n0 = n0;
        g.i12 = i12; g.d12 = f12; g.i21 = i21;
        g.p_stride = 3;
        g.P0 = kind == 0 ? k0->P : k0->sP;
        g.eP0 = kind == 0 ? nullptr : k0->eP;
        g.le0 = kind == 0 ? nullptr : k0->le;
        g.sigma2_0 = kind == 0 ? k0->pt_sigma2 : k0->ls_sigma2;
        g.pl1 = kind == 0 ? k1->pl : nullptr;
        g.pairs = kind == 0 ? pt_pairs : ls_pairs;
        g.count = cnt + kind;
        if (e == hipSuccess) e = launch_kf_gate(g, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(counts + kind, cnt + kind, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipError_t ef = hipFree(scr);
    if (e != hipSuccess || ef != hipSuccess) return GFPL_E_HIP;
    *n_pt_pairs = counts[0];
    *n_ls_pairs = counts[1];
    return GFPL_OK;
}

// lookForCommonMatches local-map stage (src/mapHandler.cpp:472-772): per kind one
// filter launch (in-view local rows, compacted with their descriptors), the two
// knn-2 launches on the compacted rows and the gate launch (k_kf.hip).
int gfpl_kf_local_map_matches(gfpl_ctx* c, const gfpl_map_view* m, const gfpl_kf_view* k1, double max_kf_epip_p,
                              double max_kf_epip_l, int32_t* pt_pairs, int* n_pt_pairs, int32_t* ls_pairs,
                              int* n_ls_pairs) {
    if (!c || !m || !k1 || !n_pt_pairs || !n_ls_pairs || !c->has_cam) return GFPL_E_INVALID;
    if (m->n_pt < 0 || m->n_ls < 0 || k1->n_pt < 0 || k1->n_ls < 0) return GFPL_E_INVALID;
    *n_pt_pairs = 0;
    *n_ls_pairs = 0;
    const bool do_pt = m->n_pt >= 2 && k1->n_pt >= 2, do_ls = m->n_ls >= 2 && k1->n_ls >= 2;
    if (do_pt && (!pt_pairs || !m->pdesc || !m->P || !k1->pdesc || !k1->pl)) return GFPL_E_INVALID;
    if (do_ls && (!ls_pairs || !m->ldesc || !m->L || !k1->ldesc || !k1->le)) return GFPL_E_INVALID;
    if (!do_pt && !do_ls) return GFPL_OK;
    const size_t n0 = (size_t)(do_pt ? m->n_pt : 0) + (do_ls ? m->n_ls : 0);
    const size_t n1 = (size_t)(do_pt ? k1->n_pt : 0) + (do_ls ? k1->n_ls : 0);
    // loc [n0] | descs [n0][32] | idx [2 (n0 + n1)] | dist [2 (n0 + n1)] | counts [4]
    const size_t bytes = n0 * 4 + n0 * 32 + 2 * (n0 + n1) * 8 + 64;
    char* scr = nullptr;
    HIPCHK(hipMalloc(&scr, bytes));
    int32_t* loc = reinterpret_cast<int32_t*>(scr);
    uint8_t* dsc = reinterpret_cast<uint8_t*>(loc + n0);
    int32_t* idx = reinterpret_cast<int32_t*>(dsc + n0 * 32);
    float* dist = reinterpret_cast<float*>(idx + 2 * (n0 + n1));
    int* cnt = reinterpret_cast<int*>(dist + 2 * (n0 + n1));
    const DevCam cam = devcam(c->cam);
    hipError_t e = hipSuccess;
    int nloc[2] = {0, 0};
    size_t o0 = 0;
    size_t lo[2] = {0, 0};
    for (int kind = 0; kind < 2 && e == hipSuccess; ++kind) {
        if (kind == 0 ? !do_pt : !do_ls) continue;
        lo[kind] = o0;
        const int n = kind == 0 ? m->n_pt : m->n_ls;
        e = launch_kf_map_filter(cam, k1->T_kf_w, kind == 0 ? m->P : m->L, n, kind, loc + o0, dsc + 32 * o0,
                                 kind == 0 ? m->pdesc : m->ldesc, cnt + kind, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(nloc + kind, cnt + kind, sizeof(int), hipMemcpyDeviceToHost, c->stream);
        o0 += n;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    gfpl::KfGate g;
    std::memset(&g, 0, sizeof g);
    g.cam = cam;
    for (int i = 0; i < 16; ++i) g.T1[i] = k1->T_kf_w[i];
    g.max_ratio_12_p = c->cfg.max_ratio_12_p;
    g.desc_th_l = c->cfg.desc_th_l;
    g.map = 1;
    g.epip_p = max_kf_epip_p;
    g.epip_l = max_kf_epip_l;
    int counts[2] = {0, 0};
    size_t o = 0;
    for (int kind = 0; kind < 2 && e == hipSuccess; ++kind) {
        if (kind == 0 ? !do_pt : !do_ls) continue;
        const int nq = nloc[kind], nt = kind == 0 ? k1->n_pt : k1->n_ls;
        if (nq < 2) continue;   // ledger U4 on the selected local rows
        const uint8_t* d0 = dsc + 32 * lo[kind];
        const uint8_t* d1 = kind == 0 ? k1->pdesc : k1->ldesc;
        int32_t* i12 = idx + 2 * o;
        float* f12 = dist + 2 * o;
        int32_t* i21 = i12 + 2 * (size_t)nq;
        float* f21 = f12 + 2 * (size_t)nq;
        o += (size_t)nq + nt;
        e = launch_knn2(d0, nq, d1, nt, 1, i12, f12, c->stream);
        if (e == hipSuccess) e = launch_knn2(d1, nt, d0, nq, 1, i21, f21, c->stream);
        g.lines = kind;
        g.n0 = nq;
        g.loc = loc + lo[kind];
        g.i12 = i12; g.d12 = f12; g.i21 = i21;
        g.P0 = kind == 0 ? m->P : m->L;
        g.eP0 = kind == 0 ? nullptr : m->L + 3;
        g.p_stride = kind == 0 ? 3 : 6;
        g.pl1 = kind == 0 ? k1->pl : nullptr;
        g.le1 = kind == 0 ? nullptr : k1->le;
        g.pairs = kind == 0 ? pt_pairs : ls_pairs;
        g.count = cnt + 2 + kind;
        if (e == hipSuccess) e = launch_kf_gate(g, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(counts + kind, cnt + 2 + kind, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipError_t ef = hipFree(scr);
    if (e != hipSuccess || ef != hipSuccess) return GFPL_E_HIP;
    *n_pt_pairs = counts[0];
    *n_ls_pairs = counts[1];
    return GFPL_OK;
}

}  // extern "C"

// ------------------------------------------------------------ transfer --
namespace {
template <typename T>
hipError_t d2h(T* dst, const T* src, size_t n, hipStream_t s) {
    if (!dst || n == 0) return hipSuccess;
    return hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyDeviceToHost, s);
}
template <typename T>
hipError_t h2d(T* dst, const T* src, size_t n, hipStream_t s) {
    if (!src || n == 0) return hipSuccess;
    return hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, s);
}
}  // namespace

extern "C" {

#define XFER(fn, a, b, n) HIPCHK(fn(a, b, n, s))

int gfpl_read_frame(gfpl_seqbatch* sb, int which, int seq, gfpl_frame_host* o) {
    if (!sb || !o || seq < 0 || seq >= sb->B || (which != GFPL_PREV && which != GFPL_CURR)) return GFPL_E_INVALID;
    hipStream_t s = sb->ctx->stream;
    const DevFrame& f = sb->slot[which == GFPL_PREV ? sb->prev_slot : 1 - sb->prev_slot];
    HIPCHK(hipStreamSynchronize(s));
    int np = 0, nl = 0;
    HIPCHK(hipMemcpy(&np, f.pt.n + seq, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&nl, f.ls.n + seq, 4, hipMemcpyDeviceToHost));
    o->n_pt = np; o->n_ls = nl;
    const size_t P = (size_t)seq * sb->kp_cap, L = (size_t)seq * sb->kl_cap;
    XFER(d2h, o->pt_pl, f.pt.pl + 2 * P, 2 * (size_t)np);
    XFER(d2h, o->pt_pl_obs, f.pt.pl_obs + 2 * P, 2 * (size_t)np);
    XFER(d2h, o->pt_disp, f.pt.disp + P, (size_t)np);
    XFER(d2h, o->pt_P, f.pt.P + 3 * P, 3 * (size_t)np);
    XFER(d2h, o->pt_sigma2, f.pt.sigma2 + P, (size_t)np);
    XFER(d2h, o->pt_idx, f.pt.idx + P, (size_t)np);
    XFER(d2h, o->pt_level, f.pt.level + P, (size_t)np);
    XFER(d2h, o->pt_inlier, f.pt.inlier + P, (size_t)np);
    XFER(d2h, o->pdesc, f.pt.desc + 32 * P, 32 * (size_t)np);
    XFER(d2h, o->ls_spl, f.ls.spl + 2 * L, 2 * (size_t)nl);
    XFER(d2h, o->ls_epl, f.ls.epl + 2 * L, 2 * (size_t)nl);
    XFER(d2h, o->ls_spl_obs, f.ls.spl_obs + 2 * L, 2 * (size_t)nl);
    XFER(d2h, o->ls_epl_obs, f.ls.epl_obs + 2 * L, 2 * (size_t)nl);
    XFER(d2h, o->ls_sdisp, f.ls.sdisp + L, (size_t)nl);
    XFER(d2h, o->ls_edisp, f.ls.edisp + L, (size_t)nl);
    XFER(d2h, o->ls_sdisp_obs, f.ls.sdisp_obs + L, (size_t)nl);
    XFER(d2h, o->ls_edisp_obs, f.ls.edisp_obs + L, (size_t)nl);
    XFER(d2h, o->ls_angle, f.ls.angle + L, (size_t)nl);
    XFER(d2h, o->ls_sigma2, f.ls.sigma2 + L, (size_t)nl);
    XFER(d2h, o->ls_sP, f.ls.sP + 3 * L, 3 * (size_t)nl);
    XFER(d2h, o->ls_eP, f.ls.eP + 3 * L, 3 * (size_t)nl);
    XFER(d2h, o->ls_le, f.ls.le + 3 * L, 3 * (size_t)nl);
    XFER(d2h, o->ls_le_obs, f.ls.le_obs + 3 * L, 3 * (size_t)nl);
    XFER(d2h, o->ls_covS, f.ls.covS + 9 * L, 9 * (size_t)nl);
    XFER(d2h, o->ls_covE, f.ls.covE + 9 * L, 9 * (size_t)nl);
    XFER(d2h, o->ls_cut, f.ls.cut + 2 * L, 2 * (size_t)nl);
    XFER(d2h, o->ls_invcov, f.ls.invcov + 36 * L, 36 * (size_t)nl);
    XFER(d2h, o->ls_idx, f.ls.idx + L, (size_t)nl);
    XFER(d2h, o->ls_level, f.ls.level + L, (size_t)nl);
    XFER(d2h, o->ls_inlier, f.ls.inlier + L, (size_t)nl);
    XFER(d2h, o->ldesc, f.ls.desc + 32 * L, 32 * (size_t)nl);
    XFER(d2h, o->Tfw, f.pose.Tfw + 16 * seq, 16);
    XFER(d2h, o->DT, f.pose.DT + 16 * seq, 16);
    XFER(d2h, o->DT_cov, f.pose.DT_cov + 36 * seq, 36);
    XFER(d2h, o->Tfw_cov, f.pose.Tfw_cov + 36 * seq, 36);
    XFER(d2h, o->DT_cov_eig, f.pose.DT_cov_eig + 6 * seq, 6);
    XFER(d2h, &o->err_norm, f.pose.err_norm + seq, 1);
    XFER(d2h, &o->time_stamp, f.pose.time_stamp + seq, 1);
    HIPCHK(hipStreamSynchronize(s));
    return GFPL_OK;
}

int gfpl_write_frame(gfpl_seqbatch* sb, int which, int seq, const gfpl_frame_host* o) {
    if (!sb || !o || seq < 0 || seq >= sb->B || (which != GFPL_PREV && which != GFPL_CURR)) return GFPL_E_INVALID;
    if (o->n_pt < 0 || o->n_pt > sb->kp_cap || o->n_ls < 0 || o->n_ls > sb->kl_cap) return GFPL_E_CAPACITY;
    hipStream_t s = sb->ctx->stream;
    DevFrame& f = sb->slot[which == GFPL_PREV ? sb->prev_slot : 1 - sb->prev_slot];
    const int np = o->n_pt, nl = o->n_ls;
    const size_t P = (size_t)seq * sb->kp_cap, L = (size_t)seq * sb->kl_cap;
    XFER(h2d, f.pt.n + seq, &o->n_pt, 1);
    XFER(h2d, f.ls.n + seq, &o->n_ls, 1);
    XFER(h2d, f.pt.pl + 2 * P, o->pt_pl, 2 * (size_t)np);
    XFER(h2d, f.pt.pl_obs + 2 * P, o->pt_pl_obs, 2 * (size_t)np);
    XFER(h2d, f.pt.disp + P, o->pt_disp, (size_t)np);
    XFER(h2d, f.pt.P + 3 * P, o->pt_P, 3 * (size_t)np);
    XFER(h2d, f.pt.sigma2 + P, o->pt_sigma2, (size_t)np);
    XFER(h2d, f.pt.idx + P, o->pt_idx, (size_t)np);
    XFER(h2d, f.pt.level + P, o->pt_level, (size_t)np);
    XFER(h2d, f.pt.inlier + P, o->pt_inlier, (size_t)np);
    XFER(h2d, f.pt.desc + 32 * P, o->pdesc, 32 * (size_t)np);
    XFER(h2d, f.ls.spl + 2 * L, o->ls_spl, 2 * (size_t)nl);
    XFER(h2d, f.ls.epl + 2 * L, o->ls_epl, 2 * (size_t)nl);
    XFER(h2d, f.ls.spl_obs + 2 * L, o->ls_spl_obs, 2 * (size_t)nl);
    XFER(h2d, f.ls.epl_obs + 2 * L, o->ls_epl_obs, 2 * (size_t)nl);
    XFER(h2d, f.ls.sdisp + L, o->ls_sdisp, (size_t)nl);
    XFER(h2d, f.ls.edisp + L, o->ls_edisp, (size_t)nl);
    XFER(h2d, f.ls.sdisp_obs + L, o->ls_sdisp_obs, (size_t)nl);
    XFER(h2d, f.ls.edisp_obs + L, o->ls_edisp_obs, (size_t)nl);
    XFER(h2d, f.ls.angle + L, o->ls_angle, (size_t)nl);
    XFER(h2d, f.ls.sigma2 + L, o->ls_sigma2, (size_t)nl);
    XFER(h2d, f.ls.sP + 3 * L, o->ls_sP, 3 * (size_t)nl);
    XFER(h2d, f.ls.eP + 3 * L, o->ls_eP, 3 * (size_t)nl);
    XFER(h2d, f.ls.le + 3 * L, o->ls_le, 3 * (size_t)nl);
    XFER(h2d, f.ls.le_obs + 3 * L, o->ls_le_obs, 3 * (size_t)nl);
    XFER(h2d, f.ls.covS + 9 * L, o->ls_covS, 9 * (size_t)nl);
    XFER(h2d, f.ls.covE + 9 * L, o->ls_covE, 9 * (size_t)nl);
    XFER(h2d, f.ls.cut + 2 * L, o->ls_cut, 2 * (size_t)nl);
    XFER(h2d, f.ls.invcov + 36 * L, o->ls_invcov, 36 * (size_t)nl);
    XFER(h2d, f.ls.idx + L, o->ls_idx, (size_t)nl);
    XFER(h2d, f.ls.level + L, o->ls_level, (size_t)nl);
    XFER(h2d, f.ls.inlier + L, o->ls_inlier, (size_t)nl);
    XFER(h2d, f.ls.desc + 32 * L, o->ldesc, 32 * (size_t)nl);
    XFER(h2d, f.pose.Tfw + 16 * seq, o->Tfw, 16);
    XFER(h2d, f.pose.DT + 16 * seq, o->DT, 16);
    XFER(h2d, f.pose.DT_cov + 36 * seq, o->DT_cov, 36);
    XFER(h2d, f.pose.Tfw_cov + 36 * seq, o->Tfw_cov, 36);
    XFER(h2d, f.pose.DT_cov_eig + 6 * seq, o->DT_cov_eig, 6);
    XFER(h2d, f.pose.err_norm + seq, &o->err_norm, 1);
    XFER(h2d, f.pose.time_stamp + seq, &o->time_stamp, 1);
    HIPCHK(hipStreamSynchronize(s));
    sb->initialized = true;
    if (which == GFPL_CURR) sb->has_curr = true;
    return GFPL_OK;
}

int gfpl_read_track(gfpl_seqbatch* sb, int seq, gfpl_track_host* o) {
    if (!sb || !o || seq < 0 || seq >= sb->B) return GFPL_E_INVALID;
    hipStream_t s = sb->ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    std::memset(o, 0, sizeof(*o));
    XFER(d2h, &o->n_matched_pt, sb->tr.n_matched_pt + seq, 1);
    XFER(d2h, &o->n_matched_ls, sb->tr.n_matched_ls + seq, 1);
    XFER(d2h, &o->n_inliers, sb->tr.n_inliers + seq, 1);
    XFER(d2h, &o->n_inliers_pt, sb->tr.n_inliers_pt + seq, 1);
    XFER(d2h, &o->n_inliers_ls, sb->tr.n_inliers_ls + seq, 1);
    XFER(d2h, &o->num_frame_loss, sb->tr.num_frame_loss + seq, 1);
    HIPCHK(hipStreamSynchronize(s));
    XFER(d2h, o->matched_pt, sb->tr.matched_pt + (size_t)seq * sb->mpt_cap, (size_t)o->n_matched_pt);
    XFER(d2h, o->matched_ls, sb->tr.matched_ls + (size_t)seq * sb->mls_cap, (size_t)o->n_matched_ls);
    HIPCHK(hipStreamSynchronize(s));
    return GFPL_OK;
}

int gfpl_read_last_track(gfpl_seqbatch* sb, int seq, gfpl_track_host* o) {
    if (!sb || !o || seq < 0 || seq >= sb->B) return GFPL_E_INVALID;
    hipStream_t s = sb->ctx->stream;
    HIPCHK(hipStreamSynchronize(s));
    std::memset(o, 0, sizeof(*o));
    XFER(d2h, &o->n_matched_pt, sb->last_n_pt + seq, 1);
    XFER(d2h, &o->n_matched_ls, sb->last_n_ls + seq, 1);
    XFER(d2h, &o->n_inliers, sb->tr.n_inliers + seq, 1);
    XFER(d2h, &o->n_inliers_pt, sb->tr.n_inliers_pt + seq, 1);
    XFER(d2h, &o->n_inliers_ls, sb->tr.n_inliers_ls + seq, 1);
    XFER(d2h, &o->num_frame_loss, sb->tr.num_frame_loss + seq, 1);
    HIPCHK(hipStreamSynchronize(s));
    XFER(d2h, o->matched_pt, sb->tr.matched_pt + (size_t)seq * sb->mpt_cap, (size_t)o->n_matched_pt);
    XFER(d2h, o->matched_ls, sb->tr.matched_ls + (size_t)seq * sb->mls_cap, (size_t)o->n_matched_ls);
    HIPCHK(hipStreamSynchronize(s));
    return GFPL_OK;
}

int gfpl_write_track(gfpl_seqbatch* sb, int seq, const gfpl_track_host* o) {
    if (!sb || !o || seq < 0 || seq >= sb->B) return GFPL_E_INVALID;
    if (o->n_matched_pt < 0 || o->n_matched_pt > sb->mpt_cap || o->n_matched_ls < 0 || o->n_matched_ls > sb->mls_cap)
        return GFPL_E_CAPACITY;
    hipStream_t s = sb->ctx->stream;
    XFER(h2d, sb->tr.n_matched_pt + seq, &o->n_matched_pt, 1);
    XFER(h2d, sb->tr.n_matched_ls + seq, &o->n_matched_ls, 1);
    XFER(h2d, sb->tr.n_inliers + seq, &o->n_inliers, 1);
    XFER(h2d, sb->tr.n_inliers_pt + seq, &o->n_inliers_pt, 1);
    XFER(h2d, sb->tr.n_inliers_ls + seq, &o->n_inliers_ls, 1);
    XFER(h2d, sb->tr.num_frame_loss + seq, &o->num_frame_loss, 1);
    XFER(h2d, sb->tr.matched_pt + (size_t)seq * sb->mpt_cap, o->matched_pt, (size_t)o->n_matched_pt);
    XFER(h2d, sb->tr.matched_ls + (size_t)seq * sb->mls_cap, o->matched_ls, (size_t)o->n_matched_ls);
    HIPCHK(hipStreamSynchronize(s));
    return GFPL_OK;
}

int gfpl_set_timing(gfpl_ctx* c, int enable) {
    if (!c) return GFPL_E_INVALID;
    c->timing = enable != 0;
    return GFPL_OK;
}

int gfpl_get_stage_times(gfpl_ctx* c, float* ms7) {
    if (!c || !ms7) return GFPL_E_INVALID;
    if (!c->timing) return GFPL_E_STATE;
    HIPCHK(hipEventSynchronize(c->ev[6]));
    for (int i = 0; i < 6; ++i) HIPCHK(hipEventElapsedTime(&ms7[i], c->ev[i], c->ev[i + 1]));
    HIPCHK(hipEventElapsedTime(&ms7[6], c->ev[0], c->ev[6]));
    return GFPL_OK;
}

int gfpl_get_kernel_times(gfpl_ctx* c, float* ms4) {
    if (!c || !ms4) return GFPL_E_INVALID;
    if (!c->timing) return GFPL_E_STATE;
    if (!c->cfg.use_line_conf_cut) return GFPL_E_STATE;   // no cut kernels were marked
    HIPCHK(hipEventSynchronize(c->ev[6]));
    HIPCHK(hipEventElapsedTime(&ms4[0], c->ev[4], c->ev[7]));   // k_cut_prep
    HIPCHK(hipEventElapsedTime(&ms4[1], c->ev[7], c->ev[8]));   // k_cut_search
    HIPCHK(hipEventElapsedTime(&ms4[2], c->ev[8], c->ev[5]));   // k_cut_finish (+ k_step_bytes)
    HIPCHK(hipEventElapsedTime(&ms4[3], c->ev[5], c->ev[9]));   // k_pose
    return GFPL_OK;
}

}  // extern "C"

namespace {
// column sums over the B per-sequence step records (k_step_bytes)
int step_rec_sums(gfpl_seqbatch* sb, int64_t* sums) {
    std::vector<int64_t> v((size_t)sb->B * STEP_REC);
    HIPCHK(hipStreamSynchronize(sb->ctx->stream));
    HIPCHK(hipMemcpy(v.data(), sb->scr.bytes, sizeof(int64_t) * v.size(), hipMemcpyDeviceToHost));
    for (int s = 0; s < STEP_REC; ++s) {
        int64_t t = 0;
        for (int b = 0; b < sb->B; ++b) t += v[(size_t)b * STEP_REC + s];
        sums[s] = t;
    }
    return GFPL_OK;
}
}  // namespace

extern "C" {

int gfpl_last_step_kernel_bytes(gfpl_seqbatch* sb, int64_t* bytes4) {
    if (!sb || !bytes4) return GFPL_E_INVALID;
    int64_t v[STEP_REC];
    int e = step_rec_sums(sb, v);
    if (e) return e;
    // k_cut_search bytes are recorded per sequence; k_pose's are the pose stage's.  k_cut_prep and
    // k_cut_finish from the summed matched counts (v[13] M_p, v[14] M_l):
    //   prep:   per matched line its cut inputs sP eP covS covE le_obs (208 B) + index (4 B), per
    //           matched point P + pl_obs (40 B) + index (4 B); per sequence the two Tfw (256 B),
    //           DT_inv and invCov_sum out (128 + 168 B)
    //   finish: per matched line its cut inputs + index + ratios (228 B) read, invCovPose (288 B) and
    //           the cut endpoints sP eP spl epl sdisp edisp (96 B) written
    const bool cut = sb->last_cut_mode >= 0;
    bytes4[0] = cut ? 212 * v[14] + 44 * v[13] + 552 * (int64_t)sb->B : 0;
    bytes4[1] = v[7];
    bytes4[2] = cut ? 612 * v[14] : 0;
    bytes4[3] = v[5];
    return GFPL_OK;
}

int gfpl_last_step_stage_bytes(gfpl_seqbatch* sb, int64_t* bytes7) {
    if (!sb || !bytes7) return GFPL_E_INVALID;
    int64_t v[STEP_REC];
    int e = step_rec_sums(sb, v);
    if (e) return e;
    for (int s = 0; s < 7; ++s) bytes7[s] = v[s];
    return GFPL_OK;
}

int gfpl_last_step_counts(gfpl_seqbatch* sb, int64_t* counts8) {
    if (!sb || !counts8) return GFPL_E_INVALID;
    int64_t v[STEP_REC];
    int e = step_rec_sums(sb, v);
    if (e) return e;
    for (int s = 0; s < 8; ++s) counts8[s] = v[8 + s];
    return GFPL_OK;
}

int gfpl_last_step_track_counts(gfpl_seqbatch* sb, int64_t* counts4) {
    if (!sb || !counts4) return GFPL_E_INVALID;
    int64_t v[STEP_REC];
    int e = step_rec_sums(sb, v);
    if (e) return e;
    for (int s = 0; s < 4; ++s) counts4[s] = v[16 + s];
    return GFPL_OK;
}

int gfpl_last_step_cut_proof(gfpl_seqbatch* sb, int64_t* counts4) {
    if (!sb || !counts4) return GFPL_E_INVALID;
    int64_t v[STEP_REC];
    int e = step_rec_sums(sb, v);
    if (e) return e;
    // slots [20..23] are written by k_cut_verify only: report them for a step that ran it
    const bool on = sb->last_cut_mode == 1 || sb->last_cut_mode == 3;
    for (int s = 0; s < 4; ++s) counts4[s] = on ? v[20 + s] : 0;
    return GFPL_OK;
}

int gfpl_debug_cut_records(gfpl_seqbatch* sb, int b, double* out, int n_lines) {
    if (!sb || !out || b < 0 || b >= sb->B || n_lines < 0 || n_lines > sb->mls_cap) return GFPL_E_INVALID;
    if (hipSetDevice(sb->ctx->device) != hipSuccess) return GFPL_E_HIP;
    if (hipStreamSynchronize(sb->ctx->stream) != hipSuccess) return GFPL_E_HIP;
    const size_t n = (size_t)n_lines * CUT_REC;
    return hipMemcpy(out, sb->scr.cut_rec + (size_t)b * sb->mls_cap * CUT_REC, n * sizeof(double),
                     hipMemcpyDeviceToHost) == hipSuccess ? GFPL_OK : GFPL_E_HIP;
}

int gfpl_debug_step_records(gfpl_seqbatch* sb, int64_t* out) {
    if (!sb || !out) return GFPL_E_INVALID;
    if (hipSetDevice(sb->ctx->device) != hipSuccess) return GFPL_E_HIP;
    if (hipStreamSynchronize(sb->ctx->stream) != hipSuccess) return GFPL_E_HIP;
    return hipMemcpy(out, sb->scr.bytes, (size_t)sb->B * STEP_REC * sizeof(int64_t), hipMemcpyDeviceToHost) == hipSuccess
               ? GFPL_OK : GFPL_E_HIP;
}

int gfpl_debug_clocks(gfpl_seqbatch* sb, int64_t* out) {
    if (!sb || !out) return GFPL_E_INVALID;
    if (hipSetDevice(sb->ctx->device) != hipSuccess) return GFPL_E_HIP;
    if (hipStreamSynchronize(sb->ctx->stream) != hipSuccess) return GFPL_E_HIP;
    return hipMemcpy(out, sb->scr.dbg, (size_t)sb->B * 8 * sizeof(int64_t), hipMemcpyDeviceToHost) == hipSuccess
               ? GFPL_OK : GFPL_E_HIP;
}

int gfpl_last_step_bytes(gfpl_seqbatch* sb, int64_t* bytes) {
    if (!bytes) return GFPL_E_INVALID;
    int64_t v[7];
    int e = gfpl_last_step_stage_bytes(sb, v);
    if (e) return e;
    *bytes = v[6];
    return GFPL_OK;
}

}  // extern "C"
