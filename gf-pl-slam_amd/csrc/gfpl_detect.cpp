// gfpl_detect.cpp — the image-input boundary (include/gfpl.h, gfpl_detector_*):
// StereoFrame's detection for B stereo frames on the device, composed from the
// ORB (k_orb.hip), LSD (k_lsd.hip) and LBD (k_lbd.hip) objects.
//
// Reference: StereoFrame::StereoFrame(img_l, img_r, idx, cam, ts) + extractStereoFeatures /
// extractInitialStereoFeatures' detection half (src/stereoFrame.cpp:148-172, 411-450):
// detectPointFeatures (:1128-1152) runs ORB_SLAM2::ORBextractor(orbNFeatures,
// orbScaleFactor, orbNLevels, 20, 7) on each image, detectLineFeatures (:1155-1227)
// LSDDetectorC::detect with the Config LSD options, the lsdNFeatures response sort, then
// BinaryDescriptor::compute.  Called by StereoFrameHandler::initialize / insertStereoPair
// (src/stereoFrameHandler.cpp:45-151) on the images the app passes
// (app/plslam_mod.cpp:377,387).
//
// Streams: the detector owns two contexts on streams of its own (gfpl_create_async): ORB of
// both images on one, LSD of both images (one 2B-image call: the latency-bound region growth
// wants every image in flight) then LBD of both on the other; the ORB stream joins the line
// stream before the set's `ready` event.  The input images are first copied into the set's
// image buffer ([left B | right B], the layout one LSD call reads).  Every gfpl_frames view
// carries `ready` (detection done) and `consumed` (recorded by the tracker call that reads
// it), so the next detection into the same buffer set waits for exactly that read.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../../include/gfpl.h"
#include "gfpl_kernels.hpp"

namespace {

constexpr int kMaxSets = 4;

struct DetSet {
    uint8_t* img = nullptr;        // [2B][H][W]: left images, then right images
    int* n_kp[2] = {};             // [B]
    gfpl_keypoint* kp[2] = {};     // [B][kp_cap]
    uint8_t* pdesc[2] = {};        // [B][kp_cap][32]
    int* n_kl = nullptr;           // [2B]: left then right (one LSD call)
    gfpl_keyline* kl = nullptr;    // [2B][kl_cap]
    uint8_t* ldesc[2] = {};        // [B][kl_cap][32]
    uint8_t* pyr[2] = {};          // [B][pyr_bytes]: left (ORB's working pyramid), right (the tracker's pyr_r)
    double* ts = nullptr;          // [B]
    gfpl_event* ready = nullptr;   // on the line stream: the set's detection is complete
    gfpl_event* orb_done = nullptr;
    gfpl_event* copied = nullptr;  // the set's image copy is complete (the ORB stream waits for it)
    gfpl_event* consumed = nullptr;
    bool handed = false;           // a view of this set was returned ...
    int64_t handed_at = 0;         // ... when `consumed` had been recorded this often
};

#define DET_HIPCHK(x)                                                                   \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "gfpl_detector: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return GFPL_E_HIP;                                                          \
        }                                                                               \
    } while (0)

#define DET_CHK(x)            \
    do {                      \
        const int e_ = (x);   \
        if (e_) return e_;    \
    } while (0)

}  // namespace

struct gfpl_detector {
    gfpl_ctx* ctx = nullptr;                        // the caller's context (counted in)
    gfpl_ctx* c_orb = nullptr, *c_lines = nullptr;  // the detector's own streams
    gfpl_orb* orb = nullptr;
    gfpl_lsd* lsd = nullptr;
    gfpl_lbd* lbd = nullptr;
    gfpl_event* inputs = nullptr;   // recorded on the caller's stream: the images are produced
    int B = 0, kp_cap = 0, kl_cap = 0, sets = 0, W = 0, H = 0;
    int64_t pyr_bytes = 0;
    void* base = nullptr;
    DetSet set[kMaxSets];
    int64_t k = 0;
};

namespace {

void teardown(gfpl_detector* d) {
    if (d->c_lines) (void)gfpl_synchronize(d->c_lines);
    if (d->c_orb) (void)gfpl_synchronize(d->c_orb);
    if (d->orb) gfpl_orb_destroy(d->orb);
    if (d->lsd) gfpl_lsd_destroy(d->lsd);
    if (d->lbd) gfpl_lbd_destroy(d->lbd);
    for (int s = 0; s < kMaxSets; ++s)
        for (gfpl_event* e : {d->set[s].ready, d->set[s].orb_done, d->set[s].copied, d->set[s].consumed})
            if (e) gfpl_event_destroy(e);
    if (d->inputs) gfpl_event_destroy(d->inputs);
    if (d->base) (void)hipFree(d->base);
    if (d->c_orb) gfpl_destroy(d->c_orb);
    if (d->c_lines) gfpl_destroy(d->c_lines);
    if (d->ctx) gfpl_ctx_detach(d->ctx);
    delete d;
}

// first half of a detection: pick the set, check it is free, order both streams after the
// caller's stream and the set's last tracker read
int begin(gfpl_detector* d, int n, DetSet** out) {
    DetSet& S = d->set[d->k % d->sets];
    if (S.handed && gfpl_event_records(S.consumed) <= S.handed_at) return GFPL_E_STATE;
    DET_CHK(gfpl_event_record(d->inputs, d->ctx));
    for (gfpl_ctx* c : {d->c_lines, d->c_orb}) {
        DET_CHK(gfpl_event_wait(c, d->inputs));
        DET_CHK(gfpl_event_wait(c, S.consumed));
    }
    (void)n;
    *out = &S;
    return GFPL_OK;
}

// second half: ORB on the ORB stream, LSD + LBD on the line stream, the join, the view
int run(gfpl_detector* d, DetSet& S, int n, gfpl_frames* out) {
    const size_t img = (size_t)d->W * d->H;
    const uint8_t* left = S.img;
    const uint8_t* right = S.img + (size_t)n * img;
    DET_CHK(gfpl_event_record(S.copied, d->c_lines));
    DET_CHK(gfpl_event_wait(d->c_orb, S.copied));
    // the caller's stream is ordered after the input copies: work it enqueues after this call
    // (e.g. writing the next frame into the same img_l / img_r / time_stamp) cannot overtake them
    DET_CHK(gfpl_event_wait(d->ctx, S.copied));
    for (int side = 0; side < 2; ++side)
        DET_CHK(gfpl_orb_extract_async(d->orb, side ? right : left, n, S.kp[side], S.pdesc[side], S.n_kp[side], nullptr,
                                       nullptr, S.pyr[side], d->pyr_bytes));
    DET_CHK(gfpl_event_record(S.orb_done, d->c_orb));
    // LSD of the 2n images in one call: keylines [2n][kl_cap], left images first
    DET_CHK(gfpl_lsd_detect_async(d->lsd, S.img, 2 * n, S.kl, S.n_kl, nullptr));
    DET_CHK(gfpl_lbd_compute_async(d->lbd, left, n, S.kl, S.n_kl, S.ldesc[0]));
    DET_CHK(gfpl_lbd_compute_async(d->lbd, right, n, S.kl + (size_t)n * d->kl_cap, S.n_kl + n, S.ldesc[1]));
    DET_CHK(gfpl_event_wait(d->c_lines, S.orb_done));
    DET_CHK(gfpl_event_record(S.ready, d->c_lines));
    gfpl_frames f{};
    f.batch = n;
    f.kp_cap = d->kp_cap;
    f.kl_cap = d->kl_cap;
    f.n_kp_l = S.n_kp[0];
    f.n_kp_r = S.n_kp[1];
    f.kp_l = S.kp[0];
    f.kp_r = S.kp[1];
    f.pdesc_l = S.pdesc[0];
    f.pdesc_r = S.pdesc[1];
    f.n_kl_l = S.n_kl;
    f.n_kl_r = S.n_kl + n;
    f.kl_l = S.kl;
    f.kl_r = S.kl + (size_t)n * d->kl_cap;
    f.ldesc_l = S.ldesc[0];
    f.ldesc_r = S.ldesc[1];
    f.pyr_r = S.pyr[1];
    f.time_stamp = S.ts;
    f.ready = S.ready;
    f.consumed = S.consumed;
    *out = f;
    S.handed = true;
    S.handed_at = gfpl_event_records(S.consumed);
    ++d->k;
    return GFPL_OK;
}

}  // namespace

extern "C" {

int gfpl_detector_params_default(const gfpl_camera* cam, const gfpl_config* cfg, gfpl_detector_params* prm) {
    if (!cam || !prm) return GFPL_E_INVALID;
    gfpl_config c;
    if (cfg) c = *cfg;
    else gfpl_config_default(&c);
    std::memset(prm, 0, sizeof *prm);
    // src/stereoFrame.cpp:33-36, Config::orbNFeatures 1000 (src/config.cpp:134; BASELINE cfg 2 sets 2000)
    prm->orb.nfeatures = 1000;
    prm->orb.scale_factor = (float)c.orb_scale_factor;
    prm->orb.nlevels = c.orb_n_levels;
    prm->orb.ini_th_fast = 20;
    prm->orb.min_th_fast = 7;
    // src/stereoFrame.cpp:1160-1171 with src/config.cpp:143-152; min_line_length =
    // Config::minLineLength() * min(W, H) (src/stereoFrame.cpp:151, :416)
    prm->lsd.refine = 1;
    prm->lsd.scale = c.lsd_scale;
    prm->lsd.quant = 2.0;
    prm->lsd.ang_th = 22.5;
    prm->lsd.density_th = 0.6;
    prm->lsd.n_bins = 1024;
    prm->lsd.min_length = 0.025 * (double)(cam->width < cam->height ? cam->width : cam->height);
    prm->lsd.n_features = 300;
    prm->seg_cap = 4096;
    return GFPL_OK;
}

int gfpl_detector_create(gfpl_ctx* ctx, const gfpl_detector_params* prm, int max_batch, int kp_cap, int kl_cap,
                         int sets, gfpl_detector** out) {
    if (!ctx || !prm || !out || max_batch < 1 || kp_cap < 1 || kl_cap < 1 || sets < 1 || sets > kMaxSets ||
        prm->seg_cap < 1)
        return GFPL_E_INVALID;
    const gfpl_camera* cam = gfpl_ctx_camera(ctx);
    if (!cam) return GFPL_E_STATE;   // the pyramid the tracker reads follows the context's camera
    if (kp_cap > 8192 || kl_cap > 2048) return GFPL_E_INVALID;   // the seqbatch capacities
    gfpl_detector* d = new gfpl_detector();
    d->ctx = ctx;
    gfpl_ctx_attach(ctx);
    d->B = max_batch;
    d->kp_cap = kp_cap;
    d->kl_cap = kl_cap;
    d->sets = sets;
    d->W = cam->width;
    d->H = cam->height;
    int e = GFPL_OK;
    const int dev = gfpl_ctx_device(ctx);
    if (!e) e = gfpl_create_async(dev, &d->c_orb);
    if (!e) e = gfpl_create_async(dev, &d->c_lines);
    for (gfpl_ctx* c : {d->c_orb, d->c_lines})
        if (!e) e = gfpl_set_camera(c, cam);
    if (!e) e = gfpl_orb_create(d->c_orb, d->W, d->H, &prm->orb, max_batch, kp_cap, &d->orb);
    if (!e) e = gfpl_orb_pyramid_bytes(d->orb, &d->pyr_bytes);
    // ORB writes the tracker's right pyramid: its level geometry must be the camera's
    if (!e && (d->pyr_bytes > cam->pyr_bytes || prm->orb.nlevels != cam->n_levels)) e = GFPL_E_INVALID;
    if (!e) d->pyr_bytes = cam->pyr_bytes;   // the stride gfpl_frames.pyr_r is read at
    if (!e) e = gfpl_lsd_create(d->c_lines, &prm->lsd, d->W, d->H, 2 * max_batch, kl_cap, prm->seg_cap, &d->lsd);
    if (!e) e = gfpl_lbd_create(d->c_lines, d->W, d->H, max_batch, kl_cap, &d->lbd);
    if (!e) e = gfpl_event_create(ctx, &d->inputs);
    for (int s = 0; s < sets && !e; ++s)
        for (gfpl_event** ev : {&d->set[s].ready, &d->set[s].orb_done, &d->set[s].copied, &d->set[s].consumed})
            if (!e) e = gfpl_event_create(ctx, ev);
    if (e) { teardown(d); return e; }
    // one allocation for every set, 256-B aligned fields
    const size_t B = max_batch, img = (size_t)d->W * d->H;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t per_set = al(2 * B * img) + 2 * al(4 * B) + 2 * al(B * kp_cap * sizeof(gfpl_keypoint)) +
                           2 * al(B * kp_cap * 32) + al(8 * B) + al(2 * B * kl_cap * sizeof(gfpl_keyline)) +
                           2 * al(B * kl_cap * 32) + 2 * al(B * (size_t)d->pyr_bytes) + al(8 * B);
    if (hipSetDevice(dev) != hipSuccess || hipMalloc(&d->base, per_set * sets) != hipSuccess ||
        hipMemset(d->base, 0, per_set * sets) != hipSuccess) {
        teardown(d);
        return GFPL_E_HIP;
    }
    char* p = (char*)d->base;
    auto take = [&](size_t bytes) { char* q = p; p += al(bytes); return q; };
    for (int s = 0; s < sets; ++s) {
        DetSet& S = d->set[s];
        S.img = (uint8_t*)take(2 * B * img);
        for (int side = 0; side < 2; ++side) {
            S.n_kp[side] = (int*)take(4 * B);
            S.kp[side] = (gfpl_keypoint*)take(B * kp_cap * sizeof(gfpl_keypoint));
            S.pdesc[side] = (uint8_t*)take(B * kp_cap * 32);
        }
        S.n_kl = (int*)take(8 * B);
        S.kl = (gfpl_keyline*)take(2 * B * kl_cap * sizeof(gfpl_keyline));
        for (int side = 0; side < 2; ++side) S.ldesc[side] = (uint8_t*)take(B * kl_cap * 32);
        for (int side = 0; side < 2; ++side) S.pyr[side] = (uint8_t*)take(B * (size_t)d->pyr_bytes);
        S.ts = (double*)take(8 * B);
    }
    *out = d;
    return GFPL_OK;
}

int gfpl_detector_destroy(gfpl_detector* d) {
    if (!d) return GFPL_E_INVALID;
    teardown(d);
    return GFPL_OK;
}

int gfpl_detect_stereo_async(gfpl_detector* d, const uint8_t* img_l, const uint8_t* img_r, int n,
                             const double* time_stamp, gfpl_frames* out) {
    if (!d || !img_l || !img_r || !time_stamp || !out || n < 1 || n > d->B) return GFPL_E_INVALID;
    DetSet* S = nullptr;
    DET_CHK(begin(d, n, &S));
    const size_t bytes = (size_t)n * d->W * d->H;
    hipStream_t s = (hipStream_t)gfpl_get_stream(d->c_lines);
    DET_HIPCHK(hipMemcpyAsync(S->img, img_l, bytes, hipMemcpyDeviceToDevice, s));
    DET_HIPCHK(hipMemcpyAsync(S->img + bytes, img_r, bytes, hipMemcpyDeviceToDevice, s));
    DET_HIPCHK(hipMemcpyAsync(S->ts, time_stamp, 8 * (size_t)n, hipMemcpyDeviceToDevice, s));
    return run(d, *S, n, out);
}

int gfpl_detect_stereo_host(gfpl_detector* d, const uint8_t* img_l, const uint8_t* img_r, int n,
                            const double* time_stamp, gfpl_frames* out) {
    if (!d || !img_l || !img_r || !time_stamp || !out || n < 1 || n > d->B) return GFPL_E_INVALID;
    DetSet* S = nullptr;
    DET_CHK(begin(d, n, &S));
    const size_t bytes = (size_t)n * d->W * d->H;
    hipStream_t s = (hipStream_t)gfpl_get_stream(d->c_lines);
    DET_HIPCHK(hipMemcpyAsync(S->img, img_l, bytes, hipMemcpyHostToDevice, s));
    DET_HIPCHK(hipMemcpyAsync(S->img + bytes, img_r, bytes, hipMemcpyHostToDevice, s));
    DET_HIPCHK(hipMemcpyAsync(S->ts, time_stamp, 8 * (size_t)n, hipMemcpyHostToDevice, s));
    // the caller's host buffers may change once this returns
    DET_HIPCHK(hipStreamSynchronize(s));
    return run(d, *S, n, out);
}

int gfpl_detector_status(gfpl_detector* d) {
    if (!d) return GFPL_E_INVALID;
    int e = gfpl_orb_status(d->orb);
    const int e2 = gfpl_lsd_status(d->lsd);
    const int e3 = gfpl_lbd_status(d->lbd);
    return e ? e : (e2 ? e2 : e3);
}

int gfpl_detect_stereo(gfpl_detector* d, const uint8_t* img_l, const uint8_t* img_r, int n, const double* time_stamp,
                       int host_pointers, gfpl_frames* out) {
    const int e = host_pointers ? gfpl_detect_stereo_host(d, img_l, img_r, n, time_stamp, out)
                                : gfpl_detect_stereo_async(d, img_l, img_r, n, time_stamp, out);
    if (e) return e;
    return gfpl_detector_status(d);
}

int gfpl_detector_discard(gfpl_detector* d, const gfpl_frames* f) {
    if (!d || !f || !f->consumed) return GFPL_E_INVALID;
    for (int s = 0; s < d->sets; ++s)
        if (d->set[s].consumed == f->consumed) return gfpl_event_record(f->consumed, d->c_lines);
    return GFPL_E_INVALID;
}

int gfpl_read_detections(gfpl_ctx* ctx, const gfpl_frames* f, int seq, gfpl_detections_host* out) {
    if (!ctx || !f || !out || seq < 0 || seq >= f->batch) return GFPL_E_INVALID;
    if (f->ready) DET_CHK(gfpl_event_synchronize(f->ready));
    DET_HIPCHK(hipSetDevice(gfpl_ctx_device(ctx)));
    int n[4];
    const int* cnt[4] = {f->n_kp_l, f->n_kp_r, f->n_kl_l, f->n_kl_r};
    for (int i = 0; i < 4; ++i) DET_HIPCHK(hipMemcpy(&n[i], cnt[i] + seq, 4, hipMemcpyDeviceToHost));
    out->n_kp_l = n[0];
    out->n_kp_r = n[1];
    out->n_kl_l = n[2];
    out->n_kl_r = n[3];
    for (int i = 0; i < 2; ++i)
        if (n[i] < 0 || n[i] > f->kp_cap || n[2 + i] < 0 || n[2 + i] > f->kl_cap) return GFPL_E_CAPACITY;
    const size_t kp0 = (size_t)seq * f->kp_cap, kl0 = (size_t)seq * f->kl_cap;
    struct Cp { void* dst; const void* src; size_t bytes; } cps[] = {
        {out->kp_l, f->kp_l + kp0, n[0] * sizeof(gfpl_keypoint)},
        {out->kp_r, f->kp_r + kp0, n[1] * sizeof(gfpl_keypoint)},
        {out->pdesc_l, f->pdesc_l + 32 * kp0, 32 * (size_t)n[0]},
        {out->pdesc_r, f->pdesc_r + 32 * kp0, 32 * (size_t)n[1]},
        {out->kl_l, f->kl_l + kl0, n[2] * sizeof(gfpl_keyline)},
        {out->kl_r, f->kl_r + kl0, n[3] * sizeof(gfpl_keyline)},
        {out->ldesc_l, f->ldesc_l + 32 * kl0, 32 * (size_t)n[2]},
        {out->ldesc_r, f->ldesc_r + 32 * kl0, 32 * (size_t)n[3]},
    };
    for (const Cp& c : cps)
        if (c.dst && c.bytes) DET_HIPCHK(hipMemcpy(c.dst, c.src, c.bytes, hipMemcpyDeviceToHost));
    return GFPL_OK;
}

}  // extern "C"
