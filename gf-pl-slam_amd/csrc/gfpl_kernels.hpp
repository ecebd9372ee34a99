// gfpl_kernels.hpp — launchers implemented in the k_*.hip translation units.
#pragma once
#include "gfpl_state.hpp"

#include <atomic>

namespace gfpl {

// A kernel's dynamic-LDS ceiling above the 64 KB default, set once per device (the attribute
// belongs to the device's kernel object; contexts on several devices may share the process).
// *done: one bit per device id < 64 (idempotent: two threads setting it race harmlessly)
inline hipError_t ensure_dyn_lds(const void* fn, int bytes, std::atomic<unsigned long long>* done) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = dev < 64 ? 1ull << dev : 0ull;
    if (bit && (done->load(std::memory_order_acquire) & bit)) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess && bit) done->fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

// the batch size up to which the stereo and cross stages run 16 waves per sequence (k_stereo.hip)
int sp_wide_max_b();
hipError_t launch_stereo_points(const KParams& p, hipStream_t s);
hipError_t launch_stereo_lines(const KParams& p, hipStream_t s);
hipError_t launch_line_uncertainty(const KParams& p, hipStream_t s);
hipError_t launch_init(const KParams& p, hipStream_t s);
hipError_t launch_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, int32_t* idx, float* dist,
                       hipStream_t s);
// k_match.hip: radiusMatch rows (count pass, then the rows at row_off) and knn-2 list statistics
hipError_t launch_radius_count(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, float radius,
                               int32_t* cnt, hipStream_t s);
hipError_t launch_radius_rows(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, float radius,
                              const int32_t* row_off, int32_t* idx, float* dist, hipStream_t s);
hipError_t launch_match_stats(int kind, const float* d0, const float* d1, int n, int max_num, double* out,
                              hipStream_t s);
hipError_t launch_cross_points(const KParams& p, hipStream_t s);
hipError_t launch_cross_lines(const KParams& p, hipStream_t s);
hipError_t launch_line_cut(const KParams& p, hipStream_t s, const hipEvent_t* marks /* [2] or null */);
hipError_t launch_pose(const KParams& p, hipStream_t s, hipEvent_t mark /* or null */);
hipError_t launch_step_bytes(const KParams& p, hipStream_t s);
hipError_t launch_need_kf(const KParams& p, hipStream_t s);
hipError_t launch_curr_frame_is_kf(const KParams& p, const int32_t* mask /* device [B] */, hipStream_t s);

size_t stereo_lines_lds(int cap);

// lookForCommonMatches keyframe-pair gate (k_kf.hip); all pointers device
struct KfGate {
    DevCam cam;
    double T0[16], T1[16];
    double max_ratio_12_p, desc_th_l;
    int lines, n0;
    int map;                // 0: keyframe pair (DT = inv(T1) T0), 1: local map (Twf = inv(T1))
    const int32_t* loc;     // map mode: query row -> caller's map row
    int p_stride;           // doubles between rows of P0 / eP0 (3, or 6 for line3D)
    double epip_p, epip_l;  // map mode: maxKFEpipP / maxKFEpipL
    const double* le1;      // map mode: kf1 le [n1][3] (lines)
    const int32_t* i12;     // knn-2 kf0 -> kf1 [2 n0]
    const float* d12;
    const int32_t* i21;     // knn-2 kf1 -> kf0 [2 n1]
    const double* P0;       // kf0 P (points) / sP (lines) [n0][3]
    const double* eP0;      // kf0 eP [n0][3] (lines)
    const double* le0;      // kf0 le [n0][3] (lines)
    const double* sigma2_0; // kf0 sigma2 [n0]
    const double* pl1;      // kf1 pl [n1][2] (points)
    int32_t* pairs;         // [2 n0]
    int* count;
};
hipError_t launch_kf_gate(const KfGate& g, hipStream_t s);
// local-map rows in view in front of kf1 (map order): loc / n (device)
hipError_t launch_kf_map_filter(const DevCam& cam, const double* T1, const double* P, int n, int lines,
                                int32_t* loc, uint8_t* desc_out, const uint8_t* desc_in, int* count, hipStream_t s);

}  // namespace gfpl

namespace gfpl {
// levels 1.. of packed pyramids (the camera's geometry) from their level 0, as ComputePyramid
// resizes them (k_orb.hip: the ORB extractor's O1 tables and k_orb_resize)
struct PyrBuild;
int pyrbuild_create(const gfpl_camera* cam, PyrBuild** out);
hipError_t pyrbuild_run(PyrBuild* pb, uint8_t* pyr, long long stride, int n, hipStream_t s);
void pyrbuild_destroy(PyrBuild* pb);
}  // namespace gfpl

// context accessors for the other extern "C" objects built on a context (gfpl_abi.hip)
int gfpl_ctx_device(const gfpl_ctx* c);
void* gfpl_ctx_stream(const gfpl_ctx* c);
const gfpl_camera* gfpl_ctx_camera(const gfpl_ctx* c);   // NULL before gfpl_set_camera
// a detector created on the context counts itself in until it is destroyed (gfpl_destroy refuses meanwhile)
void gfpl_ctx_attach(gfpl_ctx* c);
void gfpl_ctx_detach(gfpl_ctx* c);
// how often the event was recorded (gfpl_event_record, or as a tracker call's gfpl_frames.consumed)
int64_t gfpl_event_records(const gfpl_event* e);

namespace gfpl {
// Deferred error status of the stream-ordered detector calls (gfpl_*_async): the kernels
// OR error bits into a device word; each call ends with a copy of it into pinned host
// memory and an event, so the call returns without synchronising; *_status waits for
// the event, reports the bits of every call since the previous status and clears them.
struct AsyncStatus {
    int* dev = nullptr;
    int* host = nullptr;
    hipEvent_t ev = nullptr;
    bool pending = false;
    hipError_t init(int* dev_word, hipStream_t s) {
        dev = dev_word;
        hipError_t e = hipHostMalloc((void**)&host, sizeof(int), hipHostMallocDefault);
        if (e == hipSuccess) { *host = 0; e = hipEventCreateWithFlags(&ev, hipEventDisableTiming); }
        if (e == hipSuccess) e = hipMemsetAsync(dev, 0, sizeof(int), s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e;
    }
    hipError_t enqueue(hipStream_t s) {
        hipError_t e = hipMemcpyAsync(host, dev, sizeof(int), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipEventRecord(ev, s);
        if (e == hipSuccess) pending = true;
        return e;
    }
    // bits of the calls since the last wait (0 when none is pending)
    hipError_t wait(hipStream_t s, int* bits) {
        *bits = 0;
        if (!pending) return hipSuccess;
        hipError_t e = hipEventSynchronize(ev);
        if (e != hipSuccess) return e;
        *bits = *host;
        pending = false;
        if (*bits) {
            *host = 0;
            e = hipMemsetAsync(dev, 0, sizeof(int), s);   // ordered before the next call's kernels
        }
        return e;
    }
    void destroy() {
        if (host) (void)hipHostFree(host);
        if (ev) (void)hipEventDestroy(ev);
        host = nullptr;
        ev = nullptr;
    }
};
}  // namespace gfpl
