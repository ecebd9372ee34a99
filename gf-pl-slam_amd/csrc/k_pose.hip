// k_pose.hip — robust Gauss-Newton pose: optimizePose(prev_frame->DT)
// (src/stereoFrameHandler.cpp:1939-2030) with gaussNewtonOptimization (:2032-2056),
// optimizeFunctions (:2118-2245), removeOutliers (:2058-2116) and
// vector_stdv_mad (src/auxiliar.cpp:521-537).
//
// One 64-lane wave owns one sequence for the whole two-stage solve:
//  * the matched list's inputs (P, pl_obs, sigma2 / sP, eP, le_obs, sigma2) are
//    gathered once into per-sequence scratch, one contiguous record per list entry
//    (48 / 80 B) — lane l owns list positions l, l+64, ... for gather and residuals;
//    each GN run compacts the active entries' records in list order (when any entry
//    is inactive), so a chunk's lane reads its own record with 16-B loads at an
//    address known without an index load;
//  * every GN iteration walks the lists in chunks of 64: each lane evaluates one
//    point and one line (J[6], |e|, Cauchy weight; inactive or past-the-end
//    entries are zero rows) into LDS, then lanes 0-27 (points) and 28-55 (lines)
//    each add one of the 28 reduction entries (21 H + 6 g + 1 e) over the chunk
//    in list order — the reference's accumulation order, so H is bit-identical
//    (a zero row adds +0.0, which leaves a sum that started at +0.0 unchanged);
//  * lane 0 solves the 6x6 LDLT and tests convergence; the wave applies the SE(3)
//    update element-parallel (se3_update_wave).
// The outlier pass takes the MAD medians by bitwise selection over register-held
// residuals (wave_select; lists above 512 entries sort in LDS).
#include <cstdlib>

#include "gfpl_kernels.hpp"

namespace gfpl {

// Small batches (B <= POSE_MULTI_MAX_B) run k_pose<POSE_W>: W waves per sequence, wave 0 the
// solver as in k_pose<1> and waves 1.. helpers that evaluate a GN chunk each per round (the
// list-ordered reduction stays wave 0's, so H keeps its bits).  Wave 0's own phases then
// synchronise as one wave (pose_bar<W>); the block barriers are the helper protocol's alone.
template <int W>
__device__ __forceinline__ void pose_bar() {
    if (W == 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
}

struct PoseLDS {
    double DT[16];
    double DTini[16];
    double H[36];     // (the reduction partials, the increment and se3_update_wave's scratch live
                      // in the chunk region, dead between chunk loops: 944 B less per wave)
    int brk;
    int upd;          // apply inc to DT (the error test did not stop the loop)
    int ninl;
    int cnt[2];
    double err;
    int cmd, c0, np_act, nl_act, nch;   // k_pose<W > 1>: helper command (0 exit, 1 evaluate chunks c0 + w)
    int pcomp, lcomp;                   // k_pose<W > 1>: the run reads the compacted records (pose_act)
    int gen;                            // k_pose<W > 1>: GN run number (the helpers' register-held inputs)
#ifdef GFPL_POSE_CLOCK   // (diagnostic build: wave 0's shader-clock cycles per phase, scr.dbg 0-7)
    unsigned long long ck[8], ck0;
#endif
};
#ifdef GFPL_POSE_CLOCK
#define POSE_CK(S, i) do { if (threadIdx.x == 0) { const unsigned long long t_ = clock64(); (S).ck[i] += t_ - (S).ck0; (S).ck0 = t_; } } while (0)
#else
#define POSE_CK(S, i) do { } while (0)
#endif

// DT <- DT * inverse_se3(expmap_se3(inc)) (gaussNewtonOptimization, src/stereoFrameHandler.cpp:
// 2046-2050) by the wave, element-parallel: every element is formed by the expression the serial
// helpers use for it (expmap_se3, inverse_se3, mat4_mul in gfpl_device.hpp), so the bits are
// theirs; theta, sin and cos are computed identically by every lane.  inc, DT, X in LDS.
// Out of line: inlined into the GN loop it raised k_pose to 172 VGPRs (2 waves / SIMD, 6.31 ms);
// as a call it costs a 48-B stack save and the kernel keeps 3 waves / SIMD (5.82 ms; the serial
// lane-0 update ran 5.95 ms)
template <int W>
__device__ __attribute__((noinline)) void se3_update_wave(const double* inc, double* DT, double* X) {
    const int lane = threadIdx.x;
    double* E = X;        // [16] expmap_se3(inc)
    double* Sm = X + 16;  // [9] skew(w) / theta, then V
    double* Ei = X + 32;  // [16] inverse_se3(E)
    const double w0 = inc[3], w1 = inc[4], w2 = inc[5];
    const double theta = sqrt((w0 * w0 + w1 * w1) + w2 * w2);
    const int r9 = lane / 3, c9 = lane - 3 * (lane / 3);
    if (!(theta < 0.000001)) {   // wave-uniform
        if (lane < 9) {
            const double sk = lane == 1 ? -w2 : lane == 2 ? w1 : lane == 3 ? w2 : lane == 5 ? -w0
                            : lane == 6 ? -w1 : lane == 7 ? w0 : 0.0;
            Sm[lane] = sk / theta;
        }
        pose_bar<W>();
        const double st = det_sin(theta), ct = det_cos(theta);
        double Vi = 0.0;
        if (lane < 9) {
            const double si = Sm[lane];
            const double ssi = (Sm[r9 * 3 + 0] * Sm[0 * 3 + c9] + Sm[r9 * 3 + 1] * Sm[1 * 3 + c9]) + Sm[r9 * 3 + 2] * Sm[2 * 3 + c9];
            const double Ii = (r9 == c9) ? 1.0 : 0.0;
            const double omc = 1.0 - ct;
            E[r9 * 4 + c9] = (Ii + si * st) + ssi * omc;
            const double tms = theta - st;
            Vi = (Ii + (si * omc) / theta) + (ssi * tms) / theta;
        }
        pose_bar<W>();
        if (lane < 9) Sm[lane] = Vi;
        pose_bar<W>();
        if (lane < 3) E[lane * 4 + 3] = (Sm[lane * 3 + 0] * inc[0] + Sm[lane * 3 + 1] * inc[1]) + Sm[lane * 3 + 2] * inc[2];
    } else {
        if (lane < 9) E[r9 * 4 + c9] = (r9 == c9) ? 1.0 : 0.0;
        if (lane < 3) E[lane * 4 + 3] = inc[lane];
    }
    if (lane >= 12 && lane < 16) E[lane] = (lane == 15) ? 1.0 : 0.0;
    pose_bar<W>();
    const int r = (lane >> 2) & 3, c = lane & 3;
    if (lane < 16) {
        double ei;
        if (r < 3 && c < 3) ei = E[c * 4 + r];
        else if (r < 3) ei = ((-E[0 * 4 + r]) * E[3] + (-E[1 * 4 + r]) * E[7]) + (-E[2 * 4 + r]) * E[11];
        else ei = (c == 3) ? 1.0 : 0.0;
        Ei[lane] = ei;
    }
    pose_bar<W>();
    double dn = 0.0;
    if (lane < 16)
        dn = ((DT[r * 4 + 0] * Ei[0 * 4 + c] + DT[r * 4 + 1] * Ei[1 * 4 + c]) + DT[r * 4 + 2] * Ei[2 * 4 + c]) +
             DT[r * 4 + 3] * Ei[3 * 4 + c];
    pose_bar<W>();
    if (lane < 16) DT[lane] = dn;
    pose_bar<W>();
}

#define PT_K 6    // X Y Z ox oy sigma2
// chunk rows are 66 doubles (528 B) apart: the reduction lanes read rows ia, ib
// of the same columns k, k + 1 as 16-B pairs, and a 64-double stride would put
// every row in the same LDS bank
#define CH_STRIDE 66
// register budget of the GN loop (DESIGN.md §4 k_pose): DT read from LDS, the next chunk's
// inputs prefetched into registers and a 4-deep reduction unroll: 149 VGPRs (3 waves /
// SIMD, which the ~10 KB LDS workgroup allows), 7.3 -> 6.9 ms measured; without the
// prefetch (117 VGPRs) it was slower again
#define GFPL_POSE_RED_UNROLL 4
#define LS_K 10   // sX sY sZ eX eY eZ l0 l1 l2 sigma2

// projection (gfpl_device.hpp) with the two divisions by P[2] sharing the reciprocal
__device__ __forceinline__ void projection_sd(const DevCam& c, const double* P, double* uv) {
    const double nx = c.fx * P[0], ny = c.fy * P[1];
    const SharedDiv dz = div_prep(P[2], nx);
    uv[0] = c.cx + div_by(dz, nx);
    uv[1] = c.cy + div_by(dz, ny);
}

// evaluate one point row (src/stereoFrameHandler.cpp:2130-2160) -> J[6], n, w;
// in = X Y Z ox oy sigma2 (registers)
__device__ __forceinline__ void eval_point(const DevCam& cam, double homog, const double* DT, const double* in,
                                           double* o) {
    const double Pp[3] = {in[0], in[1], in[2]};
    double Pc[3], uv[2];
    se3_apply(DT, Pp, Pc);
    projection_sd(cam, Pc, uv);
    const double ex = uv[0] - in[3], ey = uv[1] - in[4];
    const double n = sqrt(ex * ex + ey * ey);
    double J[6];
    poseJac(cam, homog, Pc, ex, ey, J);
    const double m = ref_max(homog, n);
    const SharedDiv dm = div_prep(m, J[0]);
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] = div_by(dm, J[i]);
    o[6] = n;
    o[7] = 1.0 / (1.0 + (n * n) * in[5]);
}

// evaluate one line row (src/stereoFrameHandler.cpp:2175-2235);
// in = sX sY sZ eX eY eZ l0 l1 l2 sigma2 (registers)
__device__ __forceinline__ void eval_line(const DevCam& cam, double homog, const double* DT, const double* in,
                                          double* o) {
    const double sP[3] = {in[0], in[1], in[2]};
    const double eP[3] = {in[3], in[4], in[5]};
    double sc[3], ec[3], su[2], eu[2];
    se3_apply(DT, sP, sc);
    projection_sd(cam, sc, su);
    se3_apply(DT, eP, ec);
    projection_sd(cam, ec, eu);
    const double l0 = in[6], l1 = in[7], l2 = in[8];
    const double ds = (l0 * su[0] + l1 * su[1]) + l2;
    const double de = (l0 * eu[0] + l1 * eu[1]) + l2;
    const double n = sqrt(ds * ds + de * de);
    double Js[6], Je[6];
    poseJac(cam, homog, sc, l0, l1, Js);
    poseJac(cam, homog, ec, l0, l1, Je);
    const double m = ref_max(homog, n);
    double t[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) t[i] = Js[i] * ds + Je[i] * de;
    const SharedDiv dm = div_prep(m, t[0]);
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] = div_by(dm, t[i]);
    o[6] = n;
    o[7] = 1.0 / (1.0 + (n * n) * in[9]);
}

struct PoseCtx {
    const double* pin;   // [npt][PT_K] records of this sequence, list order
    const double* lin;   // [nls][LS_K]
    double* pact;        // [np_act][PT_K] the active points' records, compacted per GN run (HBM)
    double* lact;        // [nl_act][LS_K]
    const uint8_t* act;  // LDS [npt + nls] list-position inlier flags
    int npt, nls;
};

// one record: 16-B loads (records are 16-B aligned: 48 / 80 B, the scratch 256-B aligned).  The
// address space is stated: through PoseCtx the compiler lost it for the line records and issued
// flat loads, which count in lgkmcnt as well — every LDS sync of the chunk loop then waited for the
// next chunk's prefetch
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const f64x2 g_double2;
template <int K>
__device__ __forceinline__ void load_rec(const double* base, int f, double* v) {
    const g_double2* r = (const g_double2*)(base + (size_t)K * f);
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
        const f64x2 t = r[i];
        v[2 * i] = t.x;
        v[2 * i + 1] = t.y;
    }
}
typedef __attribute__((address_space(1))) f64x2 g_double2w;
template <int K>
__device__ __forceinline__ void store_rec(double* base, int f, const double* v) {
    g_double2w* r = (g_double2w*)(base + (size_t)K * f);
#pragma unroll
    for (int i = 0; i < K / 2; ++i) r[i] = f64x2{v[2 * i], v[2 * i + 1]};
}

// k_pose<W > 1>: chunk c0 + w of the active entries (points and lines) evaluated into wave w's rows.
// The chunk's inputs are gathered into pv / lv when `load`; a GN run whose chunks fit one round
// (nch <= W) evaluates the same entries every iteration, so the callers keep them in registers and
// load once per run (only DT changes between iterations).
template <int W>
__device__ __forceinline__ void pose_eval_chunk(const KParams& p, const double* pa, const double* la, const double* DT,
                                                int c0, int np_act, int nl_act, double* cp, double* cl, int w,
                                                double* pv, double* lv, bool load) {
    const int lane = threadIdx.x & 63;
    const int c = c0 + w;
    const int f = (c << 6) + lane;
    double* cpw = cp + w * (16 * CH_STRIDE);
    double* clw = cl + w * (16 * CH_STRIDE);
    if (load) {
        load_rec<PT_K>(pa, f < np_act ? f : 0, pv);
        load_rec<LS_K>(la, f < nl_act ? f : 0, lv);
    }
    double o[8];
    if (f < np_act) {
        eval_point(p.cam, p.cfg.homog_th, DT, pv, o);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) cpw[i * CH_STRIDE + lane] = o[i];
    if (f < nl_act) {
        eval_line(p.cam, p.cfg.homog_th, DT, lv, o);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) clw[i * CH_STRIDE + lane] = o[i];
}

// the helper waves of k_pose<W > 1>: evaluate chunk c0 + w on every command until the exit command
// (inputs kept in registers across the iterations of a one-round GN run: S.gen numbers the runs)
template <int W>
__device__ void pose_helper(const KParams& p, const PoseCtx& X, PoseLDS& S, double* cp, double* cl) {
    const int w = threadIdx.x >> 6;
    double pv[PT_K], lv[LS_K];
    int gen = -1;
    for (;;) {
        __syncthreads();   // (A)
        if (S.cmd == 0) return;
        const int c0 = S.c0, nch = S.nch;
        if (c0 + w < nch) {
            const bool keep = W >= 8 && nch <= W;   // (see gauss_newton)
            pose_eval_chunk<W>(p, S.pcomp ? X.pact : X.pin, S.lcomp ? X.lact : X.lin, S.DT, c0, S.np_act, S.nl_act,
                               cp, cl, w, pv, lv, !(keep && gen == S.gen));
            gen = keep ? S.gen : -1;
        }
        __syncthreads();   // (B)
    }
}

// gaussNewtonOptimization (:2032-2056): DT updated in place in S, H = last evaluated
// Issue priority by progress: 3 in the first half of the first GN run, down to 0 in the second half
// of the second, so the waves dispatched last are not starved by the older ones (the arbiter favours
// the older of two ready waves) at the end of the grid: 4.92 -> 4.76 ms (profiles/r04_t)
__device__ __forceinline__ void pose_prio(int stage, int it, int n) {
    const int q = 2 * stage + (2 * it >= n ? 1 : 0);
    if (q <= 0) __builtin_amdgcn_s_setprio(3);
    else if (q == 1) __builtin_amdgcn_s_setprio(2);
    else if (q == 2) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// entry pairs of chunk c the reduction lane adds: its list's remaining entries (rounded up to a pair),
// none for lanes 56-63
__device__ __forceinline__ int red_pairs(int lane, int list, int np_act, int nl_act, int c) {
    const int rem = min(64, max(0, (list == 0 ? np_act : nl_act) - (c << 6)));
    return lane < 56 ? (rem + 1) >> 1 : 0;
}

template <int W>
__device__ void gauss_newton(const KParams& p, const PoseCtx& X, PoseLDS& S, double* cp, double* cl,
                             int max_iters, int stage) {
    const int lane = threadIdx.x;
    const DevCam& cam = p.cam;
    const double homog = p.cfg.homog_th;
    double err_prev = 999999999.9;   // lane 0 only
    if (lane == 0) S.err = 0.0;
    // reduction role: lanes 0-27 points, 28-55 lines; entry e: H lower (ti,tj), g_i, e
    const int list = lane / 28, e = lane % 28;
    int ia, ib;
    if (e < 21) { int ti = 0; while ((ti + 1) * (ti + 2) / 2 <= e) ++ti; ia = ti; ib = e - ti * (ti + 1) / 2; }
    else if (e < 27) { ia = e - 21; ib = 6; }
    else { ia = 6; ib = 6; }
    const double* buf = list == 0 ? cp : cl;
    const uint8_t* actp = X.act;
    const uint8_t* actl = X.act + X.npt;
    // the active entries, compacted in list order (an inactive entry is a zero row, and adding
    // +0.0 to a sum that started at +0.0 never changes it: skipping them leaves H bit-identical);
    // after removeOutliers about a third of the entries are inactive.  Their records are copied
    // into pose_act, contiguous, so chunk c is records [64 c, 64 c + 64) of one array: no index
    // load ahead of the inputs' loads, no inactive records between them
    int np_act = 0, nl_act = 0;
    {
        for (int b0 = 0; b0 < X.npt; b0 += 64) np_act += __popcll(__ballot(b0 + lane < X.npt && actp[b0 + lane]));
        for (int b0 = 0; b0 < X.nls; b0 += 64) nl_act += __popcll(__ballot(b0 + lane < X.nls && actl[b0 + lane]));
    }
    const bool cpts = np_act != X.npt, clns = nl_act != X.nls;   // (wave-uniform)
    {
        const unsigned long long lt = (1ull << lane) - 1ull;
        if (cpts) {
            int n = 0;
            for (int b0 = 0; b0 < X.npt; b0 += 64) {
                const int f = b0 + lane;
                const bool a = f < X.npt && actp[f];
                const unsigned long long m = __ballot(a);
                if (a) {
                    double v[PT_K];
                    load_rec<PT_K>(X.pin, f, v);
                    store_rec<PT_K>(X.pact, n + __popcll(m & lt), v);
                }
                n += __popcll(m);
            }
        }
        if (clns) {
            int n = 0;
            for (int b0 = 0; b0 < X.nls; b0 += 64) {
                const int f = b0 + lane;
                const bool a = f < X.nls && actl[f];
                const unsigned long long m = __ballot(a);
                if (a) {
                    double v[LS_K];
                    load_rec<LS_K>(X.lin, f, v);
                    store_rec<LS_K>(X.lact, n + __popcll(m & lt), v);
                }
                n += __popcll(m);
            }
        }
        if (W > 1 && lane == 0) { S.pcomp = cpts ? 1 : 0; S.lcomp = clns ? 1 : 0; }
        pose_bar<W>();
    }
    const double* pa = cpts ? X.pact : X.pin;
    const double* la = clns ? X.lact : X.lin;
    const int ntot = max(np_act, nl_act), nch = (ntot + 63) >> 6;
    // k_pose<W >= 8>: wave 0's chunk inputs, kept over a one-round run (k_pose<4> at B <= 1024 keeps its
    // occupancy: 4 waves / SIMD need <= 128 VGPRs)
    constexpr bool KEEP = W >= 8;
    double pv0[PT_K], lv0[LS_K];
    if (W > 1 && lane == 0) S.gen = S.gen + 1;
    double* part = cp;        // [64] the 28 + 28 reduction partials
    double* incs = cp + 64;   // [6] the increment
    double* xs = cp + 72;     // [48] se3_update_wave scratch
    POSE_CK(S, 7);
    for (int it = 0; it < max_iters; ++it) {
        pose_prio(stage, it, max_iters);
        // the evaluations read DT from LDS (wave-uniform broadcast reads) instead of
        // holding 16 doubles in registers across the chunk loop
        const double* DT = S.DT;
        double s = 0.0;
        // raw inputs of chunk c + 1 are loaded into registers while chunk c is
        // reduced, so the SoA scratch latency hides behind the LDS reduction
        double pv[PT_K], lv[LS_K];
        auto load_chunk = [&](int c) {
            const int f = (c << 6) + lane;
            load_rec<PT_K>(pa, f < np_act ? f : 0, pv);
            load_rec<LS_K>(la, f < nl_act ? f : 0, lv);
        };
        if (W == 1) {
            load_chunk(0);
            for (int c = 0; c < nch; ++c) {
                const int f = (c << 6) + lane;
                double o[8];
                if (f < np_act) eval_point(cam, homog, DT, pv, o);
                else {
    #pragma unroll
                    for (int i = 0; i < 8; ++i) o[i] = 0.0;
                }
    #pragma unroll
                for (int i = 0; i < 8; ++i) cp[i * CH_STRIDE + lane] = o[i];
                if (f < nl_act) eval_line(cam, homog, DT, lv, o);
                else {
    #pragma unroll
                    for (int i = 0; i < 8; ++i) o[i] = 0.0;
                }
    #pragma unroll
                for (int i = 0; i < 8; ++i) cl[i * CH_STRIDE + lane] = o[i];
                if (c + 1 < nch) load_chunk(c + 1);
                pose_bar<W>();
                const double* A = buf + ia * CH_STRIDE;
                const double* Bv = buf + ib * CH_STRIDE;
                const double* Wr = buf + 7 * CH_STRIDE;
                const double2* A2 = reinterpret_cast<const double2*>(A);
                const double2* B2 = reinterpret_cast<const double2*>(Bv);
                const double2* W2 = reinterpret_cast<const double2*>(Wr);
                // the entry pairs of this chunk the lane's list has (the rows past its end are zero: +0.0
                // leaves the sum's bits); lanes 56-63 hold no entry — the LDS reads, not the adds, bound
                // this loop at 4 waves per SIMD
                const int kmax = red_pairs(lane, list, np_act, nl_act, c);
    #pragma unroll GFPL_POSE_RED_UNROLL
                for (int k = 0; k < kmax; ++k) {
                    const double2 a = A2[k], bb = B2[k], w = W2[k];
                    s = s + (a.x * bb.x) * w.x;
                    s = s + (a.y * bb.y) * w.y;
                }
                pose_bar<W>();
            }
        } else {
            // rounds of W chunks: wave w evaluates chunk c0 + w (the helpers on a command), then
            // the reduction lanes add the round's chunks in list order
            if (lane == 0) { S.np_act = np_act; S.nl_act = nl_act; S.nch = nch; }
            for (int c0 = 0; c0 < nch; c0 += W) {
                if (lane == 0) { S.cmd = 1; S.c0 = c0; }
                __syncthreads();   // (A) the helpers read the command, DT and the positions
                pose_eval_chunk<W>(p, pa, la, S.DT, c0, np_act, nl_act, cp, cl, 0, pv0, lv0, !(KEEP && nch <= W && it > 0));
                __syncthreads();   // (B) the round's rows are in LDS
                POSE_CK(S, 5);
                const int nw = min(W, nch - c0);
                for (int wb = 0; wb < nw; ++wb) {
                    const double* bw = (list == 0 ? cp : cl) + wb * (16 * CH_STRIDE);
                    const double2* A2 = reinterpret_cast<const double2*>(bw + ia * CH_STRIDE);
                    const double2* B2 = reinterpret_cast<const double2*>(bw + ib * CH_STRIDE);
                    const double2* W2 = reinterpret_cast<const double2*>(bw + 7 * CH_STRIDE);
                    const int kmax = red_pairs(lane, list, np_act, nl_act, c0 + wb);
                    if (W >= 8) {
                        // the add chain is the serial part (list order): reads issued 16 entries ahead of
                        // it (the 8-wave kernel has the registers)
#pragma unroll 8
                        for (int k = 0; k < 32; ++k) {   // (a fixed trip count: the reads stay 16 entries ahead)
                            const double2 a = A2[k], bb = B2[k], w = W2[k];
                            s = s + (a.x * bb.x) * w.x;
                            s = s + (a.y * bb.y) * w.y;
                        }
                    } else {
#pragma unroll GFPL_POSE_RED_UNROLL
                        for (int k = 0; k < kmax; ++k) {
                            const double2 a = A2[k], bb = B2[k], w = W2[k];
                            s = s + (a.x * bb.x) * w.x;
                            s = s + (a.y * bb.y) * w.y;
                        }
                    }
                }
            }
            pose_bar<W>();
        }
        POSE_CK(S, 1);
        part[lane] = s;
        pose_bar<W>();
        // H = H_p + H_l, one element per lane (the symmetric pair gets the same sum)
        if (lane < 36) {
            const int r = lane / 6, c = lane - 6 * (lane / 6);
            const int t = r >= c ? tri(r, c) : tri(c, r);
            S.H[lane] = part[t] + part[28 + t];
        }
        pose_bar<W>();
        if (lane == 0) {
            double H[36], g[6];
            for (int i = 0; i < 36; ++i) H[i] = S.H[i];
            for (int i = 0; i < 6; ++i) g[i] = part[21 + i] + part[28 + 21 + i];
            double ee = part[27] + part[28 + 27];
            ee = ee / (double)(S.cnt[1] + S.cnt[0]);
            S.err = ee;
            int brk = 0, upd = 0;
            if ((fabs(ee - err_prev) < p.cfg.min_error_change) || (ee < p.cfg.min_error)) {
                brk = 1;
            } else {
                double inc[6];
                ldlt_solve6_one_lane(H, g, inc);
                for (int i = 0; i < 6; ++i) incs[i] = inc[i];
                upd = 1;
                const double nrm = sqrt(((((inc[0] * inc[0] + inc[1] * inc[1]) + inc[2] * inc[2]) + inc[3] * inc[3]) +
                                         inc[4] * inc[4]) + inc[5] * inc[5]);
                if (nrm < 2.220446049250313e-16) brk = 1;
                err_prev = ee;
            }
            S.brk = brk;
            S.upd = upd;
        }
        pose_bar<W>();
        POSE_CK(S, 2);
        if (S.upd) se3_update_wave<W>(incs, S.DT, xs);   // DT * inverse_se3(expmap_se3(inc)), before the nrm break
        POSE_CK(S, 3);
        if (S.brk) break;
    }
}

// vector_stdv_mad on buf[0..n) (LDS, destroyed); buf has NP2 entries
template <int W>
__device__ double stdv_mad(double* buf, int n, int NP2) {
    const int nthr = W == 1 ? (int)blockDim.x : 64;   // (W > 1: wave 0 alone)
    if (n == 0) return 0.0;   // uniform
    for (int i = threadIdx.x + n; i < NP2; i += nthr) buf[i] = __builtin_inf();
    pose_bar<W>();
    for (int k = 2; k <= NP2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < NP2; i += nthr) {
                int ixj = i ^ j;
                if (ixj > i) {
                    bool up = ((i & k) == 0);
                    double x = buf[i], y = buf[ixj];
                    if ((x > y) == up) { buf[i] = y; buf[ixj] = x; }
                }
            }
            pose_bar<W>();
        }
    const double median = buf[n / 2];
    pose_bar<W>();
    for (int i = threadIdx.x; i < n; i += nthr) buf[i] = (double)fabsf((float)(buf[i] - median));
    pose_bar<W>();
    for (int k = 2; k <= NP2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < NP2; i += nthr) {
                int ixj = i ^ j;
                if (ixj > i) {
                    bool up = ((i & k) == 0);
                    double x = buf[i], y = buf[ixj];
                    if ((x > y) == up) { buf[i] = y; buf[ixj] = x; }
                }
            }
            pose_bar<W>();
        }
    const double mad = buf[n / 2];
    pose_bar<W>();
    return 1.4826 * mad;
}

// k-th smallest (0-based) of the unsigned keys a wave holds in registers (lane l, slot r:
// list position l + 64 r; slots past the list hold all-ones keys, never selected since
// k < n).  The answer is built bit by bit from the top: the largest P with
// #{x < P} <= k is the k-th smallest key, and each bit costs one compare per slot (the
// compare mask is the ballot) and a scalar popcount — no sort.  For non-negative doubles
// (floats) the bit patterns order like the values, so this is the element
// std::sort(...)[k] leaves at k (vector_stdv_mad, src/auxiliar.cpp:521-537); residuals
// sqrt(.) * sqrt(sigma2) and fabsf(.) are never -0.0.
template <typename K>
__device__ __forceinline__ K readlane_key(K v, int l) {
    if (sizeof(K) == 8) {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
        return (K)(((uint64_t)hi << 32) | lo);
    }
    return (K)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
template <typename K, int R>
__device__ __forceinline__ K wave_select(const K* key, int n, int k) {
    // two bits per pass: the three thresholds' counts are independent (one pass's compares and
    // popcounts overlap), and the largest threshold with count <= k is the bit-by-bit choice of
    // both bits (the counts are monotone in the threshold).  lo / hi count the keys below the
    // window [P, P + 2^(b+2)) the choices so far leave (lo <= k < hi); once it holds one key, that
    // key is the k-th (the remaining bits are its own) and is read out.  (Keys are non-negative
    // doubles / floats: P + 2^b stays below the sign bit; padding keys ~0 never count.)
    K P = 0;
    int lo = 0, hi = n;
    for (int b = 8 * (int)sizeof(K) - 2; b >= 0; b -= 2) {
        const K T1 = P | ((K)1 << b), T2 = P | ((K)2 << b), T3 = P | ((K)3 << b);
        int c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r * 64 < n) {
                c1 += __popcll(__ballot(key[r] < T1));
                c2 += __popcll(__ballot(key[r] < T2));
                c3 += __popcll(__ballot(key[r] < T3));
            }
        if (c3 <= k) { P = T3; lo = c3; }
        else if (c2 <= k) { P = T2; lo = c2; hi = c3; }
        else if (c1 <= k) { P = T1; lo = c1; hi = c2; }
        else { hi = c1; }
        if (hi - lo == 1 && b > 0) {   // (wave-uniform) the window's one key
            const K wd = (K)1 << b;
            K v = 0;
            bool in = false;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (r * 64 < n && (K)(key[r] - P) < wd) { v = key[r]; in = true; }
            return readlane_key<K>(v, __builtin_ctzll(__ballot(in)));
        }
    }
    return P;
}

// vector_stdv_mad of n <= 64 R residuals held in registers (r[slot] = list position
// lane + 64 slot): the median, then the median of (double)fabsf((float)(x - median))
template <int R>
__device__ __forceinline__ double stdv_mad_regs(const double* r, int n) {
    if (n == 0) return 0.0;   // uniform
    const int lane = threadIdx.x & 63;
    uint64_t k64[R];
#pragma unroll
    for (int s = 0; s < R; ++s)
        k64[s] = (lane + 64 * s < n) ? (uint64_t)__double_as_longlong(r[s]) : ~0ull;
    const double median = __longlong_as_double((long long)wave_select<uint64_t, R>(k64, n, n / 2));
    uint32_t k32[R];
#pragma unroll
    for (int s = 0; s < R; ++s)
        k32[s] = (lane + 64 * s < n) ? __float_as_uint(fabsf((float)(r[s] - median))) : ~0u;
    const double mad = (double)__uint_as_float(wave_select<uint32_t, R>(k32, n, n / 2));
    return 1.4826 * mad;
}
#define POSE_MAD_R 8   // residuals per lane held in registers (lists of up to 512 entries)

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// removeOutliers(DT_) (:2058-2116): the residual of list entry k (its record in pose_in)
__device__ __forceinline__ double point_residual(const KParams& p, const double* pin, const double* DTs, int k) {
    double in[PT_K];
    load_rec<PT_K>(pin, k, in);
    const double Pp[3] = {in[0], in[1], in[2]};
    double Pc[3], uv[2];
    se3_apply(DTs, Pp, Pc);
    projection(p.cam, Pc, uv);
    const double ex = uv[0] - in[3], ey = uv[1] - in[4];
    return sqrt(ex * ex + ey * ey) * sqrt(in[5]);
}
__device__ __forceinline__ double line_residual(const KParams& p, const double* lin, const double* DTs, int k) {
    double in[LS_K];
    load_rec<LS_K>(lin, k, in);
    const double sP[3] = {in[0], in[1], in[2]};
    const double eP[3] = {in[3], in[4], in[5]};
    double sc[3], ec[3], su[2], eu[2];
    se3_apply(DTs, sP, sc);
    se3_apply(DTs, eP, ec);
    projection(p.cam, sc, su);
    projection(p.cam, ec, eu);
    const double l0 = in[6], l1 = in[7], l2 = in[8];
    const double e0 = (l0 * su[0] + l1 * su[1]) + l2;
    const double e1 = (l0 * eu[0] + l1 * eu[1]) + l2;
    return sqrt(e0 * e0 + e1 * e1) * sqrt(in[9]);
}

// the line list's outlier flags from register-held residuals (n <= 64 POSE_MAD_R): returns the
// wave's flagged count
__device__ __forceinline__ int line_outliers_regs(const KParams& p, const double* lin, const double* DTs,
                                                  uint8_t* act, int npt, int nls, size_t lb, const int32_t* mls) {
    const int lane = threadIdx.x & 63;
    double r[POSE_MAD_R];
#pragma unroll
    for (int s = 0; s < POSE_MAD_R; ++s) r[s] = (lane + 64 * s < nls) ? line_residual(p, lin, DTs, lane + 64 * s) : 0.0;
    const double th_l = p.cfg.inlier_k * stdv_mad_regs<POSE_MAD_R>(r, nls);
    int ol = 0;
#pragma unroll
    for (int s = 0; s < POSE_MAD_R; ++s) {
        const int k = lane + 64 * s;
        if (k < nls && r[s] > th_l) { p.prev.ls.inlier[lb + mls[k]] = 0; act[npt + k] = 0; ++ol; }
    }
    return wave_sum(ol);
}

// dynamic LDS: {cp[8*CH_STRIDE] cl[8*CH_STRIDE] | buf[NP2]} f64 | act[mpt+mls] u8 (16-B padded):
// 9.3 KB + 576 B static at the default caps (500 / 300), so 16 waves fit a CU's 160 KB (4 per
// SIMD, as the 122 VGPRs allow); the compacted positions gauss_newton walks live in HBM
#ifndef GFPL_POSE_WAVES
#define GFPL_POSE_WAVES 4
#endif
template <int W>
__global__ void __launch_bounds__(64 * W, W == 1 ? GFPL_POSE_WAVES : 1) k_pose(KParams p, int NP2) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ PoseLDS S;
    const int b = blockIdx.x;
    const int lane = threadIdx.x;   // (W > 1: wave 0's lanes; the helpers branch off below)
    const int npt = p.tr.n_matched_pt[b], nls = p.tr.n_matched_ls[b];
    // the GN chunk rows and the outlier residuals are never live together
    const int region = max(W * 16 * CH_STRIDE, NP2);
    double* cp = (double*)smem;
    double* cl = cp + 8 * CH_STRIDE;
    double* buf = cp;   // MAD sort buffer: never live together with the GN chunk rows
    uint8_t* act = (uint8_t*)(cp + region);
    const DevPose& PP = p.prev.pose;
    const DevPoints& P = p.prev.pt;
    const DevLines& L = p.prev.ls;
    const int32_t* mpt = p.tr.matched_pt + (size_t)b * p.mpt_cap;
    const int32_t* mls = p.tr.matched_ls + (size_t)b * p.mls_cap;
    const size_t pb = (size_t)b * p.kp_cap, lb = (size_t)b * p.kl_cap;
    PoseCtx X;
    double* pin = p.scr.pose_in + (size_t)b * (PT_K * p.mpt_cap + LS_K * p.mls_cap);
    double* lin = pin + PT_K * p.mpt_cap;
    X.pin = pin; X.lin = lin; X.act = act; X.npt = npt; X.nls = nls;
    X.pact = p.scr.pose_act + (size_t)b * (PT_K * p.mpt_cap + LS_K * p.mls_cap);
    X.lact = X.pact + PT_K * p.mpt_cap;
    if (W > 1 && threadIdx.x >= 64) {   // helper waves: GN chunk evaluation on wave 0's commands
        pose_helper<W>(p, X, S, cp, cl);
        return;
    }
    if (lane < 16) {   // Q2: the app passes prev_frame->DT (app/plslam_mod.cpp:408)
        S.DTini[lane] = p.dt_ini ? p.dt_ini[16 * b + lane] : PP.DT[16 * b + lane];
        S.DT[lane] = S.DTini[lane];
    }
    if (lane == 0) { S.ninl = p.tr.n_inliers[b]; S.gen = 0; }
#ifdef GFPL_POSE_CLOCK
    if (lane < 8) S.ck[lane] = 0;
    if (lane == 0) S.ck0 = clock64();
#endif
    // gather the matched lists once (lane l owns positions l, l+64, ...)
    int cpn = 0, cln = 0;
    for (int f = lane; f < npt; f += 64) {
        const size_t q = pb + mpt[f];
        const double v[PT_K] = {P.P[3 * q], P.P[3 * q + 1], P.P[3 * q + 2], P.pl_obs[2 * q], P.pl_obs[2 * q + 1],
                                P.sigma2[q]};
        store_rec<PT_K>(pin, f, v);
        act[f] = P.inlier[q] ? 1 : 0;
        cpn += act[f];
    }
    for (int f = lane; f < nls; f += 64) {
        const size_t q = lb + mls[f];
        const double v[LS_K] = {L.sP[3 * q], L.sP[3 * q + 1], L.sP[3 * q + 2], L.eP[3 * q], L.eP[3 * q + 1],
                                L.eP[3 * q + 2], L.le_obs[3 * q], L.le_obs[3 * q + 1], L.le_obs[3 * q + 2], L.sigma2[q]};
        store_rec<LS_K>(lin, f, v);
        act[npt + f] = L.inlier[q] ? 1 : 0;
        cln += act[npt + f];
    }
    cpn = wave_sum(cpn);
    cln = wave_sum(cln);
    if (lane == 0) { S.cnt[0] = cpn; S.cnt[1] = cln; }
    pose_bar<W>();
    POSE_CK(S, 0);
    int ok = 0;        // 1: stage-2 DT usable
    double err = 0.0;  // err of the last GN run (reference: uninitialised when no GN runs, pinned 0)
    if (S.ninl > p.cfg.min_features) {
        gauss_newton<W>(p, X, S, cp, cl, p.cfg.max_iters, 0);
        POSE_CK(S, 7);
        err = S.err;
        double DTs[16];
        for (int i = 0; i < 16; ++i) DTs[i] = S.DT[i];
        bool fin = true;
        for (int i = 0; i < 16; ++i) { double d = DTs[i] - DTs[i]; if (!(d == d)) fin = false; }
        if (fin) {
            // removeOutliers(DT_) (:2058-2116): residuals of every list entry
            auto res_p = [&](int k) { return point_residual(p, pin, DTs, k); };
            auto res_l = [&](int k) { return line_residual(p, lin, DTs, k); };
            // Lists of up to 512 entries keep their residuals in registers and take both
            // medians by wave_select (no sort); longer lists sort in the GN chunk region (buf
            // aliases it) and the flag pass re-evaluates each residual (same operands, same
            // bits).  Duplicates of one prev point share P, pl_obs and sigma2, hence the
            // residual: flagging per list position equals the reference's per-feature flag.
            int op = 0, ol = 0;
            pose_bar<W>();
            // (the line list's pass on a helper wave beside the points' here measured slower: the
            // helper's registers slowed wave 0's chunk reduction by more than the overlap saved)
            if (npt <= 64 * POSE_MAD_R) {
                double r[POSE_MAD_R];
#pragma unroll
                for (int s = 0; s < POSE_MAD_R; ++s) r[s] = (lane + 64 * s < npt) ? res_p(lane + 64 * s) : 0.0;
                const double th_p = p.cfg.inlier_k * stdv_mad_regs<POSE_MAD_R>(r, npt);
#pragma unroll
                for (int s = 0; s < POSE_MAD_R; ++s) {
                    const int k = lane + 64 * s;
                    if (k < npt && r[s] > th_p) { P.inlier[pb + mpt[k]] = 0; act[k] = 0; ++op; }
                }
            } else {
                for (int k = lane; k < npt; k += 64) buf[k] = res_p(k);
                pose_bar<W>();
                const double th_p = p.cfg.inlier_k * stdv_mad<W>(buf, npt, NP2);
                for (int k = lane; k < npt; k += 64)
                    if (res_p(k) > th_p) { P.inlier[pb + mpt[k]] = 0; act[k] = 0; ++op; }
            }
            pose_bar<W>();
            if (nls <= 64 * POSE_MAD_R) {
                ol = line_outliers_regs(p, lin, DTs, act, npt, nls, lb, mls);
            } else {
                for (int k = lane; k < nls; k += 64) buf[k] = res_l(k);
                pose_bar<W>();
                const double th_l = p.cfg.inlier_k * stdv_mad<W>(buf, nls, NP2);
                for (int k = lane; k < nls; k += 64)
                    if (res_l(k) > th_l) { L.inlier[lb + mls[k]] = 0; act[npt + k] = 0; ++ol; }
                ol = wave_sum(ol);
            }
            op = wave_sum(op);
            // active counts for stage 2
            int ap = 0, al = 0;
            pose_bar<W>();
            for (int k = lane; k < npt; k += 64) ap += act[k];
            for (int k = lane; k < nls; k += 64) al += act[npt + k];
            ap = wave_sum(ap);
            al = wave_sum(al);
            if (lane == 0) {
                S.ninl = S.ninl - op - ol;
                p.tr.n_inliers[b] = S.ninl;
                p.tr.n_inliers_pt[b] -= op;
                p.tr.n_inliers_ls[b] -= ol;
                S.cnt[0] = ap; S.cnt[1] = al;
            }
            pose_bar<W>();
            POSE_CK(S, 4);
            if (S.ninl > p.cfg.min_features) {
                if (lane < 16) S.DT[lane] = S.DTini[lane];   // Q3: stage 2 restarts from DT_ini
                pose_bar<W>();
                gauss_newton<W>(p, X, S, cp, cl, p.cfg.max_iters_ref, 1);
                err = S.err;
                ok = 1;
            }
        }
    }
    POSE_CK(S, 7);
    if (W > 1) {   // release the helpers
        if (lane == 0) S.cmd = 0;
        __syncthreads();
    }
#ifdef GFPL_POSE_CLOCK
    if (lane < 8) p.scr.dbg[8 * (size_t)b + lane] = (int64_t)S.ck[lane];
#endif
    if (lane == 0) {
        for (int i = 0; i < 16; ++i) p.scr.pose_DT[16 * b + i] = S.DT[i];
        for (int i = 0; i < 36; ++i) p.scr.pose_H[36 * b + i] = S.H[i];
        p.scr.pose_err[b] = err;
        p.scr.pose_ok[b] = ok;
    }
}

// Final bookkeeping of optimizePose (src/stereoFrameHandler.cpp:1983-2028), one
// lane per sequence: inverse_se3, motion-step gate, Tfw, DT_cov = H^-1 (Q13),
// its eigenvalues, Tfw_cov = unccomp_se3, err_norm, numFrameLoss.
// Two waves per 64 sequences: both form DT_cov = H^-1; wave 1 takes its eigenvalues (the 6x6 cyclic
// Jacobi, the longest serial chain here) while wave 0 does the rest, on another SIMD — the same
// expressions, so the same bits (two lanes of one wave would run the two paths one after the other)
__global__ void __launch_bounds__(128) k_pose_finish(KParams p) {
    const int b = blockIdx.x * 64 + (threadIdx.x & 63), role = threadIdx.x >> 6;
    if (b >= p.B) return;
#ifdef GFPL_PFIN_CLOCK
    const uint64_t pf0 = clock64();
#endif
    if (role == 0) p.scr.bytes[(size_t)STEP_REC * b + 18] = p.tr.n_inliers[b];   // inliers after removeOutliers (step record)
    DevPose& CP = p.curr.pose;
    const DevPose& PP = p.prev.pose;
    const int ok = p.scr.pose_ok[b];
    const double err = p.scr.pose_err[b];
    double DT[16], DT_cov[36];
    if (ok) {
        double H[36];
#pragma unroll
        for (int i = 0; i < 16; ++i) DT[i] = p.scr.pose_DT[16 * b + i];
#pragma unroll
        for (int i = 0; i < 36; ++i) H[i] = p.scr.pose_H[36 * b + i];
        inverse6(H, DT_cov);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) DT[i] = (i % 5 == 0) ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < 36; ++i) DT_cov[i] = 0.0;
    }
#ifdef GFPL_PFIN_CLOCK
    const uint64_t pf1 = clock64();
#endif
    if (role == 1) {
        double eig[6];
        eig_sym<6>(DT_cov, eig);
#ifdef GFPL_PFIN_CLOCK
        p.scr.dbg[8 * (size_t)b + 1] = (int64_t)(clock64() - pf1);
        p.scr.dbg[8 * (size_t)b + 0] = (int64_t)(pf1 - pf0);
#endif
#pragma unroll
        for (int i = 0; i < 6; ++i) CP.DT_cov_eig[6 * b + i] = eig[i];
        return;
    }
    bool fin = true;
#pragma unroll
    for (int i = 0; i < 16; ++i) { double d = DT[i] - DT[i]; if (!(d == d)) fin = false; }
    double Tp[16], Tpc[36];
#pragma unroll
    for (int i = 0; i < 16; ++i) Tp[i] = PP.Tfw[16 * b + i];
#pragma unroll
    for (int i = 0; i < 36; ++i) Tpc[i] = PP.Tfw_cov[36 * b + i];
    double cDT[16], Tfw[16], Tcov[36];
    double err_norm;
    bool moved = false;
    if (fin) {
        inverse_se3(DT, cDT);
        const double tn = sqrt((cDT[3] * cDT[3] + cDT[7] * cDT[7]) + cDT[11] * cDT[11]);
        moved = tn < p.cfg.motion_step_th * (CP.time_stamp[b] - PP.time_stamp[b]);
        p.tr.num_frame_loss[b] = 0;
    } else {
        p.tr.num_frame_loss[b] = p.tr.num_frame_loss[b] + 1;
    }
    if (moved) {
        mat4_mul(Tp, cDT, Tfw);
        // unccomp_se3(prev.Tfw, prev.Tfw_cov, DT_cov) (src/auxiliar.cpp:216-238)
        double Ad[36];
        adjoint_se3(Tp, Ad);
        sandwich6(Ad, DT_cov, Tpc, Tcov);
        err_norm = err;
    } else {
        // rejected step or non-finite pose: identity, prev pose kept, err_norm = -1
#pragma unroll
        for (int i = 0; i < 16; ++i) { cDT[i] = (i % 5 == 0) ? 1.0 : 0.0; Tfw[i] = Tp[i]; }
#pragma unroll
        for (int i = 0; i < 36; ++i) Tcov[i] = Tpc[i];
        err_norm = -1.0;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) { CP.DT[16 * b + i] = cDT[i]; CP.Tfw[16 * b + i] = Tfw[i]; }
#pragma unroll
    for (int i = 0; i < 36; ++i) { CP.DT_cov[36 * b + i] = DT_cov[i]; CP.Tfw_cov[36 * b + i] = Tcov[i]; }
    CP.err_norm[b] = err_norm;
#ifdef GFPL_PFIN_CLOCK
    p.scr.dbg[8 * (size_t)b + 2] = (int64_t)(clock64() - pf1);
#endif
}

// needNewKF (src/stereoFrameHandler.cpp:2309-2349), one lane per sequence, on the
// curr frame's DT / DT_cov (called after optimizePose, app/plslam_mod.cpp:436)
__global__ void __launch_bounds__(64) k_need_kf(KParams p) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    const DevPose& CP = p.curr.pose;
    DevTrack& T = p.tr;
    double DT[16], DTc[36];
#pragma unroll
    for (int i = 0; i < 16; ++i) DT[i] = CP.DT[16 * b + i];
#pragma unroll
    for (int i = 0; i < 36; ++i) DTc[i] = CP.DT_cov[36 * b + i];
    double e0 = T.kf_entropy0[b];
    if (T.kf_prev_iskf[b]) {
        e0 = kf_entropy(DTc);
        T.kf_entropy0[b] = e0;
        T.kf_prev_iskf[b] = 0;
    }
    double Tk[16], adj[36], Ti[16], adjTinv[36], covDTinv[36], cov[36], acc[36];
#pragma unroll
    for (int i = 0; i < 16; ++i) Tk[i] = T.kf_T[16 * b + i];
    adjoint_se3(Tk, adj);
    inverse_se3(DT, Ti);                 // uncTinv_se3 (src/auxiliar.cpp:225-231)
    adjoint_se3(Ti, adjTinv);
    sandwich6(adjTinv, DTc, nullptr, covDTinv);
#pragma unroll
    for (int i = 0; i < 36; ++i) cov[i] = T.kf_cov[36 * b + i];
    sandwich6(adj, covDTinv, cov, acc);
#pragma unroll
    for (int i = 0; i < 36; ++i) T.kf_cov[36 * b + i] = acc[i];
    const double ratio = kf_entropy(acc) / e0;
    bool zero_cov = true, ident = true;
#pragma unroll
    for (int i = 0; i < 36; ++i) zero_cov = zero_cov && DTc[i] == 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) ident = ident && DT[i] == ((i % 5 == 0) ? 1.0 : 0.0);
    const bool bad = !(ratio == ratio) || ratio == __builtin_inf() || ratio == -__builtin_inf();
    T.kf_ratio[b] = ratio;
    T.kf_flag[b] = (T.kf_nsince[b] > p.cfg.max_kf_num_frames || ratio < p.cfg.min_entropy_ratio || bad ||
                    (zero_cov && ident)) ? 1 : 0;
}

// currFrameIsKF (src/stereoFrameHandler.cpp:2351-2379) for the masked sequences
__global__ void __launch_bounds__(64) k_curr_frame_is_kf(KParams p, const int32_t* mask) {
    const int b = blockIdx.x;
    if (!mask[b]) return;
    DevFrame& C = p.curr;
    const size_t pb = (size_t)b * p.kp_cap, lb = (size_t)b * p.kl_cap;
    for (int i = threadIdx.x; i < C.pt.n[b]; i += blockDim.x) C.pt.idx[pb + i] = i;
    for (int i = threadIdx.x; i < C.ls.n[b]; i += blockDim.x) C.ls.idx[lb + i] = i;
    if (threadIdx.x < 16) {
        const double v = (threadIdx.x % 5 == 0) ? 1.0 : 0.0;
        C.pose.Tfw[16 * b + threadIdx.x] = v;
        p.tr.kf_T[16 * b + threadIdx.x] = v;   // T_prevKF = curr_frame->Tfw (= I)
    }
    if (threadIdx.x < 36) {
        C.pose.Tfw_cov[36 * b + threadIdx.x] = (threadIdx.x % 7 == 0) ? 1.0 : 0.0;
        p.tr.kf_cov[36 * b + threadIdx.x] = 0.0;
    }
    if (threadIdx.x == 0) {
        p.tr.kf_nsince[b] = 0;
        p.tr.kf_prev_iskf[b] = 1;
    }
}

hipError_t launch_need_kf(const KParams& p, hipStream_t s) {
    hipLaunchKernelGGL(k_need_kf, dim3((p.B + 63) / 64), dim3(64), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_curr_frame_is_kf(const KParams& p, const int32_t* mask, hipStream_t s) {
    hipLaunchKernelGGL(k_curr_frame_is_kf, dim3(p.B), dim3(64), 0, s, p, mask);
    return hipGetLastError();
}

#ifndef POSE_W
#define POSE_W 4
#endif
#ifndef POSE_MULTI_MAX_B
#define POSE_MULTI_MAX_B 1024
#endif
// the batch size up to which k_pose runs POSE_W waves per sequence (GFPL_POSE_MULTI_MAX_B overrides)
static int pose_multi_max_b() {
    const char* e = getenv("GFPL_POSE_MULTI_MAX_B");
    return e ? atoi(e) : POSE_MULTI_MAX_B;
}
// ... and up to which it runs 8 (a list of <= 512 active entries is then one round of chunks per GN
// iteration; 1 workgroup of 8 waves per CU at B <= 256); GFPL_POSE_W8_MAX_B overrides
#ifndef POSE_W8_MAX_B
#define POSE_W8_MAX_B 256
#endif
static int pose_w8_max_b() {
    const char* e = getenv("GFPL_POSE_W8_MAX_B");
    return e ? atoi(e) : POSE_W8_MAX_B;
}

hipError_t launch_pose(const KParams& p, hipStream_t s, hipEvent_t mark) {
    int NP2 = 1;
    while (NP2 < p.mpt_cap || NP2 < p.mls_cap) NP2 <<= 1;
    const bool w8 = p.B <= pose_w8_max_b();
    const bool multi = p.B <= pose_multi_max_b();   // small batches: POSE_W waves per sequence
    const int Wl = w8 ? 8 : (multi ? POSE_W : 1);
    const size_t region = (size_t)std::max(Wl * 16 * CH_STRIDE, NP2);
    const size_t lds = region * 8 + ((p.mpt_cap + p.mls_cap + 15) & ~15) + 16;
    if (w8) {
        static std::atomic<unsigned long long> attr{0};   // (dynamic LDS above the 64 KB default)
        const hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(k_pose<8>), 160 * 1024 - 1024, &attr);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_pose<8>, dim3(p.B), dim3(64 * 8), lds, s, p, NP2);
    } else if (multi)
        hipLaunchKernelGGL(k_pose<POSE_W>, dim3(p.B), dim3(64 * POSE_W), lds, s, p, NP2);
    else
        hipLaunchKernelGGL(k_pose<1>, dim3(p.B), dim3(64), lds, s, p, NP2);
    if (mark) (void)hipEventRecord(mark, s);
    hipLaunchKernelGGL(k_pose_finish, dim3((p.B + 63) / 64), dim3(128), 0, s, p);
    return hipGetLastError();
}

}  // namespace gfpl
