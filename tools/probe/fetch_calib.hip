// Probe: FETCH_SIZE calibration for k_stereo_points' SAD access pattern.
// The MI355X guide's factor 2 (FETCH_SIZE reports half of the bytes of wide coalesced reads on
// gfx950) is measured on 16-B streaming loads; the SAD reads window rows as dword-aligned 16-B
// and 8-B vector loads at scattered, misaligned row offsets (sad_load_row).  Three kernels read a
// buffer of KNOWN size exactly once (each 64-B line by one lane group), so FETCH_SIZE x 1 KB /
// bytes gives the factor per pattern:
//   stream  — 16-B loads, consecutive lanes consecutive 16 B (the guide's case)
//   gather  — the SAD's pattern: per lane one 16-B + one 8-B load at a misaligned byte offset
//             (rounded down to a dword) of a random 64-B-aligned row segment, covering each
//             line once
//   rows    — per lane 11 rows x (16 + 24) B windows of random pixels of a 640x480 image set,
//             as the SAD does (overlap between lanes is counted once: distinct lines touched)
// usage: fetch_calib [MiB]   (run under rocprofv3 --pmc FETCH_SIZE --kernel-trace)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));

__global__ void k_stream(const uint4* a, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// each lane covers one 64-B line: a 16-B load at byte offset sh (dword-aligned down) and an
// 8-B load 16 B further, then the rest of the line by two more 16-B loads (every line read once)
__global__ void k_gather(const uint8_t* a, const uint32_t* perm, size_t nlines, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nlines; i += (size_t)gridDim.x * blockDim.x) {
        const size_t line = perm[i];
        const uint8_t* base = a + line * 64;
        const int sh = (int)(i & 3) * 4;   // dword offsets 0, 4, 8, 12 within the line
        const u32x4a4 x = *reinterpret_cast<const u32x4a4*>(base + sh);
        const u32x2a4 y = *reinterpret_cast<const u32x2a4*>(base + sh + 16);
        const u32x4a4 z = *reinterpret_cast<const u32x4a4*>(base + 32);
        const u32x4a4 w = *reinterpret_cast<const u32x4a4*>(base + 48);
        acc ^= x.x ^ x.w ^ y.x ^ y.y ^ z.x ^ w.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// the SAD window loads of random keypoints on 640 x 480 images (one image per 256 lanes)
__global__ void k_rows(const uint8_t* imgs, int nimg, const uint32_t* kp, int nkp, uint32_t* out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nkp) return;
    const uint32_t k = kp[t];
    const int img = (int)(k >> 20) % nimg, u = (int)((k >> 9) & 511) + 64, v = (int)(k & 511) % 460 + 10;
    const uint8_t* I = imgs + (size_t)img * 640 * 480;
    uint32_t acc = 0;
    for (int r = -5; r <= 5; ++r) {
        const int64_t pl = (int64_t)(v + r) * 640 + u - 5, pr = (int64_t)(v + r) * 640 + u - 40;
        const u32x4a4 x = *reinterpret_cast<const u32x4a4*>(I + (pl & ~3));
        const u32x4a4 y = *reinterpret_cast<const u32x4a4*>(I + (pr & ~3));
        const u32x2a4 z = *reinterpret_cast<const u32x2a4*>(I + (pr & ~3) + 16);
        acc ^= x.x ^ x.w ^ y.y ^ z.x;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atoll(argv[1]) : 1024;
    const size_t bytes = mib << 20;
    uint8_t* a;
    uint32_t* out;
    hipMalloc(&a, bytes + 64);
    hipMalloc(&out, 64);
    hipMemset(a, 1, bytes + 64);
    const size_t nlines = bytes / 64;
    std::vector<uint32_t> perm(nlines);
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < nlines; ++i) perm[i] = (uint32_t)i;
    for (size_t i = nlines; i > 1; --i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        std::swap(perm[i - 1], perm[s % i]);
    }
    uint32_t* dperm;
    hipMalloc(&dperm, nlines * 4);
    hipMemcpy(dperm, perm.data(), nlines * 4, hipMemcpyHostToDevice);
    // the row pattern: 4096 images, 1800 keypoints each
    const int nimg = (int)std::min<size_t>(4096, bytes / (640 * 480)), nkp = nimg * 1800;
    std::vector<uint32_t> kps(nkp);
    for (int i = 0; i < nkp; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        kps[i] = ((uint32_t)(i / 1800) << 20) | (uint32_t)(s & 0xFFFFF);
    }
    uint32_t* dkp;
    hipMalloc(&dkp, (size_t)nkp * 4);
    hipMemcpy(dkp, kps.data(), (size_t)nkp * 4, hipMemcpyHostToDevice);
    // distinct 64-B lines the row pattern touches (host count)
    std::vector<uint8_t> touched((size_t)nimg * 640 * 480 / 64 + 16, 0);
    size_t nt = 0;
    for (int i = 0; i < nkp; ++i) {
        const uint32_t k = kps[i];
        const int img = (int)(k >> 20) % nimg, u = (int)((k >> 9) & 511) + 64, v = (int)(k & 511) % 460 + 10;
        for (int r = -5; r <= 5; ++r) {
            const int64_t base = (int64_t)img * 640 * 480 + (int64_t)(v + r) * 640;
            const int64_t segs[2][2] = {{(base + u - 5) & ~3, 16}, {(base + u - 40) & ~3, 24}};
            for (auto& sg : segs)
                for (int64_t l = sg[0] / 64; l <= (sg[0] + sg[1] - 1) / 64; ++l)
                    if (!touched[l]) { touched[l] = 1; ++nt; }
        }
    }
    hipDeviceSynchronize();
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, (const uint4*)a, bytes / 16, out);
        hipLaunchKernelGGL(k_gather, dim3(4096), dim3(256), 0, 0, a, dperm, nlines, out);
        hipLaunchKernelGGL(k_rows, dim3((nkp + 255) / 256), dim3(256), 0, 0, a, nimg, dkp, nkp, out);
    }
    hipDeviceSynchronize();
    std::printf("{\"stream_bytes\": %zu, \"gather_bytes\": %zu, \"rows_distinct_line_bytes\": %zu, "
                "\"rows_loaded_bytes\": %zu}\n", bytes, bytes, nt * 64, (size_t)nkp * 11 * 40);
    return 0;
}
