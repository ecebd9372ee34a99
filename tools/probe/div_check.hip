// Bitwise check of k_pose's shared-reciprocal division (div_prep / div_by) against `a / b`:
// random doubles over the whole exponent range plus zeros, subnormals, infinities and NaNs,
// several numerators per denominator (as in eval_point / eval_line).  Build:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/probe/div_check.hip -o tools/probe/div_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

struct SharedDiv { double b, sb, r; };
__device__ __forceinline__ double div_refine(double sb) {
    double r = __builtin_amdgcn_rcp(sb);
    double t = __builtin_fma(-sb, r, 1.0);
    r = __builtin_fma(r, t, r);
    t = __builtin_fma(-sb, r, 1.0);
    return __builtin_fma(r, t, r);
}
__device__ __forceinline__ SharedDiv div_prep(double b, double a0) {
    bool f;
    const double sb = __builtin_amdgcn_div_scale(a0, b, false, &f);
    return SharedDiv{b, sb, div_refine(sb)};
}
__device__ __forceinline__ double div_by(const SharedDiv& d, double a) {
    bool f, vcc;
    const double sb = __builtin_amdgcn_div_scale(a, d.b, false, &f);
    double r = d.r;
    if (__builtin_expect(__double_as_longlong(sb) != __double_as_longlong(d.sb), 0)) r = div_refine(sb);
    const double sa = __builtin_amdgcn_div_scale(a, d.b, true, &vcc);
    const double m = sa * r;
    const double e = __builtin_fma(-sb, m, sa);
    return __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(e, r, m, vcc), d.b, a);
}

__device__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ double pick(uint64_t h) {
    const int k = (int)(h & 15);
    const uint64_t r = mix(h);
    switch (k) {
        case 0: return 0.0;
        case 1: return -0.0;
        case 2: return __longlong_as_double((long long)(r & 0x000FFFFFFFFFFFFFull));   // subnormal
        case 3: return (h & 16) ? __builtin_inf() : -__builtin_inf();
        case 4: return __longlong_as_double(0x7FF8000000000001ll);
        case 5: return __longlong_as_double((long long)(r & 0x801FFFFFFFFFFFFFull));   // tiny normal
        case 6: return __longlong_as_double((long long)((r & 0x800FFFFFFFFFFFFFull) | 0x7FE0000000000000ull));   // huge
        default: {   // moderate range, the pose's values
            const uint64_t e = 1023 - 40 + (r >> 52) % 80;
            return __longlong_as_double((long long)((r & 0x800FFFFFFFFFFFFFull) | (e << 52)));
        }
    }
}
__global__ void kcheck(uint64_t seed, int per, unsigned long long* bad, unsigned long long* total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t h = mix(seed ^ (i * 0x100000001B3ull));
    double b = pick(h);
    double a[8];
    for (int k = 0; k < 8; ++k) { h = mix(h); a[k] = pick(h); }
    const SharedDiv d = div_prep(b, a[0]);
    unsigned long long nb = 0;
    for (int k = 0; k < 8; ++k) {
        volatile double x = a[k], y = b;
        const double ref = x / y;
        const double got = div_by(d, a[k]);
        if (__double_as_longlong(ref) != __double_as_longlong(got)) {
            if (nb == 0 && atomicAdd(bad + 1, 1ull) < 4)
                printf("mismatch a %a b %a ref %a got %a\n", a[k], b, ref, got);
            ++nb;
        }
    }
    if (nb) atomicAdd(bad, nb);
    atomicAdd(total, 8ull);
}
int main() {
    unsigned long long *bad, *tot;
    hipMalloc(&bad, 16);
    hipMalloc(&tot, 8);
    hipMemset(bad, 0, 16);
    hipMemset(tot, 0, 8);
    for (int s = 0; s < 16; ++s) hipLaunchKernelGGL(kcheck, dim3(16384), dim3(256), 0, 0, (uint64_t)s * 7919u + 1, 8, bad, tot);
    unsigned long long hb[2], ht;
    hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost);
    hipMemcpy(&ht, tot, 8, hipMemcpyDeviceToHost);
    printf("div_check: %llu divisions, %llu mismatches\n", ht, hb[0]);
    return hb[0] ? 1 : 0;
}
