// Probe: are f64 sqrt / div and f32 div correctly rounded on gfx950 with -ffp-contract=off?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>
#include <cstring>

__global__ void k(const double* a, const double* b, double* s, double* d,
                  const float* fa, const float* fb, float* fd, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    s[i] = sqrt(a[i]);
    d[i] = a[i] / b[i];
    fd[i] = fa[i] / fb[i];
  }
}

static uint64_t sm(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> a(n), b(n), s(n), d(n);
  std::vector<float> fa(n), fb(n), fd(n);
  uint64_t st = 1;
  for (int i = 0; i < n; ++i) {
    double u = (sm(st) >> 11) * 0x1.0p-53, v = (sm(st) >> 11) * 0x1.0p-53;
    a[i] = std::ldexp(u + 0.5, (int)(sm(st) % 200) - 100);
    b[i] = std::ldexp(v + 0.5, (int)(sm(st) % 200) - 100);
    fa[i] = (float)std::ldexp(u + 0.5, (int)(sm(st) % 60) - 30);
    fb[i] = (float)std::ldexp(v + 0.5, (int)(sm(st) % 60) - 30);
  }
  double *da, *db, *ds, *dd; float *dfa, *dfb, *dfd;
  hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&ds, n * 8); hipMalloc(&dd, n * 8);
  hipMalloc(&dfa, n * 4); hipMalloc(&dfb, n * 4); hipMalloc(&dfd, n * 4);
  hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dfa, fa.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dfb, fb.data(), n * 4, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(da, db, ds, dd, dfa, dfb, dfd, n);
  hipMemcpy(s.data(), ds, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(d.data(), dd, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(fd.data(), dfd, n * 4, hipMemcpyDeviceToHost);
  long bs = 0, bd = 0, bf = 0;
  for (int i = 0; i < n; ++i) {
    double cs = std::sqrt(a[i]), cd = a[i] / b[i]; float cf = fa[i] / fb[i];
    if (std::memcmp(&cs, &s[i], 8)) ++bs;
    if (std::memcmp(&cd, &d[i], 8)) ++bd;
    if (std::memcmp(&cf, &fd[i], 4)) ++bf;
  }
  printf("f64 sqrt mismatches %ld / %d\nf64 div mismatches %ld / %d\nf32 div mismatches %ld / %d\n", bs, n, bd, n, bf, n);
  return (bs || bd || bf) ? 1 : 0;
}
