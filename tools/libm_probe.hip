// Diagnostic: how do gfx950 device f64 sqrt / div / acos / sin compare with the
// host glibc results the reference (Rust std -> glibc libm) would produce?
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/libm_probe.hip -o tools/libm_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

__global__ void probe(const double* __restrict__ a, const double* __restrict__ b,
                      double* __restrict__ o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = a[i], y = b[i];
  o[5 * i + 0] = sqrt(y);
  o[5 * i + 1] = x / y;
  o[5 * i + 2] = acos(x);
  o[5 * i + 3] = sin(y);
  o[5 * i + 4] = cos(y);
}

static int64_t ulpdiff(double p, double q) {
  if (std::isnan(p) && std::isnan(q)) return 0;
  int64_t a, b; memcpy(&a, &p, 8); memcpy(&b, &q, 8);
  if (a < 0) a = INT64_MIN - a;
  if (b < 0) b = INT64_MIN - b;
  return a > b ? a - b : b - a;
}

int main() {
  const int n = 1 << 22;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> ua(-1.0, 1.0), ub(1e-3, 3.1415926535897931);
  std::vector<double> a(n), b(n), o(5 * (size_t)n);
  for (int i = 0; i < n; ++i) { a[i] = ua(rng); b[i] = ub(rng); }
  // edge-ish values
  a[0] = 1.0; a[1] = -1.0; a[2] = 0.0; a[3] = 0.9999999999999999; a[4] = 1.0000000000000002;
  double *da, *db, *dout;
  hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dout, 5 * (size_t)n * 8);
  hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice);
  probe<<<(n + 255) / 256, 256>>>(da, db, dout, n);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  hipMemcpy(o.data(), dout, 5 * (size_t)n * 8, hipMemcpyDeviceToHost);
  const char* names[5] = {"sqrt", "div", "acos", "sin", "cos"};
  for (int k = 0; k < 5; ++k) {
    long mism = 0; int64_t maxu = 0;
    for (int i = 0; i < n; ++i) {
      double x = a[i], y = b[i], h;
      switch (k) { case 0: h = sqrt(y); break; case 1: h = x / y; break;
                   case 2: h = acos(x); break; case 3: h = sin(y); break; default: h = cos(y); }
      int64_t u = ulpdiff(h, o[5 * i + k]);
      if (u) { ++mism; if (u > maxu) maxu = u; }
    }
    printf("%-5s mismatches %ld / %d  (%.4f%%)  max ulp %lld\n", names[k], mism, n,
           100.0 * mism / n, (long long)maxu);
  }
  return 0;
}
