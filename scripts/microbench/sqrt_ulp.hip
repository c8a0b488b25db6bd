// Accuracy of the hardware v_sqrt_f64 (and of one Newton correction on it) against the correctly
// rounded sqrt, on the squared-distance range of the row kernel. Prints the max |ulp| error.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k(int n, const double* x, double* hw, double* hw1, double* ref) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double s = x[i];
  const double h = __builtin_amdgcn_sqrt(s);
  hw[i] = h;
  // one Newton / Heron correction: h + (s - h^2) / (2h) with the residual by FMA
  const double r = fma(-h, h, s);
  hw1[i] = fma(r, 0.5 * __builtin_amdgcn_rcp(h), h);
  ref[i] = sqrt(s);
}

static double ulps(double a, double b) {
  int64_t ia, ib;
  memcpy(&ia, &a, 8); memcpy(&ib, &b, 8);
  return (double)llabs(ia - ib);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) * 0x1.0p-53;
    x[i] = std::ldexp(1.0 + u, (int)(s % 40) - 36);   // squared distances ~2^-36 .. 2^4
  }
  double *dx, *dh, *dh1, *dr;
  hipMalloc(&dx, n * 8); hipMalloc(&dh, n * 8); hipMalloc(&dh1, n * 8); hipMalloc(&dr, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, n, dx, dh, dh1, dr);
  std::vector<double> h(n), h1(n), r(n);
  hipMemcpy(h.data(), dh, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(h1.data(), dh1, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0, mr = 0;
  for (int i = 0; i < n; ++i) {
    const double c = std::sqrt(x[i]);
    m0 = fmax(m0, ulps(h[i], c)); m1 = fmax(m1, ulps(h1[i], c)); mr = fmax(mr, ulps(r[i], c));
  }
  printf("max ulp: v_sqrt_f64 %.0f, +1 correction %.0f, device sqrt() %.0f\n", m0, m1, mr);
  return 0;
}
