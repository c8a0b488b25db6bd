// Elementwise piece of the Vecchia Fisher information (vecchia_fisher.h): the D^-1 (dD_k B^-T z - dB_k Sigma z)
// term of re_model_template.h:9266-9267 over probe-interleaved n x t blocks. HBM-bound (4 n t + 2 n doubles).
#include <hip/hip_runtime.h>

#include "common.h"

namespace gpb_amd {
namespace {

__global__ void __launch_bounds__(256) fisher_mix_kernel(int n, int t, const double* __restrict__ Do,
                                                         const double* __restrict__ dD, const double* __restrict__ U,
                                                         const double* __restrict__ W, double* __restrict__ Y) {
  const size_t total = (size_t)n * t;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const size_t i = e / (size_t)t;
    Y[e] = Do[i] * fma(dD[i], W[e], -U[e]);
  }
}

}  // namespace

void launch_fisher_mix(int n, int t, const double* Do, const double* dD, const double* U, const double* W, double* Y,
                       hipStream_t s) {
  const size_t total = (size_t)n * t;
  if (total == 0) return;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(fisher_mix_kernel, dim3(blocks), dim3(256), 0, s, n, t, Do, dD, U, W, Y);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
