// Microbenchmark: does data written by one kernel stay in the writing XCD's L2 for the next
// kernel on the same stream? Block b writes an 8 KB chunk; the next kernel's block b reads its
// own chunk (same blockIdx -> same XCD under round-robin dispatch) or block b+1's (another XCD).
// Run under rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum; the program checks every value read.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kBlocks = 2048, kChunk = 1024;   // doubles per block: 8 KB, 16 MB in total (2 MB per XCD)

__global__ void write_kernel(double* buf, int gen) {
  double* c = buf + (size_t)blockIdx.x * kChunk;
  for (int i = threadIdx.x; i < kChunk; i += 256) c[i] = gen * 1e6 + blockIdx.x * 1e3 + i;
}
__global__ void read_kernel(const double* buf, int shift, int gen, double* out, int* bad) {
  const int src = (blockIdx.x + shift) % kBlocks;
  const double* c = buf + (size_t)src * kChunk;
  double s = 0.;
  for (int i = threadIdx.x; i < kChunk; i += 256) {
    const double v = c[i];
    if (v != gen * 1e6 + src * 1e3 + i) atomicAdd(bad, 1);
    s += v;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

int main() {
  double *buf, *out;
  int* bad;
  if (hipMalloc(&buf, sizeof(double) * kBlocks * kChunk) != hipSuccess) return 1;
  if (hipMalloc(&out, sizeof(double) * kBlocks) != hipSuccess) return 1;
  if (hipMalloc(&bad, sizeof(int)) != hipSuccess) return 1;
  (void)hipMemset(bad, 0, sizeof(int));
  for (int rep = 0; rep < 3; ++rep) {
    int gen = 2 * rep + 1;
    hipLaunchKernelGGL(write_kernel, dim3(kBlocks), dim3(256), 0, 0, buf, gen);
    hipLaunchKernelGGL(read_kernel, dim3(kBlocks), dim3(256), 0, 0, buf, 0, gen, out, bad);   // same XCD
    ++gen;
    hipLaunchKernelGGL(write_kernel, dim3(kBlocks), dim3(256), 0, 0, buf, gen);
    hipLaunchKernelGGL(read_kernel, dim3(kBlocks), dim3(256), 0, 0, buf, 1, gen, out, bad);   // neighbour XCD
  }
  int h = 0;
  (void)hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
  std::printf("mismatches: %d\n", h);
  return h != 0;
}
