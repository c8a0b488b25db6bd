// Host-only statistics of the sparse Cholesky plan (symbolic analysis) for synthetic Vecchia data:
//   hipcc -O2 -fopenmp -I gpboost_amd/csrc scripts/chol/chol_stats.cpp gpboost_amd/csrc/sparse_chol_sym.cpp
//         gpboost_amd/csrc/vecchia_host.cpp -o /tmp/chol_stats && /tmp/chol_stats 100000 30 64
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <algorithm>
#include "sparse_chol.h"
#include "vecchia_host.h"
namespace gpb_amd {
void Fatal(const char* fmt, ...) { va_list a; va_start(a, fmt); vfprintf(stderr, fmt, a); va_end(a); std::exit(1); }
void Info(const char*, ...) {}
void Warning(const char*, ...) {}
}
using namespace gpb_amd;
int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 100000, m = argc > 2 ? atoi(argv[2]) : 30, leaf = argc > 3 ? atoi(argv[3]) : 64;
  const int d = 2;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(0., 1.);
  std::vector<double> X0((size_t)n * d);
  for (auto& x : X0) x = u(g);
  std::vector<int> perm = vecchia_order(n, 0, true);
  std::vector<double> X((size_t)n * d);
  for (int i = 0; i < n; ++i) for (int q = 0; q < d; ++q) X[(size_t)i * d + q] = X0[(size_t)perm[i] * d + q];
  std::vector<int> nbr((size_t)n * m);
  vecchia_neighbors(X.data(), n, d, m, 0, n, nbr.data());
  CholPlan P;
  chol_analyze(n, m, nbr.data(), d, X.data(), leaf, P);
  printf("n=%d m=%d leaf=%d: nsup=%d levels=%d nnzL=%.1fM fronts=%.1fM doubles flops=%.2f GF max_fs=%d max_ns=%d analyze %.0f ms\n",
         n, m, leaf, P.nsup, (int)P.lvl_ptr.size() - 1, P.nnz_l / 1e6, P.front_doubles / 1e6, P.flops / 1e9, P.max_fs, P.max_ns, P.ms_analyze);
  const int nl = (int)P.lvl_ptr.size() - 1;
  for (int l = 0; l < nl; ++l) {
    int cnt = P.lvl_ptr[l + 1] - P.lvl_ptr[l];
    int mxf = 0, mxn = 0; double fl = 0, fr = 0; long sn = 0;
    for (int k = P.lvl_ptr[l]; k < P.lvl_ptr[l + 1]; ++k) {
      int s = P.lvl_sup[k]; double ns = P.ns(s), nr = P.nr(s);
      mxf = std::max(mxf, P.fs(s)); mxn = std::max(mxn, P.ns(s)); sn += P.ns(s);
      fl += ns * ns * ns / 3 + ns * ns * nr + ns * nr * nr; fr += (ns + nr) * (ns + nr);
    }
    printf("  level %3d: %6d fronts, cols %7ld, max fs %5d max ns %5d, %.3f GF, fronts %.1fM\n", l, cnt, sn, mxf, mxn, fl / 1e9, fr / 1e6);
  }
  // histogram of ns / fs
  int hist[8] = {0};
  for (int s = 0; s < P.nsup; ++s) { int f = P.fs(s); int b = f <= 64 ? 0 : f <= 128 ? 1 : f <= 256 ? 2 : f <= 512 ? 3 : f <= 1024 ? 4 : f <= 2048 ? 5 : 6; hist[b]++; }
  printf("fs histogram <=64:%d <=128:%d <=256:%d <=512:%d <=1024:%d <=2048:%d >2048:%d\n", hist[0], hist[1], hist[2], hist[3], hist[4], hist[5], hist[6]);
  return 0;
}
