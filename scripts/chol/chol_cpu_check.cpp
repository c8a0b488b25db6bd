// Development check of the sparse Cholesky plan and its task schedules on the host (no GPU): every
// op of the factorization / selected-inverse / solve schedules executed by plain loops on a random
// matrix A = B^T D^-1 B + W with the Vecchia clique structure, compared with a dense Cholesky.
//   hipcc -O2 -fopenmp -I gpboost_amd/csrc scripts/chol/chol_cpu_check.cpp gpboost_amd/csrc/sparse_chol_sym.cpp \
//         gpboost_amd/csrc/vecchia_host.cpp -o /tmp/chol_cpu_check && /tmp/chol_cpu_check 1500 10 32
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <algorithm>
#include "sparse_chol.h"
#include "vecchia_host.h"
namespace gpb_amd {
void Fatal(const char* fmt, ...) { va_list a; va_start(a, fmt); vfprintf(stderr, fmt, a); va_end(a); fprintf(stderr, "\n"); std::exit(1); }
void Info(const char*, ...) {}
void Warning(const char*, ...) {}
}
using namespace gpb_amd;

struct Exec {
  const CholPlan& P;
  std::vector<double>& F; std::vector<double>& S; std::vector<double>& Wd; std::vector<double>& Y; std::vector<double>& Pp;
  const std::vector<double>* A;   // dense n x n (matrix labels)
  int n;
  const double* b = nullptr; double* X = nullptr; int t = 1; const std::vector<int64_t>* vofs = nullptr;
  double* buf(int id) { return id == kCbF ? F.data() : id == kCbS ? S.data() : id == kCbW ? Wd.data() : id == kCbY ? Y.data() : Pp.data(); }
  void run(const CholSchedule& sch) {
    for (const CholOp& op : sch.ops)
      for (int q = 0; q < op.ntask; ++q) {
        const int64_t ti = op.task0 + q;
        switch (op.type) {
          case kOpGemm: gemm(sch.gemm[ti]); break;
          case kOpDiag: diag(sch.diag[ti]); break;
          case kOpReduce: reduce(sch.red[ti]); break;
          case kOpFSolve1: fsolve1(P.lvl_sup[op.task0 + q]); break;
          case kOpBSolve1: bsolve1(P.lvl_sup[op.task0 + q]); break;
          default: col(op.type, sch.col[ti]);
        }
      }
  }
  void gemm(const CholGemmTask& g) {
    const double* Ab = buf((g.flags >> 4) & 7) + g.a;
    const double* Bb = buf((g.flags >> 7) & 7) + g.b;
    double* Cb = buf((g.flags >> 10) & 7) + g.c;
    const bool ta = g.flags & kCgTA, tb = g.flags & kCgTB, lo = g.flags & kCgLower;
    std::vector<double> out((size_t)g.M * g.N);
    for (int j = 0; j < g.N; ++j)
      for (int i = 0; i < g.M; ++i) {
        double s = 0.;
        for (int k = 0; k < g.K; ++k) {
          const double av = ta ? Ab[k + (size_t)i * g.lda] : Ab[i + (size_t)k * g.lda];
          const double bv = tb ? Bb[j + (size_t)k * g.ldb] : Bb[k + (size_t)j * g.ldb];
          s += av * bv;
        }
        out[i + (size_t)j * g.M] = s;
      }
    for (int j = 0; j < g.N; ++j)
      for (int i = 0; i < g.M; ++i) {
        if (lo && i - j + g.doff < 0) continue;
        double& c = Cb[i + (size_t)j * g.ldc];
        c = (g.beta == 0. ? 0. : g.beta * c) + g.alpha * out[i + (size_t)j * g.M];
      }
  }
  void fsolve1(int s) {
    const int sf = P.sfirst[s], ns = P.ns(s), fs = P.fs(s);
    double* V = Y.data() + (*vofs)[s];
    const double* L = F.data() + P.foff[s];
    for (int r = 0; r < fs; ++r) V[r] = r < ns ? b[P.perm[sf + r]] : 0.;
    for (int q = P.cptr[s]; q < P.cptr[s + 1]; ++q) {
      const int ch = P.child[q];
      for (int i = 0; i < P.nr(ch); ++i) V[P.rel[P.rptr[ch] + i]] += Y[(*vofs)[ch] + P.ns(ch) + i];
    }
    for (int k = 0; k < P.nblk(s); ++k) {
      const int j0 = 64 * k, ib = std::min(64, ns - j0);
      const double* W = Wd.data() + P.woff[s] + (int64_t)k * 4096;
      double x[64];
      for (int i = 0; i < ib; ++i) { double v = 0.; for (int j = 0; j <= i; ++j) v += W[i + j * 64] * V[j0 + j]; x[i] = v; }
      for (int i = 0; i < ib; ++i) V[j0 + i] = x[i];
      for (int r = j0 + ib; r < fs; ++r) for (int j = 0; j < ib; ++j) V[r] -= L[r + (size_t)(j0 + j) * fs] * x[j];
    }
  }
  void bsolve1(int s) {
    const int sf = P.sfirst[s], ns = P.ns(s), nr = P.nr(s), fs = P.fs(s);
    double* V = Y.data() + (*vofs)[s];
    const double* L = F.data() + P.foff[s];
    for (int i = 0; i < nr; ++i) V[ns + i] = X[P.perm[P.rows[P.rptr[s] + i]]];
    for (int k = P.nblk(s) - 1; k >= 0; --k) {
      const int j0 = 64 * k, ib = std::min(64, ns - j0), r0 = j0 + ib;
      const double* W = Wd.data() + P.woff[s] + (int64_t)k * 4096;
      double vb[64];
      for (int j = 0; j < ib; ++j) { double d = 0.; for (int r = r0; r < fs; ++r) d += L[r + (size_t)(j0 + j) * fs] * V[r]; vb[j] = V[j0 + j] - d; }
      for (int i = 0; i < ib; ++i) { double v = 0.; for (int j = i; j < ib; ++j) v += W[j + i * 64] * vb[j]; V[j0 + i] = v; }
    }
    for (int i = 0; i < ns; ++i) X[P.perm[sf + i]] = V[i];
  }
  void reduce(const CholReduceTask& r) {
    double* C = buf(r.bufc) + r.c;
    const double* Pb = Pp.data() + r.p;
    for (int j = 0; j < r.N; ++j)
      for (int i = 0; i < r.M; ++i) {
        double s = 0.;
        for (int q = 0; q < r.nslices; ++q) s += Pb[q * r.pstride + i + j * 64];
        double& c = C[i + (size_t)j * r.ldc];
        c = (r.beta == 0. ? 0. : r.beta * c) + r.alpha * s;
      }
  }
  void diag(const CholDiagTask& d) {
    double* L = F.data() + d.c;
    const int ld = d.ld, ib = d.ib;
    for (int j = 0; j < ib; ++j) {
      double p = L[j + (size_t)j * ld];
      if (!(p > 0.)) Fatal("not PD");
      p = std::sqrt(p);
      L[j + (size_t)j * ld] = p;
      for (int i = j + 1; i < ib; ++i) L[i + (size_t)j * ld] /= p;
      for (int c = j + 1; c < ib; ++c)
        for (int i = c; i < ib; ++i) L[i + (size_t)c * ld] -= L[i + (size_t)j * ld] * L[c + (size_t)j * ld];
    }
    double* W = Wd.data() + d.w;
    for (int c = 0; c < ib; ++c)
      for (int i = 0; i < ib; ++i) {
        if (i < c) { W[i + c * 64] = 0.; continue; }
        double s = (i == c) ? 1. : 0.;
        for (int p = c; p < i; ++p) s -= L[i + (size_t)p * ld] * W[p + c * 64];
        W[i + c * 64] = s / L[i + (size_t)i * ld];
      }
  }
  int rowpos(int s, int r) const {   // front row r -> elimination position
    const int ns = P.ns(s);
    return r < ns ? P.sfirst[s] + r : P.rows[P.rptr[s] + r - ns];
  }
  void col(int type, const CholColTask& c) {
    const int s = c.s, fs = P.fs(s), ns = P.ns(s), nr = P.nr(s);
    double* Fs = F.data() + P.foff[s];
    double* Ss = S.data() + P.foff[s];
    if (type == kOpAsmTile) {
      const int rt = c.c0, ct = c.c1;
      for (int j = ct; j < std::min(ct + 64, fs); ++j)
        for (int i = std::max(rt, j); i < std::min(rt + 64, fs); ++i) {
          double v = 0.;
          for (int q = P.cptr[s]; q < P.cptr[s + 1]; ++q) {
            const int ch = P.child[q], fc = P.fs(ch), nsc = P.ns(ch);
            const int ia = P.cinv[P.cinv_off[ch] + i], ib = P.cinv[P.cinv_off[ch] + j];
            if (ia >= 0 && ib >= 0) v += F[P.foff[ch] + (nsc + ia) + (size_t)(nsc + ib) * fc];
          }
          Fs[i + (size_t)j * fs] = v;
        }
    } else if (type == kOpAsmEntries) {
      for (int j = c.c0; j < c.c1; ++j) {
        const int gj = P.perm[P.sfirst[s] + j];
        for (int r = j; r < fs; ++r) Fs[r + (size_t)j * fs] += (*A)[(size_t)P.perm[rowpos(s, r)] * n + gj];
      }
    } else if (type == kOpGatherS) {
      const int p = P.sparent[s], fp = P.fs(p);
      const int* rel = P.rel.data() + P.rptr[s];
      const double* Sp = S.data() + P.foff[p];
      for (int bb = c.c0; bb < c.c1; ++bb)
        for (int a = 0; a < nr; ++a) Ss[(ns + a) + (size_t)(ns + bb) * fs] = Sp[rel[a] + (size_t)rel[bb] * fp];
    } else if (type == kOpMirror) {
      for (int j = c.c0; j < c.c1; ++j)
        for (int r = std::max(j + 1, c.pad); r < std::min(fs, c.pad + 64); ++r) Ss[j + (size_t)r * fs] = Ss[r + (size_t)j * fs];
    } else if (type == kOpAsmV) {
      double* V = Y.data() + (*vofs)[s];
      for (int k = 0; k < t; ++k) {
        for (int r = 0; r < fs; ++r) V[r + (size_t)k * fs] = r < ns ? b[P.perm[P.sfirst[s] + r] + (size_t)k * n] : 0.;
      }
      for (int q = P.cptr[s]; q < P.cptr[s + 1]; ++q) {
        const int ch = P.child[q], fc = P.fs(ch), nsc = P.ns(ch), nrc = P.nr(ch);
        const int* rel = P.rel.data() + P.rptr[ch];
        const double* Vc = Y.data() + (*vofs)[ch];
        for (int k = 0; k < t; ++k)
          for (int a = 0; a < nrc; ++a) V[rel[a] + (size_t)k * fs] += Vc[nsc + a + (size_t)k * fc];
      }
    } else if (type == kOpGatherX) {
      double* V = Y.data() + (*vofs)[s];
      for (int k = 0; k < t; ++k)
        for (int a = c.c0; a < c.c1; ++a) V[ns + a + (size_t)k * fs] = X[P.perm[P.rows[P.rptr[s] + a]] + (size_t)k * n];
    } else if (type == kOpScatterX) {
      const double* V = Y.data() + (*vofs)[s];
      for (int k = 0; k < t; ++k)
        for (int a = c.c0; a < c.c1; ++a) X[P.perm[P.sfirst[s] + a] + (size_t)k * n] = V[a + (size_t)k * fs];
    }
  }
};

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1500, m = argc > 2 ? atoi(argv[2]) : 10, leaf = argc > 3 ? atoi(argv[3]) : 32;
  const int d = 2;
  std::mt19937_64 g(7);
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
  printf("n=%d nsup=%d levels=%d factor ops=%zu gemm tasks=%zu selinv ops=%zu\n", n, P.nsup, (int)P.lvl_ptr.size() - 1,
         P.factor.ops.size(), P.factor.gemm.size(), P.selinv.ops.size());
  // random A = B^T D^-1 B + W (dense)
  std::vector<double> Bd((size_t)n * n, 0.), A((size_t)n * n, 0.), Dinv(n), W(n);
  for (int i = 0; i < n; ++i) {
    Bd[(size_t)i * n + i] = 1.;
    for (int r = 0; r < std::min(i, m); ++r) Bd[(size_t)i * n + nbr[(size_t)i * m + r]] = -0.3 * u(g);
    Dinv[i] = 0.5 + u(g);
    W[i] = 0.1 + 0.2 * u(g);
  }
  for (int r = 0; r < n; ++r)
    for (int a = 0; a < n; ++a) {
      const double ba = Bd[(size_t)r * n + a];
      if (ba == 0.) continue;
      for (int c = 0; c < n; ++c) {
        const double bc = Bd[(size_t)r * n + c];
        if (bc != 0.) A[(size_t)a * n + c] += Dinv[r] * ba * bc;
      }
    }
  for (int i = 0; i < n; ++i) A[(size_t)i * n + i] += W[i];
  // dense Cholesky + inverse
  std::vector<double> L(A);
  for (int j = 0; j < n; ++j) {
    double p = L[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) p -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
    p = std::sqrt(p);
    L[(size_t)j * n + j] = p;
    for (int i = j + 1; i < n; ++i) {
      double s = L[(size_t)i * n + j];
      for (int k = 0; k < j; ++k) s -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
      L[(size_t)i * n + j] = s / p;
    }
  }
  double ld_dense = 0.;
  for (int j = 0; j < n; ++j) ld_dense += 2. * std::log(L[(size_t)j * n + j]);
  std::vector<double> F(P.front_doubles, 7.), S(P.front_doubles, 0.), Wd(P.woff[P.nsup], 0.), Yb(std::max<int64_t>(P.selinv.y_doubles, 1), 0.);
  std::vector<double> Pp(std::max<int64_t>(std::max(P.selinv.p_doubles, P.factor.p_doubles), 1), 0.);
  Exec ex{P, F, S, Wd, Yb, Pp, &A, n};
  ex.run(P.factor);
  double ld = 0.;
  for (int s = 0; s < P.nsup; ++s)
    for (int j = 0; j < P.ns(s); ++j) ld += 2. * std::log(F[P.foff[s] + j + (size_t)j * P.fs(s)]);
  printf("logdet sparse %.15g dense %.15g rel %.2e\n", ld, ld_dense, std::fabs(ld - ld_dense) / std::fabs(ld_dense));
  // solve with t = 3
  const int t = 3;
  std::vector<double> bvec((size_t)n * t), xs((size_t)n * t, 0.);
  for (auto& v : bvec) v = u(g) - 0.5;
  std::vector<int64_t> vofs;
  CholSchedule ss;
  chol_solve_schedule(P, t, false, ss, vofs);
  std::vector<double> V(ss.y_doubles, 0.);
  std::vector<double> Pv(std::max<int64_t>(ss.p_doubles, 1), 0.);
  Exec ev{P, F, S, Wd, V, Pv, &A, n, bvec.data(), xs.data(), t, &vofs};
  ev.run(ss);
  double res = 0., nb = 0.;
  for (int k = 0; k < t; ++k)
    for (int i = 0; i < n; ++i) {
      double s = 0.;
      for (int j = 0; j < n; ++j) s += A[(size_t)i * n + j] * xs[j + (size_t)k * n];
      res = std::max(res, std::fabs(s - bvec[i + (size_t)k * n]));
      nb = std::max(nb, std::fabs(bvec[i + (size_t)k * n]));
    }
  printf("solve residual max %.2e (|b| %.2e)\n", res, nb);
  {   // t = 1 (hybrid schedule: per-supernode level sweeps + tiled levels)
    std::vector<int64_t> vo1;
    CholSchedule s1;
    chol_solve_schedule(P, 1, false, s1, vo1);
    std::vector<double> V1(s1.y_doubles, 0.), P1(std::max<int64_t>(s1.p_doubles, 1), 0.), x1(n, 0.);
    int nf = 0;
    for (auto& o : s1.ops) nf += o.type == kOpFSolve1;
    Exec e1{P, F, S, Wd, V1, P1, &A, n, bvec.data(), x1.data(), 1, &vo1};
    e1.run(s1);
    double r1 = 0.;
    for (int i = 0; i < n; ++i) { double s2 = 0.; for (int j = 0; j < n; ++j) s2 += A[(size_t)i * n + j] * x1[j]; r1 = std::max(r1, std::fabs(s2 - bvec[i])); }
    printf("t=1 solve residual max %.2e (%d single-workgroup levels, %zu launches)\n", r1, nf, s1.ops.size());
  }
  // selected inverse vs dense inverse (columns of A^-1 by dense solves)
  ex.run(P.selinv);
  std::vector<double> Ainv((size_t)n * n);
  for (int c = 0; c < n; ++c) {
    std::vector<double> z(n, 0.);
    z[c] = 1.;
    for (int i = 0; i < n; ++i) { double s = z[i]; for (int k = 0; k < i; ++k) s -= L[(size_t)i * n + k] * z[k]; z[i] = s / L[(size_t)i * n + i]; }
    for (int i = n - 1; i >= 0; --i) { double s = z[i]; for (int k = i + 1; k < n; ++k) s -= L[(size_t)k * n + i] * z[k]; z[i] = s / L[(size_t)i * n + i]; }
    for (int i = 0; i < n; ++i) Ainv[(size_t)i * n + c] = z[i];
  }
  double err = 0., mx = 0.;
  long cnt = 0;
  for (int s = 0; s < P.nsup; ++s) {
    const int fs = P.fs(s), ns = P.ns(s);
    for (int j = 0; j < ns; ++j)
      for (int r = j; r < fs; ++r) {
        const int pr = r < ns ? P.sfirst[s] + r : P.rows[P.rptr[s] + r - ns];
        const int pc = P.sfirst[s] + j;
        const double sv = S[P.foff[s] + r + (size_t)j * fs];
        const double dv = Ainv[(size_t)P.perm[pr] * n + P.perm[pc]];
        err = std::max(err, std::fabs(sv - dv));
        mx = std::max(mx, std::fabs(dv));
        ++cnt;
      }
  }
  printf("selected inverse: %ld entries, max abs err %.2e (max |S| %.2e)\n", cnt, err, mx);
  // entry lists: A's values from the clique contributions against the dense A
  CholEntries E;
  chol_entry_lists(P, m, nbr.data(), E);
  double eerr = 0.;
  std::vector<double> Fx(P.front_doubles, 0.);
  for (int gcol = 0; gcol < n; ++gcol)
    for (int64_t e = E.ecol[gcol]; e < E.ecol[gcol + 1]; ++e) {
      double v = 0.;
      for (int64_t c = E.cptr[e]; c < E.cptr[e + 1]; ++c) {
        const int r = (int)(E.ctr[c] >> 16), a = (int)((E.ctr[c] >> 8) & 255), b = (int)(E.ctr[c] & 255);
        const double ba = a == 0 ? 1. : Bd[(size_t)r * n + nbr[(size_t)r * m + a - 1]];
        const double bb = b == 0 ? 1. : Bd[(size_t)r * n + nbr[(size_t)r * m + b - 1]];
        v += Dinv[r] * ba * bb;
      }
      Fx[E.eoff[e]] = v;
    }
  for (int gcol = 0; gcol < n; ++gcol) Fx[E.dpos[gcol]] += W[P.perm[gcol]];
  // compare with the dense A at every lower position of the fronts' panels
  for (int s = 0; s < P.nsup; ++s) {
    const int fs = P.fs(s), ns = P.ns(s);
    for (int j = 0; j < ns; ++j)
      for (int r = j; r < fs; ++r) {
        const int pr = r < ns ? P.sfirst[s] + r : P.rows[P.rptr[s] + r - ns];
        const double dv = A[(size_t)P.perm[pr] * n + P.perm[P.sfirst[s] + j]];
        eerr = std::max(eerr, std::fabs(Fx[P.foff[s] + r + (size_t)j * fs] - dv));
      }
  }
  printf("entry lists: %lld entries, %lld contributions, max abs err vs dense A %.2e\n", (long long)E.ecol[n],
         (long long)E.cptr[E.ecol[n]], eerr);
  return 0;
}
// (entry-list check appended: compile with -DENTRY_CHECK)
