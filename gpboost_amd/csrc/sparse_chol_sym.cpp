// Symbolic analysis of the sparse Cholesky of Sigma^-1 + W = B^T D^-1 B + W (sparse_chol.h): ordering,
// elimination tree, supernodes, front structures and the level schedule. Host work, once per model.
//
// The reference runs Eigen's SimplicialLLT::analyzePattern (AMD ordering, likelihoods.h:2946-2948). The
// factor is unique, so the ordering is free; this one is chosen for the GPU: nested dissection gives a
// balanced supernodal tree (many independent fronts per level at the bottom, few large dense fronts at
// the top that run on the MFMA GEMM).
#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "sparse_chol.h"

namespace gpb_amd {
namespace {

struct Graph {   // CSR adjacency without self loops
  std::vector<int64_t> ptr;
  std::vector<int> adj;
};

// The graph of B^T D^-1 B: i ~ j iff i and j lie in one clique {r} U N(r).
void build_graph(int n, int m, const int* nbr, Graph& g) {
  // cliques containing each vertex: its own row and the rows that list it as a neighbour
  std::vector<int> cnt(n + 1, 0);
  auto kcnt = [&](int i) { return std::min(i, m); };
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < kcnt(i); ++r) {
      const int j = nbr[(size_t)i * m + r];
      if (j >= 0) ++cnt[j + 1];
    }
  std::vector<int> tptr(n + 1, 0);
  for (int j = 0; j < n; ++j) tptr[j + 1] = tptr[j] + cnt[j + 1];
  std::vector<int> trow(std::max(tptr[n], 1));
  std::vector<int> fill(tptr.begin(), tptr.end() - 1);
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < kcnt(i); ++r) {
      const int j = nbr[(size_t)i * m + r];
      if (j >= 0) trow[fill[j]++] = i;
    }
  std::vector<int> deg(n, 0);
  std::vector<std::vector<int>> lists(n);
#pragma omp parallel
  {
    std::vector<int> mark(n, -1);
#pragma omp for schedule(dynamic, 512)
    for (int v = 0; v < n; ++v) {
      std::vector<int>& out = lists[v];
      mark[v] = v;
      auto take_clique = [&](int r) {
        if (mark[r] != v) { mark[r] = v; out.push_back(r); }
        for (int q = 0; q < kcnt(r); ++q) {
          const int w = nbr[(size_t)r * m + q];
          if (w >= 0 && mark[w] != v) { mark[w] = v; out.push_back(w); }
        }
      };
      take_clique(v);
      for (int e = tptr[v]; e < tptr[v + 1]; ++e) take_clique(trow[e]);
      std::sort(out.begin(), out.end());
      deg[v] = (int)out.size();
    }
  }
  g.ptr.assign(n + 1, 0);
  for (int v = 0; v < n; ++v) g.ptr[v + 1] = g.ptr[v] + deg[v];
  g.adj.resize(std::max<int64_t>(g.ptr[n], 1));
#pragma omp parallel for schedule(static)
  for (int v = 0; v < n; ++v) {
    std::copy(lists[v].begin(), lists[v].end(), g.adj.begin() + g.ptr[v]);
    std::vector<int>().swap(lists[v]);
  }
}

// Nested dissection: split V at the coordinate median along its widest axis, separate the halves by
// the boundary vertices of the side with fewer of them (every crossing edge has an endpoint there),
// recurse, order the separator last.
struct ND {
  int n, d;
  const double* X;
  const Graph& g;
  int leaf;
  std::vector<int> tag, side;
  std::vector<int> order;
  int serial = 0;
  ND(int n_, int d_, const double* X_, const Graph& g_, int leaf_)
      : n(n_), d(d_), X(X_), g(g_), leaf(leaf_), tag(n_, -1), side(n_, 0) {
    order.reserve(n_);
  }

  void run(std::vector<int>& V) {
    if ((int)V.size() <= leaf) {
      order.insert(order.end(), V.begin(), V.end());
      return;
    }
    // widest axis of the bounding box
    int axis = 0;
    double best = -1.;
    for (int q = 0; q < d; ++q) {
      double lo = X[(size_t)V[0] * d + q], hi = lo;
      for (int v : V) {
        const double x = X[(size_t)v * d + q];
        lo = std::min(lo, x);
        hi = std::max(hi, x);
      }
      if (hi - lo > best) { best = hi - lo; axis = q; }
    }
    // median split (ties broken by index: deterministic)
    std::vector<int> W(V);
    const size_t half = W.size() / 2;
    auto key_less = [&](int a, int b) {
      const double xa = d > 0 ? X[(size_t)a * d + axis] : 0., xb = d > 0 ? X[(size_t)b * d + axis] : 0.;
      return xa < xb || (xa == xb && a < b);
    };
    std::nth_element(W.begin(), W.begin() + half, W.end(), key_less);
    const int me = serial++;
    for (size_t k = 0; k < W.size(); ++k) {
      tag[W[k]] = me;
      side[W[k]] = k < half ? 0 : 1;
    }
    // boundary vertices of each side
    std::vector<int> bnd[2];
    for (int v : V) {
      for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) {
        const int w = g.adj[e];
        if (tag[w] == me && side[w] != side[v]) { bnd[side[v]].push_back(v); break; }
      }
    }
    const int sep_side = bnd[0].size() <= bnd[1].size() ? 0 : 1;
    const int sep_tag = -2 - me;   // separator vertices leave the recursion
    for (int v : bnd[sep_side]) tag[v] = sep_tag;
    std::vector<int> sub[2];
    for (int v : V)
      if (tag[v] == me) sub[side[v]].push_back(v);
    std::vector<int> S = bnd[sep_side];
    std::vector<int>().swap(V);
    std::vector<int>().swap(W);
    for (int h = 0; h < 2; ++h) run(sub[h]);
    std::sort(S.begin(), S.end());
    order.insert(order.end(), S.begin(), S.end());
  }
};

}  // namespace

void chol_finish_plan(CholPlan& P);

void chol_analyze(int n, int m, const int* nbr, int d, const double* X, int leaf, CholPlan& P) {
  const auto t0 = std::chrono::steady_clock::now();
  P = CholPlan();
  P.n = n;
  if (n <= 0) return;
  Graph g;
  build_graph(n, m, nbr, g);

  // ---- ordering
  std::vector<int> ord;
  {
    ND nd(n, d, X, g, std::max(leaf, 1));
    std::vector<int> V(n);
    std::iota(V.begin(), V.end(), 0);
    nd.run(V);
    ord.swap(nd.order);
  }
  std::vector<int> ip(n);
  for (int k = 0; k < n; ++k) ip[ord[k]] = k;

  // ---- elimination tree (Liu, path compression) of the permuted matrix
  std::vector<int> parent(n, -1), anc(n, -1);
  for (int k = 0; k < n; ++k) {
    const int v = ord[k];
    for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) {
      int j = ip[g.adj[e]];
      if (j >= k) continue;
      while (j != -1 && j < k) {
        const int nx = anc[j];
        anc[j] = k;
        if (nx == -1) parent[j] = k;
        j = nx;
      }
    }
  }
  // ---- postorder (children in ascending order), composed into the ordering
  std::vector<int> post(n);
  {
    std::vector<int> head(n, -1), next(n, -1);
    for (int j = n - 1; j >= 0; --j)
      if (parent[j] != -1) { next[j] = head[parent[j]]; head[parent[j]] = j; }
    std::vector<int> stack;
    int k = 0;
    for (int r = 0; r < n; ++r) {
      if (parent[r] != -1) continue;
      stack.push_back(r);
      while (!stack.empty()) {
        const int p = stack.back();
        const int c = head[p];
        if (c == -1) {
          stack.pop_back();
          post[k++] = p;
        } else {
          head[p] = next[c];
          stack.push_back(c);
        }
      }
    }
  }
  P.perm.resize(n);
  P.iperm.resize(n);
  {
    std::vector<int> newpos(n);
    for (int k = 0; k < n; ++k) newpos[post[k]] = k;
    std::vector<int> par2(n, -1);
    for (int k = 0; k < n; ++k) {
      P.perm[k] = ord[post[k]];
      par2[k] = parent[post[k]] == -1 ? -1 : newpos[parent[post[k]]];
    }
    parent.swap(par2);
    for (int k = 0; k < n; ++k) P.iperm[P.perm[k]] = k;
  }
  const std::vector<int>& iperm = P.iperm;
  const std::vector<int>& perm = P.perm;

  // ---- column counts by row subtrees (entries below the diagonal)
  std::vector<int> cc(n, 0), mark(n, -1);
  for (int k = 0; k < n; ++k) {
    mark[k] = k;
    const int v = perm[k];
    for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) {
      int j = iperm[g.adj[e]];
      if (j >= k) continue;
      while (mark[j] != k) {
        mark[j] = k;
        ++cc[j];
        j = parent[j];
      }
    }
  }
  // ---- fundamental supernodes
  std::vector<int> nchild(n, 0);
  for (int j = 0; j < n; ++j)
    if (parent[j] != -1) ++nchild[parent[j]];
  std::vector<int> f_first;   // fundamental supernodes' first columns
  for (int j = 0; j < n; ++j) {
    const bool cont = j > 0 && parent[j - 1] == j && cc[j - 1] == cc[j] + 1 && nchild[j] == 1;
    if (!cont) f_first.push_back(j);
  }
  const int nf = (int)f_first.size();
  f_first.push_back(n);
  std::vector<int> fsup(n);
  for (int s = 0; s < nf; ++s)
    for (int j = f_first[s]; j < f_first[s + 1]; ++j) fsup[j] = s;
  // ---- relaxed amalgamation (CHOLMOD's rule: merge a child into its parent when the merged
  // supernode stays small or the explicit zeros stay a small fraction)
  std::vector<int> first(nf), last(nf), nr(nf), par(nf, -1), rep(nf);
  std::vector<double> zeros(nf, 0.);
  std::vector<int> ends_at(n + 1, -1);   // supernode whose last column + 1 == c
  for (int s = 0; s < nf; ++s) {
    first[s] = f_first[s];
    last[s] = f_first[s + 1];
    const int ns = last[s] - first[s];
    nr[s] = cc[first[s]] - (ns - 1);
    const int pc = parent[last[s] - 1];
    par[s] = pc == -1 ? -1 : fsup[pc];
    rep[s] = s;
    ends_at[last[s]] = s;
  }
  auto merge_ok = [](int ns, double nz_total, double z) {
    if (ns <= 4) return true;
    const double frac = z / nz_total;
    if (ns <= 16) return frac < 0.8;
    if (ns <= 48) return frac < 0.1;
    if (ns <= 256) return frac < 0.05;
    return false;
  };
  std::vector<char> alive(nf, 1);
  auto find_rep = [&](int s) {
    while (rep[s] != s) s = rep[s];
    return s;
  };
  for (int p = 0; p < nf; ++p) {
    for (;;) {
      const int c = ends_at[first[p]];
      if (c < 0 || !alive[c] || par[c] < 0 || find_rep(par[c]) != p) break;
      const int nsc = last[c] - first[c], nsp = last[p] - first[p];
      const int ns = nsc + nsp;
      const double z = zeros[c] + zeros[p] + (double)nsc * (nsp + nr[p] - nr[c]);
      const double tot = 0.5 * ns * (ns + 1.) + (double)ns * nr[p];
      if (!merge_ok(ns, tot, z)) break;
      // merge c into p
      alive[c] = 0;
      first[p] = first[c];
      zeros[p] = z;
      ends_at[last[c]] = -1;
      rep[c] = p;
    }
  }
  // survivors in column order (first columns ascending); parents follow from the elimination tree
  std::vector<int> sid(nf, -1);
  int ns_total = 0;
  std::vector<int> sfirst;
  {
    std::vector<std::pair<int, int>> surv;
    for (int s = 0; s < nf; ++s)
      if (alive[s]) surv.emplace_back(first[s], s);
    std::sort(surv.begin(), surv.end());
    for (size_t k = 0; k < surv.size(); ++k) {
      sid[surv[k].second] = (int)k;
      sfirst.push_back(surv[k].first);
    }
    ns_total = (int)surv.size();
  }
  sfirst.push_back(n);
  P.nsup = ns_total;
  P.sfirst = sfirst;
  P.col_sup.resize(n);
  for (int s = 0; s < P.nsup; ++s)
    for (int j = P.sfirst[s]; j < P.sfirst[s + 1]; ++j) P.col_sup[j] = s;
  P.sparent.assign(P.nsup, -1);
  for (int s = 0; s < P.nsup; ++s) {
    const int pc = parent[P.sfirst[s + 1] - 1];
    P.sparent[s] = pc == -1 ? -1 : P.col_sup[pc];
  }

  // ---- row structures R_s: A's entries below the supernode plus the children's structures
  std::vector<std::vector<int>> kids(P.nsup);
  for (int s = 0; s < P.nsup; ++s)
    if (P.sparent[s] >= 0) kids[P.sparent[s]].push_back(s);
  P.rptr.assign(P.nsup + 1, 0);
  std::vector<std::vector<int>> R(P.nsup);
  std::fill(mark.begin(), mark.end(), -1);
  for (int s = 0; s < P.nsup; ++s) {
    const int f = P.sfirst[s], l = P.sfirst[s + 1];
    std::vector<int>& out = R[s];
    for (int j = f; j < l; ++j) {
      const int v = perm[j];
      for (int64_t e = g.ptr[v]; e < g.ptr[v + 1]; ++e) {
        const int i = iperm[g.adj[e]];
        if (i >= l && mark[i] != s) { mark[i] = s; out.push_back(i); }
      }
    }
    for (int c : kids[s])
      for (int i : R[c])
        if (i >= l && mark[i] != s) { mark[i] = s; out.push_back(i); }
    std::sort(out.begin(), out.end());
    P.rptr[s + 1] = P.rptr[s] + (int64_t)out.size();
  }
  P.rows.resize(std::max<int64_t>(P.rptr[P.nsup], 1));
  for (int s = 0; s < P.nsup; ++s) std::copy(R[s].begin(), R[s].end(), P.rows.begin() + P.rptr[s]);
  // ---- fronts, levels, statistics
  P.foff.assign(P.nsup + 1, 0);
  std::vector<int> height(P.nsup, 0);
  for (int s = 0; s < P.nsup; ++s) {
    const int64_t fs = P.fs(s), ns = P.ns(s), nrr = P.nr(s);
    P.foff[s + 1] = P.foff[s] + fs * fs;
    P.nnz_l += ns * (ns + 1) / 2 + ns * nrr;
    P.flops += (double)ns * ns * ns / 3. + (double)ns * ns * nrr + (double)ns * nrr * nrr;
    P.max_fs = std::max<int>(P.max_fs, (int)fs);
    P.max_ns = std::max<int>(P.max_ns, (int)ns);
    for (int c : kids[s]) height[s] = std::max(height[s], height[c] + 1);
  }
  P.front_doubles = P.foff[P.nsup];
  const int nlev = P.nsup ? *std::max_element(height.begin(), height.end()) + 1 : 0;
  P.lvl_ptr.assign(nlev + 1, 0);
  for (int s = 0; s < P.nsup; ++s) ++P.lvl_ptr[height[s] + 1];
  for (int l = 0; l < nlev; ++l) P.lvl_ptr[l + 1] += P.lvl_ptr[l];
  P.lvl_sup.resize(P.nsup);
  {
    std::vector<int> pos(P.lvl_ptr.begin(), P.lvl_ptr.end() - 1);
    for (int s = 0; s < P.nsup; ++s) P.lvl_sup[pos[height[s]]++] = s;
  }
  chol_finish_plan(P);
  P.ms_analyze = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}


// ---------------------------------------------------------------------------------------------------
// Schedules. Every launch of the numeric phases is one CholOp over the tasks of one tree level: the
// factorization runs the levels leaves-first (children's update blocks are complete before a parent
// assembles), the selected inverse root-first (a child reads its parent's finished S block).
namespace {

constexpr int kSplitK = 512;        // K chunk of the selected inverse's long products
constexpr int kSplitKSolve = 256;   // K chunk of the backward solve's transposed products
constexpr int64_t kSmallPanel = 64 * 1024;   // fs x ns of the largest panel a single-workgroup level sweep takes

CholGemmTask gemm_task(int bufa, int64_t a, int lda, int bufb, int64_t b, int ldb, int bufc, int64_t c, int ldc, int M,
                       int N, int K, int flags, int doff, double alpha, double beta) {
  CholGemmTask t;
  t.a = a; t.b = b; t.c = c;
  t.lda = lda; t.ldb = ldb; t.ldc = ldc;
  t.M = M; t.N = N; t.K = K;
  t.flags = flags | cg_bufs(bufa, bufb, bufc);
  t.doff = doff;
  t.alpha = alpha; t.beta = beta;
  return t;
}

struct OpBuilder {
  CholSchedule& S;
  explicit OpBuilder(CholSchedule& s) : S(s) {}
  int type = -1;
  int64_t t0 = 0;
  int64_t count(int ty) const {
    return ty == kOpDiag ? (int64_t)S.diag.size() : ty == kOpGemm ? (int64_t)S.gemm.size()
                          : ty == kOpReduce ? (int64_t)S.red.size() : (int64_t)S.col.size();
  }
  void begin(int ty) {
    type = ty;
    t0 = count(ty);
  }
  void end() {
    const int64_t t1 = count(type);
    if (t1 > t0) S.ops.push_back(CholOp{type, (int)(t1 - t0), t0});
  }
};

int level_maxblk(const CholPlan& P, int l) {
  int mb = 0;
  for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) mb = std::max(mb, P.nblk(P.lvl_sup[q]));
  return mb;
}

void build_factor_schedule(const CholPlan& P, CholSchedule& S) {
  S = CholSchedule();
  OpBuilder ob(S);
  const int nlev = (int)P.lvl_ptr.size() - 1;
  for (int l = 0; l < nlev; ++l) {
    ob.begin(kOpAsmTile);   // every lower 64 x 64 tile of the level's fronts: the children's update blocks
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q], fs = P.fs(s);
      for (int ct = 0; ct < fs; ct += 64)
        for (int rt = ct; rt < fs; rt += 64) S.col.push_back(CholColTask{s, rt, ct, 0});
    }
    ob.end();
    ob.begin(kOpAsmEntries);   // + A's entries (and W) of the panel columns
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q], ns = P.ns(s);
      for (int j0 = 0; j0 < ns; j0 += 16) S.col.push_back(CholColTask{s, j0, std::min(j0 + 16, ns), 0});
    }
    ob.end();
    const int mb = level_maxblk(P, l);
    for (int k = 0; k < mb; ++k) {
      ob.begin(kOpDiag);
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0);
        S.diag.push_back(CholDiagTask{P.foff[s] + j0 + (int64_t)j0 * fs, P.woff[s] + (int64_t)k * 4096, fs, ib});
      }
      ob.end();
      ob.begin(kOpGemm);   // TRSM: L[r0:fs, blk] = F[r0:fs, blk] W_b^T (in place)
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0), r0 = j0 + ib;
        const int64_t w = P.woff[s] + (int64_t)k * 4096;
        for (int rt = r0; rt < fs; rt += 64) {
          const int64_t c = P.foff[s] + rt + (int64_t)j0 * fs;
          S.gemm.push_back(gemm_task(kCbF, c, fs, kCbW, w, 64, kCbF, c, fs, std::min(64, fs - rt), ib, ib, kCgTB, 0,
                                     1., 0.));
        }
      }
      ob.end();
      ob.begin(kOpGemm);   // panel update: F[rt, ct] -= L[rt, blk] L[ct, blk]^T for the later panel columns
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int fs = P.fs(s), ns = P.ns(s), j0 = 64 * k, ib = std::min(64, ns - j0), r0 = j0 + ib;
        for (int ct = r0; ct < ns; ct += 64)
          for (int rt = ct; rt < fs; rt += 64) {
            const int64_t base = P.foff[s];
            S.gemm.push_back(gemm_task(kCbF, base + rt + (int64_t)j0 * fs, fs, kCbF, base + ct + (int64_t)j0 * fs, fs,
                                       kCbF, base + rt + (int64_t)ct * fs, fs, std::min(64, fs - rt),
                                       std::min(64, ns - ct), ib, kCgTB | (rt == ct ? kCgLower : 0), 0, -1., 1.));
          }
      }
      ob.end();
    }
    ob.begin(kOpGemm);   // update block: U -= L21 L21^T (K = ns)
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q];
      const int fs = P.fs(s), ns = P.ns(s);
      const int64_t base = P.foff[s];
      for (int ct = ns; ct < fs; ct += 64)
        for (int rt = ct; rt < fs; rt += 64)
          S.gemm.push_back(gemm_task(kCbF, base + rt, fs, kCbF, base + ct, fs, kCbF, base + rt + (int64_t)ct * fs, fs,
                                     std::min(64, fs - rt), std::min(64, fs - ct), ns,
                                     kCgTB | (rt == ct ? kCgLower : 0), 0, -1., 1.));
    }
    ob.end();
  }
}

void build_selinv_schedule(const CholPlan& P, CholSchedule& S) {
  S = CholSchedule();
  OpBuilder ob(S);
  const int nlev = (int)P.lvl_ptr.size() - 1;
  for (int l = nlev - 1; l >= 0; --l) {
    // scratch Y per supernode of the level (fs x 64 bound, ld = rows below the block)
    std::vector<int64_t> yoff(P.nsup, 0);
    int64_t ytot = 0;
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q];
      yoff[s] = ytot;
      ytot += (int64_t)P.fs(s) * 64;
    }
    S.y_doubles = std::max(S.y_doubles, ytot);
    ob.begin(kOpGatherS);
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q], nr = P.nr(s);
      // 8 columns per task: the top levels' few supernodes still fill the chip (64 per task left their gathers
      // on a handful of workgroups, 0.6 ms per launch)
      for (int c0 = 0; c0 < nr; c0 += 8) S.col.push_back(CholColTask{s, c0, std::min(c0 + 8, nr), 0});
    }
    ob.end();
    const int mb = level_maxblk(P, l);
    for (int k = mb - 1; k >= 0; --k) {
      ob.begin(kOpGemm);   // Y = L[R_b, b] W_b and S_bb = W_b^T W_b
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0), r0 = j0 + ib, fr = fs - r0;
        const int64_t w = P.woff[s] + (int64_t)k * 4096, base = P.foff[s];
        for (int rt = 0; rt < fr; rt += 64)
          S.gemm.push_back(gemm_task(kCbF, base + r0 + rt + (int64_t)j0 * fs, fs, kCbW, w, 64, kCbY, yoff[s] + rt, fr,
                                     std::min(64, fr - rt), ib, ib, 0, 0, 1., 0.));
        S.gemm.push_back(gemm_task(kCbW, w, 64, kCbW, w, 64, kCbS, base + j0 + (int64_t)j0 * fs, fs, ib, ib, ib, kCgTA,
                                   0, 1., 0.));
      }
      ob.end();
      // S[R_b, b] = -S[R_b, R_b] Y: split K into kSplitK chunks (partials in P, then one reduce per row tile)
      {
        std::vector<CholReduceTask> reds;
        int64_t pb = 0;
        ob.begin(kOpGemm);
        for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
          const int s = P.lvl_sup[q];
          if (P.nblk(s) <= k) continue;
          const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0), r0 = j0 + ib, fr = fs - r0;
          const int64_t base = P.foff[s];
          const int nch = (fr + kSplitK - 1) / kSplitK;
          for (int rt = 0; rt < fr; rt += 64) {
            const int M = std::min(64, fr - rt);
            for (int kc = 0; kc < nch; ++kc) {
              const int k0 = kc * kSplitK, K = std::min(kSplitK, fr - k0);
              S.gemm.push_back(gemm_task(kCbS, base + r0 + rt + (int64_t)(r0 + k0) * fs, fs, kCbY, yoff[s] + k0, fr,
                                         kCbP, pb + (int64_t)kc * 4096, 64, M, ib, K, 0, 0, 1., 0.));
            }
            CholReduceTask rd{};
            rd.c = base + r0 + rt + (int64_t)j0 * fs; rd.ldc = fs; rd.M = M; rd.N = ib; rd.bufc = kCbS;
            rd.p = pb; rd.pstride = 4096; rd.nslices = nch; rd.alpha = -1.; rd.beta = 0.;
            reds.push_back(rd);
            pb += (int64_t)nch * 4096;
          }
        }
        ob.end();
        S.p_doubles = std::max(S.p_doubles, pb);
        ob.begin(kOpReduce);
        S.red.insert(S.red.end(), reds.begin(), reds.end());
        ob.end();
      }
      // S_bb -= Y^T S[R_b, b] (split K)
      {
        std::vector<CholReduceTask> reds;
        int64_t pb = 0;
        ob.begin(kOpGemm);
        for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
          const int s = P.lvl_sup[q];
          if (P.nblk(s) <= k) continue;
          const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0), r0 = j0 + ib, fr = fs - r0;
          if (fr == 0) continue;
          const int64_t base = P.foff[s];
          const int nch = (fr + kSplitK - 1) / kSplitK;
          for (int kc = 0; kc < nch; ++kc) {
            const int k0 = kc * kSplitK, K = std::min(kSplitK, fr - k0);
            S.gemm.push_back(gemm_task(kCbY, yoff[s] + k0, fr, kCbS, base + r0 + k0 + (int64_t)j0 * fs, fs, kCbP,
                                       pb + (int64_t)kc * 4096, 64, ib, ib, K, kCgTA, 0, 1., 0.));
          }
          CholReduceTask rd{};
          rd.c = base + j0 + (int64_t)j0 * fs; rd.ldc = fs; rd.M = ib; rd.N = ib; rd.bufc = kCbS;
          rd.p = pb; rd.pstride = 4096; rd.nslices = nch; rd.alpha = -1.; rd.beta = 1.;
          reds.push_back(rd);
          pb += (int64_t)nch * 4096;
        }
        ob.end();
        S.p_doubles = std::max(S.p_doubles, pb);
        ob.begin(kOpReduce);
        S.red.insert(S.red.end(), reds.begin(), reds.end());
        ob.end();
      }
      ob.begin(kOpMirror);   // S[b, b..fs) = S[b..fs, b]^T, one task per 64-row tile
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int j0 = 64 * k, ib = std::min(64, P.ns(s) - j0);
        for (int R0 = j0; R0 < P.fs(s); R0 += 64) S.col.push_back(CholColTask{s, j0, j0 + ib, R0});
      }
      ob.end();
    }
  }
}

}  // namespace

void chol_solve_schedule(const CholPlan& P, int t, bool forward_only, CholSchedule& S, std::vector<int64_t>& vofs,
                         bool backward_only) {
  S = CholSchedule();
  OpBuilder ob(S);
  vofs.assign(P.nsup + 1, 0);
  for (int s = 0; s < P.nsup; ++s) vofs[s + 1] = vofs[s] + (int64_t)P.fs(s) * t;
  S.y_doubles = vofs[P.nsup];
  const int nlev = (int)P.lvl_ptr.size() - 1;
  // t = 1: levels whose panels are all small run one workgroup per supernode (two launches per level); the
  // levels of large separators keep the tiled form (its parallelism over row tiles).
  // GPBOOST_AMD_CHOL_SMALL_PANEL: the fs x ns bound (A/B)
  static const int64_t small_panel = [] {
    const char* e = std::getenv("GPBOOST_AMD_CHOL_SMALL_PANEL");
    return e ? std::max<int64_t>(0, std::atoll(e)) : kSmallPanel;
  }();
  std::vector<char> small(nlev, 0);
  static const bool fuse_vec = [] {   // GPBOOST_AMD_CHOL_FWDVEC=0: the two-launch tiled form for t = 1 (A/B)
    const char* e = std::getenv("GPBOOST_AMD_CHOL_FWDVEC");
    return !(e && e[0] == '0');
  }();
  if (t == 1)
    for (int l = 0; l < nlev; ++l) {
      int64_t mx = 0;
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) mx = std::max<int64_t>(mx, (int64_t)P.fs(P.lvl_sup[q]) * P.ns(P.lvl_sup[q]));
      small[l] = mx <= small_panel;
    }
  for (int l = 0; l < nlev && !backward_only; ++l) {
    if (small[l]) {
      S.ops.push_back(CholOp{kOpFSolve1, P.lvl_ptr[l + 1] - P.lvl_ptr[l], (int64_t)P.lvl_ptr[l]});
      if (forward_only) {   // the level's L^-1 b to X
        ob.begin(kOpScatterX);
        for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
          const int s = P.lvl_sup[q];
          S.col.push_back(CholColTask{s, 0, P.ns(s), 0});
        }
        ob.end();
      }
      continue;
    }
    ob.begin(kOpAsmV);
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q];
      S.col.push_back(CholColTask{s, 0, P.fs(s), 0});
    }
    ob.end();
    const int mb = level_maxblk(P, l);
    if (t == 1 && fuse_vec) {   // one launch per block step (kOpFwdVec), the level's x moved back from XS after
      for (int k = 0; k < mb; ++k) {
        ob.begin(kOpFwdVec);
        for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
          const int s = P.lvl_sup[q];
          if (P.nblk(s) <= k) continue;
          const int fs = P.fs(s), r0 = std::min(64 * (k + 1), P.ns(s));
          if (r0 >= fs) S.col.push_back(CholColTask{s, k, r0, 0});
          for (int rt = r0; rt < fs; rt += 64) S.col.push_back(CholColTask{s, k, rt, 0});
        }
        ob.end();
      }
      ob.begin(kOpCopyXS);
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        S.col.push_back(CholColTask{s, 0, P.ns(s), 0});
      }
      ob.end();
    }
    for (int k = 0; k < mb && !(t == 1 && fuse_vec); ++k) {
      ob.begin(kOpGemm);   // x_b = W_b v_b (in place)
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0);
        const int64_t w = P.woff[s] + (int64_t)k * 4096;
        for (int ct = 0; ct < t; ct += 64) {
          const int64_t v = vofs[s] + j0 + (int64_t)ct * fs;
          S.gemm.push_back(gemm_task(kCbW, w, 64, kCbY, v, fs, kCbY, v, fs, ib, std::min(64, t - ct), ib, 0, 0, 1., 0.));
        }
      }
      ob.end();
      ob.begin(kOpGemm);   // v[r0:fs] -= L[r0:fs, b] x_b
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0), r0 = j0 + ib;
        for (int ct = 0; ct < t; ct += 64)
          for (int rt = r0; rt < fs; rt += 64)
            S.gemm.push_back(gemm_task(kCbF, P.foff[s] + rt + (int64_t)j0 * fs, fs, kCbY,
                                       vofs[s] + j0 + (int64_t)ct * fs, fs, kCbY, vofs[s] + rt + (int64_t)ct * fs, fs,
                                       std::min(64, fs - rt), std::min(64, t - ct), ib, 0, 0, -1., 1.));
      }
      ob.end();
    }
    if (forward_only) {
      ob.begin(kOpScatterX);
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        S.col.push_back(CholColTask{s, 0, P.ns(s), 0});
      }
      ob.end();
    }
  }
  if (forward_only) return;
  if (backward_only) {   // the input (L^-1 b, forward-sweep layout) into every front's first ns entries
    ob.begin(kOpLoadV);
    for (int s = 0; s < P.nsup; ++s) S.col.push_back(CholColTask{s, 0, P.ns(s), 0});
    ob.end();
  }
  for (int l = nlev - 1; l >= 0; --l) {
    if (small[l]) {
      S.ops.push_back(CholOp{kOpBSolve1, P.lvl_ptr[l + 1] - P.lvl_ptr[l], (int64_t)P.lvl_ptr[l]});
      continue;
    }
    ob.begin(kOpGatherX);
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q];
      if (P.nr(s) > 0) S.col.push_back(CholColTask{s, 0, P.nr(s), 0});
    }
    ob.end();
    const int mb = level_maxblk(P, l);
    if (t == 1 && fuse_vec) {   // two launches per block step: row-chunk partials, then reduce + W_b^T per supernode
      for (int k = mb - 1; k >= 0; --k) {
        std::vector<CholColTask> fins;
        int slot = 0;
        ob.begin(kOpBwdVecPart);
        for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
          const int s = P.lvl_sup[q];
          if (P.nblk(s) <= k) continue;
          const int fr = P.fs(s) - std::min(64 * (k + 1), P.ns(s));
          const int nch = fr > 0 ? (fr + 255) / 256 : 0;
          for (int kc = 0; kc < nch; ++kc) S.col.push_back(CholColTask{s, k, kc, slot + kc});
          fins.push_back(CholColTask{s, k, nch, slot});
          slot += nch;
        }
        ob.end();
        S.p_doubles = std::max(S.p_doubles, (int64_t)slot * 64);
        ob.begin(kOpBwdVecFin);
        S.col.insert(S.col.end(), fins.begin(), fins.end());
        ob.end();
      }
    }
    for (int k = mb - 1; k >= 0 && !(t == 1 && fuse_vec); --k) {
      {   // v_b -= L[r0:fs, b]^T v[r0:fs] (split K: partials in P, then one reduce per column chunk)
        std::vector<CholReduceTask> reds;
        int64_t pb = 0;
        ob.begin(kOpGemm);
        for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
          const int s = P.lvl_sup[q];
          if (P.nblk(s) <= k) continue;
          const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0), r0 = j0 + ib, fr = fs - r0;
          if (fr == 0) continue;
          const int nch = (fr + kSplitKSolve - 1) / kSplitKSolve;
          for (int ct = 0; ct < t; ct += 64) {
            const int N = std::min(64, t - ct);
            for (int kc = 0; kc < nch; ++kc) {
              const int k0 = kc * kSplitKSolve, K = std::min(kSplitKSolve, fr - k0);
              S.gemm.push_back(gemm_task(kCbF, P.foff[s] + r0 + k0 + (int64_t)j0 * fs, fs, kCbY,
                                         vofs[s] + r0 + k0 + (int64_t)ct * fs, fs, kCbP, pb + (int64_t)kc * 4096, 64,
                                         ib, N, K, kCgTA, 0, 1., 0.));
            }
            CholReduceTask rd{};
            rd.c = vofs[s] + j0 + (int64_t)ct * fs; rd.ldc = fs; rd.M = ib; rd.N = N; rd.bufc = kCbY;
            rd.p = pb; rd.pstride = 4096; rd.nslices = nch; rd.alpha = -1.; rd.beta = 1.;
            reds.push_back(rd);
            pb += (int64_t)nch * 4096;
          }
        }
        ob.end();
        S.p_doubles = std::max(S.p_doubles, pb);
        ob.begin(kOpReduce);
        S.red.insert(S.red.end(), reds.begin(), reds.end());
        ob.end();
      }
      ob.begin(kOpGemm);   // x_b = W_b^T v_b (in place)
      for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
        const int s = P.lvl_sup[q];
        if (P.nblk(s) <= k) continue;
        const int fs = P.fs(s), j0 = 64 * k, ib = std::min(64, P.ns(s) - j0);
        const int64_t w = P.woff[s] + (int64_t)k * 4096;
        for (int ct = 0; ct < t; ct += 64) {
          const int64_t v = vofs[s] + j0 + (int64_t)ct * fs;
          S.gemm.push_back(
              gemm_task(kCbW, w, 64, kCbY, v, fs, kCbY, v, fs, ib, std::min(64, t - ct), ib, kCgTA, 0, 1., 0.));
        }
      }
      ob.end();
    }
    ob.begin(kOpScatterX);
    for (int q = P.lvl_ptr[l]; q < P.lvl_ptr[l + 1]; ++q) {
      const int s = P.lvl_sup[q];
      S.col.push_back(CholColTask{s, 0, P.ns(s), 0});
    }
    ob.end();
  }
}

void chol_finish_plan(CholPlan& P) {
  // extend-add maps and children
  P.rel.assign(std::max<int64_t>(P.rptr[P.nsup], 1), 0);
  for (int s = 0; s < P.nsup; ++s) {
    const int p = P.sparent[s];
    if (p < 0) continue;
    const int pf = P.sfirst[p], pl = P.sfirst[p + 1], nsp = pl - pf;
    const int* Rp = P.rows.data() + P.rptr[p];
    const int nrp = P.nr(p);
    for (int64_t a = P.rptr[s]; a < P.rptr[s + 1]; ++a) {
      const int i = P.rows[a];
      if (i < pl) {
        if (i < pf) Fatal("sparse Cholesky plan: row %d of supernode %d precedes its parent", i, s);
        P.rel[a] = i - pf;
      } else {
        const int* it = std::lower_bound(Rp, Rp + nrp, i);
        if (it == Rp + nrp || *it != i) Fatal("sparse Cholesky plan: row %d of supernode %d not in its parent", i, s);
        P.rel[a] = nsp + (int)(it - Rp);
      }
    }
  }
  P.cptr.assign(P.nsup + 1, 0);
  for (int s = 0; s < P.nsup; ++s)
    if (P.sparent[s] >= 0) ++P.cptr[P.sparent[s] + 1];
  for (int s = 0; s < P.nsup; ++s) P.cptr[s + 1] += P.cptr[s];
  P.child.assign(std::max(P.cptr[P.nsup], 1), 0);
  {
    std::vector<int> pos(P.cptr.begin(), P.cptr.end() - 1);
    for (int s = 0; s < P.nsup; ++s)
      if (P.sparent[s] >= 0) P.child[pos[P.sparent[s]]++] = s;
  }
  P.cinv_off.assign(P.nsup + 1, 0);
  for (int s = 0; s < P.nsup; ++s) P.cinv_off[s + 1] = P.cinv_off[s] + (P.sparent[s] >= 0 ? P.fs(P.sparent[s]) : 0);
  P.cinv.assign(std::max<int64_t>(P.cinv_off[P.nsup], 1), -1);
  for (int s = 0; s < P.nsup; ++s) {
    if (P.sparent[s] < 0) continue;
    for (int a = 0; a < P.nr(s); ++a) P.cinv[P.cinv_off[s] + P.rel[P.rptr[s] + a]] = a;
  }
  P.woff.assign(P.nsup + 1, 0);
  for (int s = 0; s < P.nsup; ++s) P.woff[s + 1] = P.woff[s] + (int64_t)P.nblk(s) * 4096;
  build_factor_schedule(P, P.factor);
  build_selinv_schedule(P, P.selinv);
}

}  // namespace gpb_amd

namespace gpb_amd {

void chol_entry_lists(const CholPlan& P, int m, const int* nbr, CholEntries& E) {
  const int n = P.n;
  if (m > 254) Fatal("sparse Cholesky: at most 254 neighbours are supported (got %d)", m);
  auto kcnt = [&](int i) { return std::min(i, m); };
  // rows of every column (elimination positions >= the column), from the cliques
  std::vector<std::vector<int>> colrows(n);
  {
    std::vector<int> cnt(n, 0);
    for (int r = 0; r < n; ++r) {
      const int k = kcnt(r);
      int q[256];
      q[0] = P.iperm[r];
      int nq = 1;
      for (int a = 0; a < k; ++a) {
        const int w = nbr[(size_t)r * m + a];
        if (w >= 0) q[nq++] = P.iperm[w];
      }
      for (int a = 0; a < nq; ++a)
        for (int b = 0; b < nq; ++b)
          if (q[a] >= q[b]) colrows[q[b]].push_back(q[a]);
    }
  }
#pragma omp parallel for schedule(dynamic, 1024)
  for (int g = 0; g < n; ++g) {
    std::vector<int>& v = colrows[g];
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
  }
  E.ecol.assign(n + 1, 0);
  for (int g = 0; g < n; ++g) E.ecol[g + 1] = E.ecol[g] + (int64_t)colrows[g].size();
  const int64_t ne = E.ecol[n];
  E.eoff.assign(ne, 0);
  E.dpos.assign(n, 0);
  std::vector<int> erow(ne);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int g = 0; g < n; ++g) {
    const int s = P.col_sup[g], f = P.sfirst[s], l = P.sfirst[s + 1], fs = P.fs(s);
    const int* R = P.rows.data() + P.rptr[s];
    const int nr = P.nr(s);
    const int jl = g - f;
    for (size_t q = 0; q < colrows[g].size(); ++q) {
      const int i = colrows[g][q];
      int pos;
      if (i < l) {
        pos = i - f;
      } else {
        const int* it = std::lower_bound(R, R + nr, i);
        if (it == R + nr || *it != i) Fatal("sparse Cholesky: entry (%d, %d) outside the factor structure", i, g);
        pos = (l - f) + (int)(it - R);
      }
      E.eoff[E.ecol[g] + q] = P.foff[s] + pos + (int64_t)jl * fs;
      erow[E.ecol[g] + q] = i;
    }
    E.dpos[g] = P.foff[s] + jl + (int64_t)jl * fs;
    std::vector<int>().swap(colrows[g]);
  }
  auto find = [&](int i, int g) -> int64_t {   // entry of (i, g), i >= g
    const int* b = erow.data() + E.ecol[g];
    const int* e = erow.data() + E.ecol[g + 1];
    const int* it = std::lower_bound(b, e, i);
    return E.ecol[g] + (it - b);
  };
  // contributions: count, then fill in row order (deterministic sums)
  E.cptr.assign(ne + 1, 0);
  for (int r = 0; r < n; ++r) {
    const int k = kcnt(r);
    int q[256];
    q[0] = P.iperm[r];
    int nq = 1;
    for (int a = 0; a < k; ++a) {
      const int w = nbr[(size_t)r * m + a];
      if (w >= 0) q[nq++] = P.iperm[w];
    }
    for (int a = 0; a < nq; ++a)
      for (int b = a; b < nq; ++b) {
        const int i = std::max(q[a], q[b]), g = std::min(q[a], q[b]);
        ++E.cptr[find(i, g) + 1];
      }
  }
  for (int64_t e = 0; e < ne; ++e) E.cptr[e + 1] += E.cptr[e];
  E.ctr.assign(std::max<int64_t>(E.cptr[ne], 1), 0);
  std::vector<int64_t> pos(E.cptr.begin(), E.cptr.end() - 1);
  for (int r = 0; r < n; ++r) {
    const int k = kcnt(r);
    int q[256], slot[256];
    q[0] = P.iperm[r];
    slot[0] = 0;
    int nq = 1;
    for (int a = 0; a < k; ++a) {
      const int w = nbr[(size_t)r * m + a];
      if (w >= 0) { slot[nq] = a + 1; q[nq++] = P.iperm[w]; }
    }
    for (int a = 0; a < nq; ++a)
      for (int b = a; b < nq; ++b) {
        const int i = std::max(q[a], q[b]), g = std::min(q[a], q[b]);
        E.ctr[pos[find(i, g)]++] = ((uint64_t)r << 16) | ((uint64_t)slot[a] << 8) | (uint64_t)slot[b];
      }
  }
}

}  // namespace gpb_amd
