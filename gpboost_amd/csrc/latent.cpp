// LatentVecchia implementation: host orchestration of the iterative latent-Vecchia path.
#include "latent.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <map>
#include <cstring>

#include "slq_host.h"

namespace gpb_amd {

namespace {
constexpr double kJitterMultVecchia = 1. + 1e-10;   // JITTER_MULT_VECCHIA (utils.h)
constexpr double kCArmijo = 1e-4;                   // c_armijo_ (likelihoods.h:12737)
// ZERO_RHS_CG_THRESHOLD = 1e-100 on sum|rhs| (utils.h:45, CG_utils.cpp:42-45); tested here as
// sum rhs^2 < 1e-200, which is implied by it and differs only below ~1e-100 magnitudes.
constexpr double kZeroRhsSq = 1e-200;
constexpr int kOutDoubles = 1024;
}  // namespace

namespace {
// Optional phase timing (GPBOOST_AMD_TIMING=1): device time of preconditioner applications,
// operator applications and the rest, printed once per evaluation.
struct PhaseTimer {
  bool on = std::getenv("GPBOOST_AMD_TIMING") != nullptr;
  hipEvent_t a = nullptr, b = nullptr;
  double ms[4] = {0, 0, 0, 0};
  int cnt[4] = {0, 0, 0, 0};
  void begin(hipStream_t s) {
    if (!on) return;
    if (!a) { (void)hipEventCreate(&a); (void)hipEventCreate(&b); }
    (void)hipEventRecord(a, s);
  }
  void end(hipStream_t s, int k) {
    if (!on) return;
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float x = 0.f;
    (void)hipEventElapsedTime(&x, a, b);
    ms[k] += x;
    ++cnt[k];
  }
};
PhaseTimer g_timer;
}  // namespace

LatentVecchia::LatentVecchia(int n, int d, int m, const double* d_X, const int* nbr, hipStream_t stream)
    : n_(n), d_(d), m_(m), d_X_(d_X), s_(stream) {
  HIP_CHECK(hipEventCreate(&ev0_));
  HIP_CHECK(hipEventCreate(&ev1_));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_out_), kOutDoubles * sizeof(double), hipHostMallocDefault));
  std::vector<int> nbr_p;
  Relabel(nbr, nbr_p);
  BuildStructure(nbr_p.data());
  for (auto* b : {&d_Bv_, &d_dBv_}) b->alloc((size_t)n * m);
  for (auto* b : {&d_y_, &d_Dinv_, &d_dD_, &d_W_, &d_dw_, &d_sdw_, &d_d1_, &d_mode_, &d_mode_upd_, &d_mode_new_,
                  &d_rhs_, &d_dir_, &d_Adir_, &d_vS_, &d_dmll_})
    b->alloc(n);
  d_out_.alloc(kOutDoubles);
}

LatentVecchia::~LatentVecchia() {
  for (GraphEntry& g : graphs_) (void)hipGraphExecDestroy(g.exec);
  for (GraphEntry& g : hgraphs_) (void)hipGraphExecDestroy(g.exec);
  if (h_out_) (void)hipHostFree(h_out_);
  if (ev0_) (void)hipEventDestroy(ev0_);
  if (ev1_) (void)hipEventDestroy(ev1_);
}

namespace {
// 2-D / 3-D Morton key of a point in the unit-scaled bounding box (21 bits per axis).
uint64_t spread_bits(uint64_t v, int dims) {
  uint64_t r = 0;
  for (int b = 0; b < 21; ++b) r |= ((v >> b) & 1ull) << (b * dims);
  return r;
}
}  // namespace

// Storage relabelling for locality. The latent problem is solved in a symmetric permutation
// of the Vecchia order: storage row p holds Vecchia row vo_[p]. Rows 0..m-1 keep their
// labels (so k_p = min(p, m) still gives each row's neighbour count), rows >= m follow the
// Morton (Z-order) curve of their coordinates, so a row's neighbours — spatially close
// points — sit close in storage and the neighbour gathers of the operator, the solves and
// the trace kernels hit L2 instead of streaming from HBM / MALL. Every quantity the path
// returns (nll, gradient, log-determinants, CG coefficients) is invariant under the
// relabelling up to summation order. GPBOOST_AMD_NO_RELABEL keeps the Vecchia order (A/B).
void LatentVecchia::Relabel(const int* nbr, std::vector<int>& nbr_p) {
  const int n = n_, m = m_, d = d_;
  vo_.resize(n);
  lab_.resize(n);
  for (int i = 0; i < n; ++i) vo_[i] = i;
  const int m0 = std::min(m, n);
  std::vector<double> X((size_t)n * d);   // the caller's upload runs on our (non-blocking) stream
  HIP_CHECK(hipMemcpyAsync(X.data(), d_X_, sizeof(double) * X.size(), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  if (std::getenv("GPBOOST_AMD_NO_RELABEL") == nullptr && n > m0 && d >= 1 && d <= 3) {
    std::vector<double> lo(d, 0.), hi(d, 0.);
    for (int q = 0; q < d; ++q) {
      lo[q] = hi[q] = X[q];
      for (int i = 1; i < n; ++i) {
        lo[q] = std::min(lo[q], X[(size_t)i * d + q]);
        hi[q] = std::max(hi[q], X[(size_t)i * d + q]);
      }
    }
    std::vector<uint64_t> key(n, 0);
    for (int i = m0; i < n; ++i) {
      uint64_t k = 0;
      for (int q = 0; q < d; ++q) {
        const double w = hi[q] > lo[q] ? (X[(size_t)i * d + q] - lo[q]) / (hi[q] - lo[q]) : 0.;
        const uint64_t c = (uint64_t)(std::min(std::max(w, 0.), 1.) * 2097151.);
        k |= spread_bits(c, d) << q;
      }
      key[i] = k;
    }
    std::stable_sort(vo_.begin() + m0, vo_.end(), [&](int a, int b) { return key[a] < key[b]; });
  }
  for (int p = 0; p < n; ++p) lab_[vo_[p]] = p;
  nbr_p.assign((size_t)n * m, 0);
  for (int p = 0; p < n; ++p) {
    const int i = vo_[p];
    const int k = std::min(i, m);
    for (int r = 0; r < k; ++r) nbr_p[(size_t)p * m + r] = lab_[nbr[(size_t)i * m + r]];
  }
  d_Xp_.alloc((size_t)n * d);
  std::vector<double> Xp((size_t)n * d);
  for (int p = 0; p < n; ++p)
    for (int q = 0; q < d; ++q) Xp[(size_t)p * d + q] = X[(size_t)vo_[p] * d + q];
  HIP_CHECK(hipMemcpyAsync(d_Xp_.get(), Xp.data(), sizeof(double) * Xp.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

// Host construction of the B^T lists and the level sets of both triangular solves (in the
// storage labels of Relabel). Level of a row in the lower solve: 1 + max level of its
// neighbours (all earlier Vecchia rows); level of column j in the B^T (unit upper) solve:
// 1 + max level of the rows that have j as a neighbour. Rows inside a level are
// independent. Level recursions walk the rows in Vecchia order (lab_ = storage label of
// each Vecchia row).
void LatentVecchia::BuildStructure(const int* nbr) {
  const int n = n_, m = m_;
  std::vector<int> cnt(n + 1, 0);
  for (int i = 0; i < n; ++i) {
    const int k = std::min(i, m);
    for (int r = 0; r < k; ++r) ++cnt[nbr[(size_t)i * m + r] + 1];
  }
  std::vector<int> tptr(n + 1, 0);
  for (int j = 0; j < n; ++j) tptr[j + 1] = tptr[j] + cnt[j + 1];
  const int nnz = tptr[n];
  std::vector<int> trow(std::max(nnz, 1)), tslot(std::max(nnz, 1)), fill(tptr.begin(), tptr.end() - 1);
  for (int i = 0; i < n; ++i) {   // ascending i -> rows ascending within each column
    const int k = std::min(i, m);
    for (int r = 0; r < k; ++r) {
      const int j = nbr[(size_t)i * m + r];
      trow[fill[j]] = i;
      tslot[fill[j]] = i * m + r;
      ++fill[j];
    }
  }
  std::vector<int> lf(n, 0), lb(n, 0);
  int Lf = 0, Lb = 0;
  for (int ii = 0; ii < n; ++ii) {
    const int i = lab_[ii];   // storage label of Vecchia row ii
    const int k = std::min(i, m);
    int l = 0;
    for (int r = 0; r < k; ++r) l = std::max(l, lf[nbr[(size_t)i * m + r]] + 1);
    lf[i] = l;
    Lf = std::max(Lf, l + 1);
  }
  for (int ii = n - 1; ii >= 0; --ii) {
    const int i = lab_[ii];   // storage label of Vecchia row ii
    const int k = std::min(i, m);
    for (int r = 0; r < k; ++r) {
      const int j = nbr[(size_t)i * m + r];
      lb[j] = std::max(lb[j], lb[i] + 1);
    }
    Lb = std::max(Lb, lb[i] + 1);
  }
  auto bucket = [n](const std::vector<int>& lev, int L, std::vector<int>& ptr, std::vector<int>& rows) {
    ptr.assign(L + 1, 0);
    for (int i = 0; i < n; ++i) ++ptr[lev[i] + 1];
    for (int l = 0; l < L; ++l) ptr[l + 1] += ptr[l];
    std::vector<int> f(ptr.begin(), ptr.end() - 1);
    rows.resize(n);
    for (int i = 0; i < n; ++i) rows[f[lev[i]]++] = i;
  };
  std::vector<int> frows, brows;
  bucket(lf, Lf, fptr_, frows);
  bucket(lb, Lb, bptr_, brows);
  BuildSweepPlan(nbr, tptr, trow, tslot, lf, lb);
  BuildHeadPlan(nbr, tptr, trow, tslot, lb);

  d_nbr_.alloc((size_t)n * m);
  d_tptr_.alloc(n + 1);
  d_trow_.alloc(trow.size());
  d_tslot_.alloc(tslot.size());
  HIP_CHECK(hipMemcpyAsync(d_nbr_.get(), nbr, sizeof(int) * (size_t)n * m, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_tptr_.get(), tptr.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_trow_.get(), trow.data(), sizeof(int) * trow.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_tslot_.get(), tslot.data(), sizeof(int) * tslot.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  sp_.n = n;
  sp_.m = m;
  sp_.nbr = d_nbr_.get();
  sp_.tptr = d_tptr_.get();
  sp_.trow = d_trow_.get();
  sp_.tslot = d_tslot_.get();
  tnnz_ = nnz;
  d_tval_.alloc(trow.size());
  sp_.tval = d_tval_.get();
  sp_.tval_of = nullptr;   // set once the values of an evaluation are gathered
  std::vector<int> longr;
  for (int j = 0; j < n; ++j)
    if (tptr[j + 1] - tptr[j] > kLongRow) longr.push_back(j);
  d_longr_.alloc(std::max<size_t>(longr.size(), 1));
  if (!longr.empty())
    HIP_CHECK(hipMemcpy(d_longr_.get(), longr.data(), sizeof(int) * longr.size(), hipMemcpyHostToDevice));
  sp_.longr = d_longr_.get();
  sp_.nlong = (int)longr.size();
}

void LatentVecchia::SetY(const double* y_vo) {
  std::vector<double> yp(n_);
  for (int p = 0; p < n_; ++p) yp[p] = y_vo[vo_[p]];
  HIP_CHECK(hipMemcpyAsync(d_y_.get(), yp.data(), sizeof(double) * n_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  y_set_ = true;
}

LatentVecchia::Block& LatentVecchia::GetBlock(int which, int t, int pmax) {
  std::unique_ptr<Block>& bp = which == 0 ? blk1_ : (which == 1 ? blkt_ : blkb_);
  if (!bp) bp.reset(new Block());
  Block& b = *bp;
  if (b.t != t) {
    const size_t nt = (size_t)n_ * t;
    for (auto* buf : {&b.R, &b.Z, &b.H, &b.V, &b.G, &b.Xt}) buf->alloc(nt);
    b.small.alloc((size_t)6 * t);
    b.act.alloc(t);
    b.t = t;
  }
  if (b.a_hist.size() < (size_t)pmax * t) {
    b.a_hist.alloc((size_t)pmax * t);
    b.b_hist.alloc((size_t)pmax * t);
  }
  const size_t need = (size_t)kMaxRedBlocks * std::max(kGradCols * t, (int)kLatentScalars);
  if (d_partials_.size() < need) d_partials_.alloc(need);
  if (d_out_.size() < (size_t)kGradCols * t) d_out_.alloc((size_t)kGradCols * t);
  return b;
}

void LatentVecchia::EnsureProbes(const IterativeConfig& cfg) {
  const int t = cfg.num_rand_vec_trace;
  if (probes_saved_ && probes_t_ == t) return;
  // GenRandVecNormalParallel (CG_utils.cpp:930-947), drawn once when reuse_rand_vec_trace
  std::vector<double> R((size_t)n_ * t);
  {   // drawn in Vecchia order (the reference's), stored in the relabelled rows
    std::vector<double> Rv((size_t)n_ * t);
    gen_probes_normal(n_, t, cfg.seed_rand_vec_trace, probe_run_id_, Rv.data());
    for (int p = 0; p < n_; ++p)
      std::copy(Rv.begin() + (size_t)vo_[p] * t, Rv.begin() + (size_t)(vo_[p] + 1) * t, R.begin() + (size_t)p * t);
  }
  ++probe_run_id_;
  d_probes_.alloc((size_t)n_ * t);
  d_Zp_.alloc((size_t)n_ * t);
  d_U_.alloc((size_t)n_ * t);
  d_P_.alloc((size_t)n_ * t);
  HIP_CHECK(hipMemcpyAsync(d_probes_.get(), R.data(), sizeof(double) * R.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  probes_t_ = t;
  probes_saved_ = cfg.reuse_rand_vec_trace;
}

void LatentVecchia::BenchOperators(int t, int reps, double* out) {
  if (!factor_ready_) Fatal("BenchOperators needs a previous evaluation (the factor of its parameters)");
  if (t < 1 || reps < 1) Fatal("BenchOperators: t and reps must be >= 1");
  Block& b = GetBlock(2, t, 1);
  const size_t nt = (size_t)n_ * t;
  HIP_CHECK(hipMemsetAsync(b.R.get(), 0, sizeof(double) * nt, s_));   // finite inputs (timing only)
  HIP_CHECK(hipMemsetAsync(b.H.get(), 0, sizeof(double) * nt, s_));
  ApplyA(b.H.get(), b.V.get(), b.G.get(), t);              // warm (and graph capture below)
  PrecondImpl(b.R.get(), b.Z.get(), b.Xt.get(), t);
  float ms = 0.f;
  HIP_CHECK(hipEventRecord(ev0_, s_));
  for (int r = 0; r < reps; ++r) ApplyA(b.H.get(), b.V.get(), b.G.get(), t);
  HIP_CHECK(hipEventRecord(ev1_, s_));
  HIP_CHECK(hipEventSynchronize(ev1_));
  HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
  out[0] = ms / reps;
  HIP_CHECK(hipEventRecord(ev0_, s_));
  for (int r = 0; r < reps; ++r) PrecondImpl(b.R.get(), b.Z.get(), b.Xt.get(), t);
  HIP_CHECK(hipEventRecord(ev1_, s_));
  HIP_CHECK(hipEventSynchronize(ev1_));
  HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
  out[1] = ms / reps;
  if (precond_mode_ == 4 && std::getenv("GPBOOST_AMD_PRECOND_SPLIT")) {   // diagnostics: per-part cost
    const double* dw = d_dw_.get();
    double* R = b.R.get();
    double* Xt = b.Xt.get();
    double* Z = b.Z.get();
    auto part = [&](const char* name, auto fn) {
      float pm = 0.f;
      HIP_CHECK(hipEventRecord(ev0_, s_));
      for (int r = 0; r < reps; ++r) fn();
      HIP_CHECK(hipEventRecord(ev1_, s_));
      HIP_CHECK(hipEventSynchronize(ev1_));
      HIP_CHECK(hipEventElapsedTime(&pm, ev0_, ev1_));
      std::fprintf(stderr, "[precond split t=%d] %-12s %.4f ms\n", t, name, pm / reps);
    };
    part("tail_bt", [&] { TailSolve(false, R, Xt, Z, t); });
    part("head_part", [&] { launch_vadu_head_partial(hpart_, R, Xt, t, s_); });
    part("head_bt", [&] { launch_vadu_head(hbt_, false, dw, nullptr, Xt, t, s_); });
    part("head_lower", [&] { launch_vadu_head(hlow_, true, dw, Xt, Z, t, s_); });
    part("tail_lower", [&] { TailSolve(true, R, Xt, Z, t); });
    std::fprintf(stderr, "[precond split t=%d] K=%d passes lower=%d bt=%d tail levels bt=%d lower=%d\n", t, head_K_,
                 hlow_.npass, hbt_.npass, tplan_.nlev_b, tplan_.nlev - tplan_.nlev_b);
  }
  out[2] = (double)tnnz_ + n_;
  out[3] = precond_mode_ != 4 ? lplan_.nlev
           : (tail_tiles_ ? (int)(sup_b_.size() + sup_f_.size()) - 2 : tplan_.nlev) + 3;   // dependent launches per application
}

// V = (B^T D^-1 B + W) H   (CG_utils.cpp:75, 161-164)
void LatentVecchia::ApplyA(const double* H, double* V, double* G, int t) {
  g_timer.begin(s_);
  launch_b_apply(sp_, d_Bv_.get(), true, H, t, d_Dinv_.get(), G, s_);
  launch_bt_apply(sp_, d_Bv_.get(), true, G, t, nullptr, d_W_.get(), H, V, s_);
  g_timer.end(s_, t == 1 ? 2 : 3);
}

// Step plan for the VADU sweep kernel: rows in level order, each level cut into steps of at
// most kSweepRows rows / kSweepEnts entries, each step one contiguous blob (SweepPlan).
void LatentVecchia::BuildSweepPlan(const int* nbr, const std::vector<int>& tptr, const std::vector<int>& trow,
                                   const std::vector<int>& tslot, const std::vector<int>& lf,
                                   const std::vector<int>& lb) {
  const int n = n_, m = m_;
  std::vector<int> blob, step_off, vpos, eslot;
  int max_words = 4;
  auto entries_of = [&](bool lower, int row, std::vector<int>& idx, std::vector<int>& slot) {
    idx.clear();
    slot.clear();
    if (lower) {
      const int k = std::min(row, m);
      for (int r = 0; r < k; ++r) { idx.push_back(nbr[(size_t)row * m + r]); slot.push_back(row * m + r); }
    } else {
      for (int e = tptr[row]; e < tptr[row + 1]; ++e) { idx.push_back(trow[e]); slot.push_back(tslot[e]); }
    }
  };
  std::vector<int> idx, slot;
  std::vector<int> lrows, beoff(1, 0), beidx, beslot, fidx, fslot, crit;
  lplan_.lptr.assign(1, 0);
  for (int phase = 0; phase < 2; ++phase) {
    const bool lower = phase == 1;
    const std::vector<int>& lev = lower ? lf : lb;
    // rows by level (stable by index)
    int L = 0;
    for (int i = 0; i < n; ++i) L = std::max(L, lev[i] + 1);
    std::vector<std::vector<int>> by_level(L);
    for (int i = 0; i < n; ++i) by_level[lev[i]].push_back(i);
    for (int l = 0; l < L; ++l) {
      const std::vector<int>& rows = by_level[l];
      for (int r : rows) {
        entries_of(lower, r, idx, slot);
        lrows.push_back(r);
        {   // the dependency finished last in level order: the sync-free solve polls it first
          int best = -1, bl = -1;
          for (int d : idx) {
            const int dl = lev[d];
            if (dl > bl) { bl = dl; best = d; }
          }
          crit.push_back(best);
        }
        if (lower) {   // fixed stride m, zero-value padding (slot -1)
          for (int q = 0; q < m; ++q) {
            fidx.push_back(q < (int)idx.size() ? idx[q] : 0);
            fslot.push_back(q < (int)idx.size() ? slot[q] : -1);
          }
        } else {
          beidx.insert(beidx.end(), idx.begin(), idx.end());
          beslot.insert(beslot.end(), slot.begin(), slot.end());
          beoff.push_back((int)beidx.size());
        }
      }
      lplan_.lptr.push_back((int)lrows.size());
      size_t q = 0;
      while (q < rows.size()) {
        // greedily take rows while both limits hold
        std::vector<int> srows;
        std::vector<int> sidx, sslot, soff(1, 0);
        while (q < rows.size() && (int)srows.size() < kSweepRows) {
          entries_of(lower, rows[q], idx, slot);
          if ((int)idx.size() > kSweepEnts) Fatal("Vecchia row with %d dependents exceeds the sweep step capacity", (int)idx.size());
          if (!srows.empty() && (int)(sidx.size() + idx.size()) > kSweepEnts) break;
          srows.push_back(rows[q]);
          sidx.insert(sidx.end(), idx.begin(), idx.end());
          sslot.insert(sslot.end(), slot.begin(), slot.end());
          soff.push_back((int)sidx.size());
          ++q;
        }
        const int R = (int)srows.size(), E = (int)sidx.size();
        const int base = (int)blob.size();
        int v0 = kSweepHdr + 2 * R + 1;
        v0 += v0 & 1;                                  // fp64 values 8-byte aligned
        int words = v0 + 3 * E;
        words = (words + 3) & ~3;                      // next blob 16-byte aligned
        blob.resize(base + words, 0);
        blob[base + 0] = R;
        blob[base + 1] = E;
        blob[base + 2] = v0;
        blob[base + 3] = words;
        blob[base + 5] = lower ? 1 : 0;
        if (!step_off.empty()) blob[step_off.back() + 4] = words;   // previous blob: size of this one
        std::copy(srows.begin(), srows.end(), blob.begin() + base + kSweepHdr);
        std::copy(soff.begin(), soff.end(), blob.begin() + base + kSweepHdr + R);
        std::copy(sidx.begin(), sidx.end(), blob.begin() + base + v0 + 2 * E);
        for (int e = 0; e < E; ++e) {
          vpos.push_back((base + v0) / 2 + e);         // index in the blob viewed as fp64
          eslot.push_back(sslot[e]);
        }
        step_off.push_back(base);
        max_words = std::max(max_words, words);
      }
    }
  }
  lplan_.nlev = (int)lplan_.lptr.size() - 1;
  lplan_.n = n;
  lplan_.m = m;
  lplan_.nlev_b = 0;
  for (int i = 0; i < n; ++i) lplan_.nlev_b = std::max(lplan_.nlev_b, lb[i] + 1);
  // value slots of both phases in one refresh gather: [beslot | fslot]
  std::vector<int> lslot(beslot);
  lslot.insert(lslot.end(), fslot.begin(), fslot.end());
  lplan_entries_ = (int)lslot.size();
  d_lrows_.alloc(lrows.size());
  h_crit_ = crit;
  d_crit_.alloc(crit.size());
  HIP_CHECK(hipMemcpyAsync(d_crit_.get(), crit.data(), sizeof(int) * crit.size(), hipMemcpyHostToDevice, s_));
  d_beoff_.alloc(beoff.size());
  d_beidx_.alloc(std::max<size_t>(beidx.size(), 1));
  d_fidx_.alloc(std::max<size_t>(fidx.size(), 1));
  d_lslot_.alloc(std::max<size_t>(lslot.size(), 1));
  d_lval_.alloc(std::max<size_t>(lslot.size(), 1));
  HIP_CHECK(hipMemcpyAsync(d_lrows_.get(), lrows.data(), sizeof(int) * lrows.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_beoff_.get(), beoff.data(), sizeof(int) * beoff.size(), hipMemcpyHostToDevice, s_));
  if (!beidx.empty())
    HIP_CHECK(hipMemcpyAsync(d_beidx_.get(), beidx.data(), sizeof(int) * beidx.size(), hipMemcpyHostToDevice, s_));
  if (!fidx.empty())
    HIP_CHECK(hipMemcpyAsync(d_fidx_.get(), fidx.data(), sizeof(int) * fidx.size(), hipMemcpyHostToDevice, s_));
  if (!lslot.empty())
    HIP_CHECK(hipMemcpyAsync(d_lslot_.get(), lslot.data(), sizeof(int) * lslot.size(), hipMemcpyHostToDevice, s_));
  lplan_.lrows = d_lrows_.get();
  lplan_.beoff = d_beoff_.get();
  lplan_.beidx = d_beidx_.get();
  lplan_.beval = d_lval_.get();
  lplan_.fidx = d_fidx_.get();
  lplan_.fval = d_lval_.get() + beslot.size();
  use_graph_ = std::getenv("GPBOOST_AMD_SWEEP_KERNEL") == nullptr;
  if (const char* pm = std::getenv("GPBOOST_AMD_PRECOND")) precond_mode_ = std::atoi(pm);
  if (!use_graph_) precond_mode_ = 2;
  {
    int dev = 0, cus = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    max_flow_blocks_ = 2 * std::max(cus, 1);   // 2 x 256-thread blocks per CU: all resident
    sf_grid_ = std::max(cus, 1);                  // one single-wave workgroup per CU
    if (const char* g = std::getenv("GPBOOST_AMD_SF_GRID")) sf_grid_ = std::max(1, std::atoi(g));
  }
  d_err_.alloc(4);
  HIP_CHECK(hipMemsetAsync(d_err_.get(), 0, sizeof(int) * 4, s_));
  plan_.nsteps = (int)step_off.size();
  plan_.first_words = step_off.empty() ? 0 : blob[3];
  // each LDS buffer is a whole number of 64-word wave slices (staging writes full slices)
  plan_.max_words = (max_words + 63) & ~63;
  plan_entries_ = (int)vpos.size();
  if ((size_t)2 * plan_.max_words * sizeof(int) > 160 * 1024) Fatal("sweep plan exceeds the LDS capacity");
  blob.resize(blob.size() + 64, 0);                  // staging of the (empty) step after the last
  d_blob_.alloc(blob.size());
  d_vpos_.alloc(std::max<size_t>(vpos.size(), 1));
  d_eslot_.alloc(std::max<size_t>(eslot.size(), 1));
  HIP_CHECK(hipMemcpyAsync(d_blob_.get(), blob.data(), sizeof(int) * blob.size(), hipMemcpyHostToDevice, s_));
  if (!vpos.empty()) {
    HIP_CHECK(hipMemcpyAsync(d_vpos_.get(), vpos.data(), sizeof(int) * vpos.size(), hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipMemcpyAsync(d_eslot_.get(), eslot.data(), sizeof(int) * eslot.size(), hipMemcpyHostToDevice, s_));
  }
  HIP_CHECK(hipStreamSynchronize(s_));
  plan_.blob = d_blob_.get();
}

// Head/tail plan of the two solves (precond mode 4; vadu_head.hip explains the split).
// Head = storage rows whose Vecchia index is < K. In the lower solve a head row depends only
// on head rows (its neighbours are earlier); in the B^T solve a tail row depends only on tail
// rows (the rows that have it as a neighbour are later). So: lower = head kernel, then the
// tail levels (levels over tail dependencies only; head values are final by then); B^T = the
// tail levels (the full-DAG levels lb, exact for tail rows), then the tail contributions to
// the head rows (one launch), then the head kernel over head-only dependencies.
void LatentVecchia::BuildHeadPlan(const int* nbr, const std::vector<int>& tptr, const std::vector<int>& trow,
                                  const std::vector<int>& tslot, const std::vector<int>& lb) {
  const int n = n_, m = m_;
  int K = 14336;   // 112 KB of LDS per column workgroup (K sweep 12288 / 14336 / 16384: 1.741 / 1.719 / 1.732 ms at t = 51)
  if (const char* e = std::getenv("GPBOOST_AMD_HEAD_ROWS")) K = std::atoi(e);
  K = std::max(0, std::min(std::min(K, kHeadMaxRows), n));
  head_K_ = K;
  const int nt = n - K;
  auto head = [&](int p) { return vo_[p] < K; };
  std::vector<int> ints;       // every index array of the plan, one upload
  std::vector<int> vslot;      // value slots into Bv (-1: zero padding), one gather per evaluation
  auto put = [&](const std::vector<int>& v) { const size_t at = ints.size(); ints.insert(ints.end(), v.begin(), v.end()); return at; };
  // ---- tail level plan
  std::vector<int> lt(n, 0);
  int Lb = 0, Lt = 0;
  for (int ii = K; ii < n; ++ii) {
    const int i = lab_[ii];
    const int k = std::min(i, m);
    int l = 0;
    for (int r = 0; r < k; ++r) {
      const int j = nbr[(size_t)i * m + r];
      if (!head(j)) l = std::max(l, lt[j] + 1);
    }
    lt[i] = l;
    Lt = std::max(Lt, l + 1);
    Lb = std::max(Lb, lb[i] + 1);
  }
  auto by_level = [&](const std::vector<int>& lev, int L) {
    std::vector<std::vector<int>> b(L);
    for (int p = 0; p < n; ++p)
      if (!head(p)) b[lev[p]].push_back(p);
    return b;
  };
  std::vector<std::vector<int>> groups_b = by_level(lb, Lb), groups_f = by_level(lt, Lt);
  std::vector<int> item_off;
  // tile-blocked schedule of the tail (launch_vadu_tile): rows regrouped by (superstep, tile,
  // local level); each group then is one (superstep, tile) item's local level
  // opt-in (measured slower: the earliest-placement schedule puts the wide early levels of a
  // tile into ONE workgroup per superstep, 5.2 vs 1.9 ms per application at t = 51)
  tail_tiles_ = false;
  if (const char* e = std::getenv("GPBOOST_AMD_TAIL_TILES")) tail_tiles_ = nt > 0 && std::atoi(e) != 0;
  int TS = 512;
  if (const char* e = std::getenv("GPBOOST_AMD_TAIL_TILE")) TS = std::max(16, std::atoi(e));
  const int LT = kTailLocalLevels;
  std::vector<long long> keys_b, keys_f;   // (s, tile) item key of every group (tiles only)
  if (tail_tiles_) {
    const int ntiles = (n + TS - 1) / TS;
    auto schedule = [&](bool lower, std::vector<std::vector<int>>& groups, std::vector<long long>& keys,
                        std::vector<int>& sup_ptr) {
      std::vector<int> ss(n, 0), lam(n, 0);
      int S = 0;
      for (int q = 0; q < nt; ++q) {   // processing order: lower ascending Vecchia index, B^T descending
        const int r = lower ? lab_[K + q] : lab_[n - 1 - q];
        const int tr = r / TS;
        int bs = 0, bl = 0;
        auto dep = [&](int d) {
          int cs, cl;
          if (d / TS == tr) { cs = ss[d]; cl = lam[d] + 1; if (cl >= LT) { ++cs; cl = 0; } }
          else { cs = ss[d] + 1; cl = 0; }
          if (cs > bs || (cs == bs && cl > bl)) { bs = cs; bl = cl; }
        };
        if (lower) {
          const int k = std::min(r, m);
          for (int e = 0; e < k; ++e) { const int d = nbr[(size_t)r * m + e]; if (!head(d)) dep(d); }
        } else {
          for (int e = tptr[r]; e < tptr[r + 1]; ++e) dep(trow[e]);
        }
        ss[r] = bs;
        lam[r] = bl;
        S = std::max(S, bs + 1);
      }
      std::map<long long, std::vector<int>> g;   // (s, tile, lam) -> rows in processing order
      for (int q = 0; q < nt; ++q) {
        const int r = lower ? lab_[K + q] : lab_[n - 1 - q];
        g[((long long)ss[r] * ntiles + r / TS) * LT + lam[r]].push_back(r);
      }
      groups.clear();
      keys.clear();
      sup_ptr.assign(S + 1, 0);
      for (auto& kv : g) {
        const long long item = kv.first / LT;
        if (keys.empty() || keys.back() != item) ++sup_ptr[(int)(item / ntiles) + 1];
        keys.push_back(item);
        groups.push_back(std::move(kv.second));
      }
      for (int q = 0; q < S; ++q) sup_ptr[q + 1] += sup_ptr[q];
    };
    schedule(false, groups_b, keys_b, sup_b_);
    schedule(true, groups_f, keys_f, sup_f_);
  }
  std::vector<int> lrows, beoff(1, 0), beidx, fidx, beslot, fslot;
  tplan_.lptr.assign(1, 0);
  for (const auto& rows : groups_b) {
    for (int j : rows) {
      lrows.push_back(j);
      for (int e = tptr[j]; e < tptr[j + 1]; ++e) { beidx.push_back(trow[e]); beslot.push_back(tslot[e]); }
      beoff.push_back((int)beidx.size());
    }
    tplan_.lptr.push_back((int)lrows.size());
  }
  for (const auto& rows : groups_f) {
    for (int i : rows) {
      lrows.push_back(i);
      const int k = std::min(i, m);
      for (int r = 0; r < m; ++r) {
        fidx.push_back(r < k ? nbr[(size_t)i * m + r] : 0);
        fslot.push_back(r < k ? i * m + r : -1);
      }
    }
    tplan_.lptr.push_back((int)lrows.size());
  }
  if (tail_tiles_) {   // item offsets from the group boundaries: each item's local levels, padded to LT + 1
    const int nb = (int)groups_b.size();
    auto make_items = [&](int g0, const std::vector<long long>& keys) {
      for (size_t gi = 0; gi < keys.size();) {
        std::vector<int> offs{tplan_.lptr[g0 + gi]};
        size_t gj = gi;
        while (gj < keys.size() && keys[gj] == keys[gi]) { offs.push_back(tplan_.lptr[g0 + gj + 1]); ++gj; }
        if ((int)offs.size() > LT + 1) Fatal("tail tile schedule: more than %d local levels in one item", LT);
        while ((int)offs.size() < LT + 1) offs.push_back(offs.back());
        item_off.insert(item_off.end(), offs.begin(), offs.end());
        gi = gj;
      }
    };
    make_items(0, keys_b);
    const int items_b = (int)(item_off.size() / (LT + 1));
    make_items(nb, keys_f);
    for (int& v : sup_f_) v += items_b;
  }
  tplan_.n = nt;
  tplan_.m = m;
  tplan_.nlev_b = nt > 0 ? Lb : 0;
  tplan_.nlev = (int)tplan_.lptr.size() - 1;
  if (nt == 0) { tplan_.lptr.assign(1, 0); tplan_.nlev = 0; }
  const size_t o_lrows = put(lrows), o_beoff = put(beoff), o_beidx = put(beidx), o_fidx = put(fidx);
  const size_t o_items = put(item_off);
  const size_t v_be = vslot.size();
  vslot.insert(vslot.end(), beslot.begin(), beslot.end());
  const size_t v_f = vslot.size();
  vslot.insert(vslot.end(), fslot.begin(), fslot.end());
  // ---- head solves: positions by level (head-only dependencies), passes of <= kHeadRowsPerPass
  struct HeadArrays { std::vector<int> rec, eidx, slot, ooff{0}, oidx, oslot, pend; };
  auto build_head = [&](bool lower) {
    HeadArrays h;
    std::vector<int> lev(K, 0);
    std::vector<std::vector<int>> deps(K), dslot(K);
    for (int ii = 0; ii < K; ++ii) {
      const int p = lab_[ii];
      if (lower) {
        const int k = std::min(p, m);
        for (int r = 0; r < k; ++r) { deps[ii].push_back(vo_[nbr[(size_t)p * m + r]]); dslot[ii].push_back(p * m + r); }
      } else {
        for (int e = tptr[p]; e < tptr[p + 1]; ++e)
          if (head(trow[e])) { deps[ii].push_back(vo_[trow[e]]); dslot[ii].push_back(tslot[e]); }
      }
    }
    int L = 0;
    for (int s = 0; s < K; ++s) {   // lower: ascending Vecchia index; B^T: descending
      const int ii = lower ? s : K - 1 - s;
      int l = 0;
      for (int d : deps[ii]) l = std::max(l, lev[d] + 1);
      lev[ii] = l;
      L = std::max(L, l + 1);
    }
    std::vector<std::vector<int>> byl(L);
    for (int s = 0; s < K; ++s) {
      const int ii = lower ? s : K - 1 - s;
      byl[lev[ii]].push_back(ii);
    }
    const int E = kHeadEpl;
    auto nslots = [&](int ii) {   // 1, 2 or 4 slots of kHeadG lanes (rows beyond 4 slots overflow)
      const int c = (int)deps[ii].size();
      return c <= kHeadG * E ? 1 : c <= 2 * kHeadG * E ? 2 : 4;
    };
    for (auto rows : byl) {
      // widest rows first: power-of-two sizes in descending order stay aligned in a pass
      std::stable_sort(rows.begin(), rows.end(), [&](int x, int y) { return nslots(x) > nslots(y); });
      size_t q = 0;
      while (q < rows.size()) {   // one pass
        const size_t r_pass = h.rec.size();
        h.rec.resize(r_pass + kHeadRowsPerPass, K);
        h.ooff.resize(r_pass + kHeadRowsPerPass + 1, (int)h.oidx.size());
        h.eidx.resize((r_pass + kHeadRowsPerPass) * E * kHeadG, 0);
        h.slot.resize((r_pass + kHeadRowsPerPass) * E * kHeadG, -1);
        int used = 0;
        while (q < rows.size() && used + nslots(rows[q]) <= kHeadRowsPerPass) {
          const int ii = rows[q], ns = nslots(ii), GL = ns * kHeadG;
          const int lg = ns == 1 ? 0 : ns == 2 ? 1 : 2;
          const size_t r0 = r_pass + used;
          const int cnt = (int)deps[ii].size();
          const bool over = cnt > GL * E;
          for (int sub = 0; sub < ns; ++sub)
            h.rec[r0 + sub] = (int)((over ? 0x80000000u : 0u) | ((unsigned)sub << 18) | ((unsigned)lg << 16) |
                                    (unsigned)(sub == 0 ? ii : K));
          for (int e = 0; e < std::min(cnt, GL * E); ++e) {   // entry e -> group lane e % GL, k = e / GL
            const int gl = e % GL, k = e / GL;
            const size_t at = ((r0 + gl / kHeadG) * E + k) * kHeadG + gl % kHeadG;
            h.eidx[at] = deps[ii][e];
            h.slot[at] = dslot[ii][e];
          }
          h.ooff[r0] = (int)h.oidx.size();
          for (int e = GL * E; e < cnt; ++e) { h.oidx.push_back(deps[ii][e]); h.oslot.push_back(dslot[ii][e]); }
          for (int sub = 1; sub <= ns; ++sub) h.ooff[r0 + sub] = (int)h.oidx.size();
          used += ns;
          ++q;
        }
        for (size_t r = r_pass + used; r <= r_pass + kHeadRowsPerPass; ++r) h.ooff[r] = (int)h.oidx.size();
        h.pend.push_back(q >= rows.size() ? 1 : 0);   // last pass of its level: barrier after it
      }
    }
    return h;
  };
  HeadArrays hl = build_head(true), hb = build_head(false);
  // B^T tail contributions to every head row (rows without any still copy R)
  std::vector<int> prow, poff(1, 0), pidx, pslot;
  for (int ii = 0; ii < K; ++ii) {
    const int j = lab_[ii];
    prow.push_back(j);
    for (int e = tptr[j]; e < tptr[j + 1]; ++e)
      if (!head(trow[e])) { pidx.push_back(trow[e]); pslot.push_back(tslot[e]); }
    poff.push_back((int)pidx.size());
  }
  std::vector<int> hrow(K);
  for (int v = 0; v < K; ++v) hrow[v] = lab_[v];
  const size_t o_hrow = put(hrow);
  size_t o_h[2][5], v_h[2][2];
  for (int w = 0; w < 2; ++w) {
    HeadArrays& h = w == 0 ? hl : hb;
    o_h[w][0] = put(h.rec);
    o_h[w][1] = put(h.eidx);
    o_h[w][2] = put(h.oidx);
    o_h[w][3] = put(h.ooff);
    o_h[w][4] = put(h.pend);
    v_h[w][0] = vslot.size();
    vslot.insert(vslot.end(), h.slot.begin(), h.slot.end());
    v_h[w][1] = vslot.size();
    vslot.insert(vslot.end(), h.oslot.begin(), h.oslot.end());
  }
  const size_t o_prow = put(prow), o_poff = put(poff), o_pidx = put(pidx);
  const size_t v_p = vslot.size();
  vslot.insert(vslot.end(), pslot.begin(), pslot.end());
  d_hint_.alloc(std::max<size_t>(ints.size(), 1));
  d_hslot_.alloc(std::max<size_t>(vslot.size(), 1));
  d_hval_.alloc(std::max<size_t>(vslot.size(), 1));
  if (!ints.empty())
    HIP_CHECK(hipMemcpyAsync(d_hint_.get(), ints.data(), sizeof(int) * ints.size(), hipMemcpyHostToDevice, s_));
  if (!vslot.empty())
    HIP_CHECK(hipMemcpyAsync(d_hslot_.get(), vslot.data(), sizeof(int) * vslot.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  hslot_count_ = (int)vslot.size();
  const int* I = d_hint_.get();
  const double* V = d_hval_.get();
  tplan_.lrows = I + o_lrows;
  tplan_.beoff = I + o_beoff;
  tplan_.beidx = I + o_beidx;
  tplan_.fidx = I + o_fidx;
  tplan_.beval = V + v_be;
  tplan_.fval = V + v_f;
  d_items_ = I + o_items;
  for (int w = 0; w < 2; ++w) {
    HeadSolve& h = w == 0 ? hlow_ : hbt_;
    const HeadArrays& a = w == 0 ? hl : hb;
    h.K = K;
    h.npass = (int)(a.rec.size() / kHeadRowsPerPass);
    h.hrow = I + o_hrow;
    h.rec = I + o_h[w][0];
    h.eidx = I + o_h[w][1];
    h.oidx = I + o_h[w][2];
    h.ooff = I + o_h[w][3];
    h.pend = I + o_h[w][4];
    h.eval = V + v_h[w][0];
    h.oval = V + v_h[w][1];
  }
  hpart_.rows = K;
  hpart_.row = I + o_prow;
  hpart_.eoff = I + o_poff;
  hpart_.eidx = I + o_pidx;
  hpart_.eval = V + v_p;
  head_passes_ = hlow_.npass + hbt_.npass;
  if (K > 0) set_vadu_head_lds_limit(K);
}

// Tail part of one solve (mode 4): level kernels, or the tile-blocked supersteps.
void LatentVecchia::TailSolve(bool lower, const double* R, double* Xt, double* Z, int t) {
  if (!tail_tiles_) {
    const int l0 = lower ? tplan_.nlev_b : 0, l1 = lower ? tplan_.nlev : tplan_.nlev_b;
    for (int l = l0; l < l1; ++l) launch_vadu_level(tplan_, l, d_dw_.get(), R, Xt, Z, t, s_);
    return;
  }
  const std::vector<int>& sp = lower ? sup_f_ : sup_b_;
  for (size_t q = 0; q + 1 < sp.size(); ++q)
    launch_vadu_tile(tplan_, lower, d_items_, kTailLocalLevels, sp[q], sp[q + 1] - sp[q], d_dw_.get(),
                     lower ? Xt : R, lower ? Z : Xt, t, s_);
}

// Z = P^-1 R, P = B^T (D^-1 + W) B (VADU, CG_utils.cpp:56-60): B^T solve then (dw B) solve.
// Default: one kernel per level replayed from a hipGraph captured once per buffer set
// (a graph boundary costs ~1.5 us, far below a host launch); alternative: the one-launch
// per-column sweep (GPBOOST_AMD_SWEEP_KERNEL).
void LatentVecchia::Precond(const double* R, double* Z, double* Xt, int t) {
  g_timer.begin(s_);
  PrecondImpl(R, Z, Xt, t);
  g_timer.end(s_, t == 1 ? 0 : 1);
}

void LatentVecchia::PrecondImpl(const double* R, double* Z, double* Xt, int t) {
  if (precond_mode_ == 0) {
    FlowArgs fa{};
    fa.n = n_;
    fa.m = m_;
    fa.t = t;
    fa.err = d_err_.get();
    fa.prof = prof_;
    fa.lrows = lplan_.lrows;              // B^T solve: Xt = B^-T R
    fa.crit = d_crit_.get();
    fa.eoff = lplan_.beoff;
    fa.eidx = lplan_.beidx;
    fa.eval = lplan_.beval;
    fa.in = R;
    fa.X = Xt;
    launch_vadu_flow(fa, false, max_flow_blocks_, s_);
    fa.lrows = lplan_.lrows + n_;         // lower solve: Z = ((D^-1 + W) B)^-1 Xt
    fa.crit = d_crit_.get() + n_;
    fa.eoff = nullptr;
    fa.eidx = lplan_.fidx;
    fa.eval = lplan_.fval;
    fa.dw = d_dw_.get();
    fa.in = Xt;
    fa.X = Z;
    if (prof_) fa.prof = prof_ + (size_t)n_ * 4;
    launch_vadu_flow(fa, true, max_flow_blocks_, s_);
    return;
  }
  if (precond_mode_ == 2) {
    launch_vadu_sweep(plan_, d_dw_.get(), R, Xt, Z, t, s_);
    return;
  }
  if (precond_mode_ == 3) {
    SfArgs sa{};
    sa.n = n_;
    sa.m = m_;
    sa.t = t;
    sa.err = d_err_.get();
    sa.lrows = lplan_.lrows;              // B^T solve: Xt = B^-T R
    sa.crit = d_crit_.get();
    sa.eoff = lplan_.beoff;
    sa.eidx = lplan_.beidx;
    sa.eval = lplan_.beval;
    sa.in = R;
    sa.X = Xt;
    launch_vadu_sf(sa, false, sf_grid_, s_);
    sa.lrows = lplan_.lrows + n_;         // lower solve: Z = ((D^-1 + W) B)^-1 Xt
    sa.crit = d_crit_.get() + n_;
    sa.eoff = nullptr;
    sa.eidx = lplan_.fidx;
    sa.eval = lplan_.fval;
    sa.dw = d_dw_.get();
    sa.in = Xt;
    sa.X = Z;
    launch_vadu_sf(sa, true, sf_grid_, s_);
    return;
  }
  static const bool eager = std::getenv("GPBOOST_AMD_NO_GRAPH") != nullptr;   // diagnostics (profilers)
  if (precond_mode_ == 4) {
    auto record = [&]() {
      TailSolve(false, R, Xt, Z, t);
      launch_vadu_head_partial(hpart_, R, Xt, t, s_);
      launch_vadu_head(hbt_, false, d_dw_.get(), nullptr, Xt, t, s_);
      launch_vadu_head(hlow_, true, d_dw_.get(), Xt, Z, t, s_);
      TailSolve(true, R, Xt, Z, t);
    };
    if (eager) { record(); return; }
    for (const GraphEntry& g : hgraphs_) {
      if (g.key[0] == R && g.key[1] == Xt && g.key[2] == Z && g.t == t) {
        HIP_CHECK(hipGraphLaunch(g.exec, s_));
        return;
      }
    }
    hipGraph_t graph;
    HIP_CHECK(hipStreamBeginCapture(s_, hipStreamCaptureModeThreadLocal));
    record();
    HIP_CHECK(hipStreamEndCapture(s_, &graph));
    GraphEntry e{{R, Xt, Z}, t, nullptr};
    HIP_CHECK(hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(graph));
    hgraphs_.push_back(e);
    HIP_CHECK(hipGraphLaunch(e.exec, s_));
    return;
  }
  if (eager) {
    for (int l = 0; l < lplan_.nlev; ++l) launch_vadu_level(lplan_, l, d_dw_.get(), R, Xt, Z, t, s_);
    return;
  }
  for (const GraphEntry& g : graphs_) {
    if (g.key[0] == R && g.key[1] == Xt && g.key[2] == Z && g.t == t) {
      HIP_CHECK(hipGraphLaunch(g.exec, s_));
      return;
    }
  }
  hipGraph_t graph;
  HIP_CHECK(hipStreamBeginCapture(s_, hipStreamCaptureModeThreadLocal));
  for (int l = 0; l < lplan_.nlev; ++l) launch_vadu_level(lplan_, l, d_dw_.get(), R, Xt, Z, t, s_);
  HIP_CHECK(hipStreamEndCapture(s_, &graph));
  GraphEntry e{{R, Xt, Z}, t, nullptr};
  HIP_CHECK(hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(graph));
  graphs_.push_back(e);
  HIP_CHECK(hipGraphLaunch(e.exec, s_));
}

// A bounded spin of the sync-free solves gave up (a dependency never arrived): fail loudly.
void LatentVecchia::CheckSolveError() {
  int err = 0;
  HIP_CHECK(hipMemcpy(&err, d_err_.get(), sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    HIP_CHECK(hipMemset(d_err_.get(), 0, sizeof(int)));
    Fatal("VADU triangular solve did not complete (dependency wait timed out)");
  }
}

double LatentVecchia::Dot1(const double* x, const double* y) {
  const double* A[1] = {x};
  const double* Bm[1] = {y};
  launch_coldots(n_, 1, 1, A, Bm, d_partials_.get(), d_out_.get(), s_);
  HIP_CHECK(hipMemcpyAsync(h_out_, d_out_.get(), sizeof(double), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  return h_out_[0];
}

void LatentVecchia::Scalars(const ScalarArgs& a, double* out) {
  launch_latent_scalars(a, d_partials_.get(), d_out_.get(), s_);
  HIP_CHECK(hipMemcpyAsync(h_out_, d_out_.get(), sizeof(double) * kLatentScalars, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  std::copy(h_out_, h_out_ + kLatentScalars, out);
}

LatentVecchia::PcgResult LatentVecchia::Pcg(Block& b, const double* RHS, double* U, int n_single, bool init_zero,
                                             bool u_is_zero, int pmax_single, int pmax_block, double delta) {
  const int t = b.t;
  const size_t nt = (size_t)n_ * t;
  PcgResult res;
  if (h_rr_.size() < (size_t)t) h_rr_.resize(t);
  pmax_single = std::min(pmax_single, n_);
  pmax_block = std::min(pmax_block, n_);
  if (t == 1 && n_single == 1) {
    if (Dot1(RHS, RHS) < kZeroRhsSq) {   // CG_utils.cpp:42-45
      HIP_CHECK(hipMemsetAsync(U, 0, sizeof(double) * nt, s_));
      res.zero_rhs = true;
      return res;
    }
  }
  if (t == 1 && n_single == 1 && !init_zero && !u_is_zero) {   // r = rhs - A u (warm start, CG_utils.cpp:53-55)
    ApplyA(U, b.V.get(), b.G.get(), t);
    launch_axpby(nt, 1., RHS, -1., b.V.get(), b.R.get(), s_);
  } else {
    HIP_CHECK(hipMemsetAsync(U, 0, sizeof(double) * nt, s_));
    launch_copy(nt, RHS, b.R.get(), s_);
  }
  std::vector<int> act(t, 1);
  HIP_CHECK(hipMemcpyAsync(b.act.get(), act.data(), sizeof(int) * t, hipMemcpyHostToDevice, s_));
  bool act_s = n_single > 0 && pmax_single > 0, act_b = n_single < t && pmax_block > 0;
  Precond(b.R.get(), b.Z.get(), b.Xt.get(), t);
  launch_copy(nt, b.Z.get(), b.H.get(), s_);
  {
    const double* A[1] = {b.R.get()};
    const double* Bm[1] = {b.Z.get()};
    launch_coldots(n_, t, 1, A, Bm, d_partials_.get(), b.rz(), s_);
  }
  for (int j = 0; act_s || act_b; ++j) {
    ApplyA(b.H.get(), b.V.get(), b.G.get(), t);
    {
      const double* A[1] = {b.H.get()};
      const double* Bm[1] = {b.V.get()};
      launch_coldots(n_, t, 1, A, Bm, d_partials_.get(), b.hv(), s_);
    }
    launch_cg_alpha(t, b.rz(), b.hv(), b.act.get(), b.a(), b.a_hist.get() + (size_t)j * t, s_);
    launch_cg_update(n_, t, b.a(), b.H.get(), b.V.get(), U, b.R.get(), d_partials_.get(), b.rr(), s_);
    HIP_CHECK(hipMemcpyAsync(h_rr_.data(), b.rr(), sizeof(double) * t, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    bool changed = false;
    if (act_s) {   // single-vector CGs: own ||r|| (CG_utils.cpp:80-90)
      res.its_single = j + 1;
      bool all_done = true;
      for (int c = 0; c < n_single; ++c) {
        if (!act[c]) continue;
        const double norm = std::sqrt(h_rr_[c]);
        if (std::isnan(norm) || std::isinf(norm)) { CheckSolveError(); res.nan = true; return res; }
        if (norm < delta || j + 1 >= pmax_single) { act[c] = 0; changed = true; }
        else all_done = false;
      }
      act_s = !all_done;
    }
    if (act_b) {   // block: mean column ||r|| (CG_utils.cpp:172-178)
      res.its_block = j + 1;
      double norm = 0.;
      for (int c = n_single; c < t; ++c) norm += std::sqrt(h_rr_[c]);
      norm /= (t - n_single);
      if (std::isnan(norm) || std::isinf(norm)) { CheckSolveError(); res.nan = true; return res; }
      if (norm < delta || j + 1 >= pmax_block) {
        for (int c = n_single; c < t; ++c) act[c] = 0;
        act_b = false;
        changed = true;
      }
    }
    if (!act_s && !act_b) break;
    if (changed) HIP_CHECK(hipMemcpyAsync(b.act.get(), act.data(), sizeof(int) * t, hipMemcpyHostToDevice, s_));
    Precond(b.R.get(), b.Z.get(), b.Xt.get(), t);
    {
      const double* A[1] = {b.R.get()};
      const double* Bm[1] = {b.Z.get()};
      launch_coldots(n_, t, 1, A, Bm, d_partials_.get(), b.rz_new(), s_);
    }
    launch_cg_beta(t, b.rz_new(), b.rz(), b.act.get(), b.b(), b.b_hist.get() + (size_t)j * t, s_);
    launch_h_update(n_, t, b.b(), b.Z.get(), b.H.get(), s_);
  }
  return res;
}

LatentResult LatentVecchia::Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                                 bool want_grad, bool want_aux_grad) {
  if (!y_set_) Fatal("response variable y has not been set");
  if (!(trafo[0] > 0. && trafo[1] > 0.)) Fatal("covariance parameters must be > 0");
  if (lik == kLikGaussian && !(aux > 0.)) Fatal("the error variance (aux_pars) must be > 0");
  const int n = n_;
  const bool gauss = lik == kLikGaussian;
  const int t = cfg.num_rand_vec_trace;
  if (t < 1) Fatal("num_rand_vec_trace must be >= 1");
  LatentResult res;
  HIP_CHECK(hipEventRecord(ev0_, s_));

  // ---- 1. latent Vecchia factor (+ range derivatives)
  LatentFactorArgs fa{};
  fa.X = d_Xp_.get();
  fa.nbr = d_nbr_.get();
  fa.n = n; fa.d = d_; fa.m = m_;
  fa.var = trafo[0];
  fa.phi = trafo[1];
  fa.jitter = kJitterMultVecchia;
  fa.Bv = d_Bv_.get();
  fa.dBv = want_grad ? d_dBv_.get() : nullptr;
  fa.Dinv = d_Dinv_.get();
  fa.dD = want_grad ? d_dD_.get() : nullptr;
  launch_latent_factor(cov_type, fa, s_);
  launch_sweep_values(plan_entries_, d_vpos_.get(), d_eslot_.get(), d_Bv_.get(), d_blob_.get(), s_);
  launch_gather(lplan_entries_, d_lslot_.get(), d_Bv_.get(), d_lval_.get(), s_);
  launch_gather(hslot_count_, d_hslot_.get(), d_Bv_.get(), d_hval_.get(), s_);
  launch_gather(tnnz_, d_tslot_.get(), d_Bv_.get(), d_tval_.get(), s_);   // B^T operator values, list order
  sp_.tval_of = d_Bv_.get();
  factor_ready_ = true;

  Block& b1 = GetBlock(0, 1, std::max(cfg.cg_max_num_it, 1));
  if (std::getenv("GPBOOST_AMD_BENCH_PRECOND")) {   // diagnostics: preconditioner cost alone
    NewtonPrepArgs np{};
    np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
    np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get(); np.W_update = 1; np.dw = d_dw_.get();
    HIP_CHECK(hipMemsetAsync(d_mode_.get(), 0, sizeof(double) * n, s_));
    launch_newton_prep(np, s_);
    HIP_CHECK(hipMemsetAsync(b1.R.get(), 0, sizeof(double) * n, s_));
    for (int tt : {1, t}) {
      Block& bb = GetBlock(tt == 1 ? 0 : 1, tt, std::max(cfg.cg_max_num_it, 1));
      HIP_CHECK(hipMemsetAsync(bb.R.get(), 0, sizeof(double) * n * tt, s_));
      Precond(bb.R.get(), bb.Z.get(), bb.Xt.get(), tt);
      HIP_CHECK(hipStreamSynchronize(s_));
      HIP_CHECK(hipEventRecord(ev0_, s_));
      for (int r = 0; r < 20; ++r) Precond(bb.R.get(), bb.Z.get(), bb.Xt.get(), tt);
      HIP_CHECK(hipEventRecord(ev1_, s_));
      HIP_CHECK(hipEventSynchronize(ev1_));
      float pm = 0.f;
      HIP_CHECK(hipEventElapsedTime(&pm, ev0_, ev1_));
      std::fprintf(stderr, "[precond bench] t=%d: %.3f ms per application (%d levels)\n", tt, pm / 20,
                   lplan_.nlev);
      if (const char* path = std::getenv("GPBOOST_AMD_FLOW_PROF")) {   // per-row timestamps of one application
        DevBuf<unsigned long long> prof((size_t)2 * n * 4);
        HIP_CHECK(hipMemsetAsync(prof.get(), 0, sizeof(unsigned long long) * 2 * n * 4, s_));
        prof_ = prof.get();
        Precond(bb.R.get(), bb.Z.get(), bb.Xt.get(), tt);
        prof_ = nullptr;
        std::vector<unsigned long long> h((size_t)2 * n * 4);
        HIP_CHECK(hipMemcpy(h.data(), prof.get(), sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
        std::string fn = std::string(path) + "_t" + std::to_string(tt) + ".bin";
        if (FILE* f = std::fopen(fn.c_str(), "wb")) {
          int hdr[4] = {n, lplan_.nlev_b, lplan_.nlev, tt};
          std::fwrite(hdr, sizeof(int), 4, f);
          std::fwrite(lplan_.lptr.data(), sizeof(int), lplan_.lptr.size(), f);
          std::fwrite(h_crit_.data(), sizeof(int), h_crit_.size(), f);
          std::vector<int> lr((size_t)2 * n);
          HIP_CHECK(hipMemcpy(lr.data(), lplan_.lrows, sizeof(int) * lr.size(), hipMemcpyDeviceToHost));
          std::fwrite(lr.data(), sizeof(int), lr.size(), f);
          std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
          std::fclose(f);
        }
      }
    }
  }
  ScalarArgs sa{};
  sa.n = n; sa.m = m_; sa.lik = lik; sa.aux = aux;
  sa.nbr = d_nbr_.get(); sa.Bv = d_Bv_.get(); sa.Dinv = d_Dinv_.get(); sa.y = d_y_.get();

  // ---- 2. mode finding (likelihoods.h:2780-3000); mode re-initialised to 0 (InitializeModeAvec)
  HIP_CHECK(hipMemsetAsync(d_mode_.get(), 0, sizeof(double) * n, s_));
  HIP_CHECK(hipMemsetAsync(d_mode_upd_.get(), 0, sizeof(double) * n, s_));
  double sc[kLatentScalars];
  sa.mode = d_mode_.get();
  Scalars(sa, sc);
  if (std::isnan(sc[kSqLogDinv]) || std::isinf(sc[kSqLogDinv]))   // Vecchia_utils.cpp:1619-1630
    Fatal("The matrix D in the Vecchia approximation contains negative or zero values. "
          "This likely results from numerical instabilities ");
  double mll = sc[kSqLogLik] - 0.5 * sc[kSqQuad];
  const bool info_changes = !gauss;              // information_changes_during/after_mode_finding_
  const int maxit = gauss ? 1 : 1000;            // maxit_mode_newton_ (likelihoods.h:255, 12721)
  const int max_shrink = gauss ? 1 : 20;         // max_number_lr_shrinkage_steps_newton_ (:256, 12725)
  const int pmax_tri = std::max(1, std::min(cfg.cg_max_num_it_tridiag, n));
  const int cg_max = std::max(0, cfg.cg_max_num_it);
  Block* bslq = nullptr;
  int n_lead = 0;   // leading non-probe columns of the SLQ block
  PcgResult slq;
  auto line_search_and_check = [&](int it, double gdd) -> bool {   // likelihoods.h:2967-2995, 11820-11870
    double lr = 1., mll_new = mll;
    for (int ih = 0; ih < max_shrink; ++ih) {
      if (ih == 0) launch_copy(n, d_mode_upd_.get(), d_mode_new_.get(), s_);
      else launch_axpby(n, 1. - lr, d_mode_.get(), lr, d_mode_upd_.get(), d_mode_new_.get(), s_);
      sa.mode = d_mode_new_.get();
      Scalars(sa, sc);
      mll_new = sc[kSqLogLik] - 0.5 * sc[kSqQuad];
      if (mll_new < mll + kCArmijo * lr * gdd || std::isnan(mll_new) || std::isinf(mll_new)) lr *= 0.5;
      else break;
    }
    std::swap(d_mode_, d_mode_new_);
    res.newton_its = it + 1;
    if (std::isnan(mll_new) || std::isinf(mll_new))
      Fatal("NaN or Inf occurred in the mode finding algorithm for the Laplace approximation");
    const double dc = cfg.delta_conv_mode_finding;
    const bool term = (it == 0) ? std::fabs(mll_new - mll) < dc * std::fabs(mll) : (mll_new - mll) < dc * std::fabs(mll);
    mll = mll_new;
    return term;
  };
  EnsureProbes(cfg);
  if (gauss) {
    // Gaussian: W = 1/aux does not depend on the mode, so the single Newton step's solve
    // (Sigma^-1 + W)^-1 (y / aux) and the SLQ block solve the same system. Both run as one
    // PCG over 1 + t columns: column 0 keeps the single-vector stopping rule, columns 1..t
    // the block rule (each column's iterates are exactly those of a separate run).
    NewtonPrepArgs np{};
    np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
    np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get(); np.W_update = 1;
    np.rhs = d_rhs_.get(); np.dw = d_dw_.get(); np.sdw = d_sdw_.get();
    launch_newton_prep(np, s_);
    n_lead = 1;
    const int tf = t + 1;
    bslq = &GetBlock(1, tf, std::max(pmax_tri, cg_max));
    d_rhsf_.alloc((size_t)n * tf);
    d_Uf_.alloc((size_t)n * tf);
    // z_i = B^T (D^-1 + W)^(1/2) r_i into columns 1..t, y / aux into column 0
    launch_bt_apply(sp_, d_Bv_.get(), true, d_probes_.get(), t, d_sdw_.get(), nullptr, nullptr, d_Zp_.get(), s_);
    launch_pack_columns(n, t, d_Zp_.get(), t, 0, d_rhsf_.get(), tf, 1, s_);
    launch_pack_columns(n, 1, d_rhs_.get(), 1, 0, d_rhsf_.get(), tf, 0, s_);
    slq = Pcg(*bslq, d_rhsf_.get(), d_Uf_.get(), 1, true, true, cg_max, pmax_tri, cfg.cg_delta_conv);
    if (slq.nan) Fatal("NaN or Inf occurred in the conjugate gradient algorithm (mode finding / log-determinant)");
    res.cg_its = slq.its_single;
    launch_pack_columns(n, 1, d_Uf_.get(), tf, 0, d_mode_upd_.get(), 1, 0, s_);
    launch_pack_columns(n, t, d_Uf_.get(), tf, 1, d_U_.get(), t, 0, s_);
    line_search_and_check(0, 0.);
  } else {
    // ---- 2. mode finding (likelihoods.h:2780-3000)
    bool upd_zero = true;
    for (int it = 0; it < maxit; ++it) {
      NewtonPrepArgs np{};
      np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
      np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get();
      np.W_update = 1;
      np.rhs = d_rhs_.get();
      np.dw = d_dw_.get();
      launch_newton_prep(np, s_);
      const PcgResult pr = Pcg(b1, d_rhs_.get(), d_mode_upd_.get(), 1, it == 0, upd_zero, cg_max, 0, cfg.cg_delta_conv);
      res.cg_its += pr.its_single;
      upd_zero = pr.zero_rhs;
      if (pr.nan) Fatal("NaN or Inf occurred in the conjugate gradient algorithm during mode finding");
      // Armijo (likelihoods.h:2957-2966)
      launch_axpby(n, 1., d_mode_upd_.get(), -1., d_mode_.get(), d_dir_.get(), s_);
      ApplyA(d_dir_.get(), d_Adir_.get(), b1.G.get(), 1);
      const double gdd = Dot1(d_dir_.get(), d_Adir_.get());
      if (line_search_and_check(it, gdd)) break;
    }
    {   // derivative / information at the mode, VADU diagonal and its square root (:3000-3005, 12163-12166)
      NewtonPrepArgs np{};
      np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
      np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get();
      np.W_update = info_changes ? 1 : 0;
      np.dw = d_dw_.get();
      np.sdw = d_sdw_.get();
      launch_newton_prep(np, s_);
    }
    // ---- 3. SLQ block (likelihoods.h:3018-3045, 12155-12212): z_i = B^T (D^-1 + W)^(1/2) r_i
    bslq = &GetBlock(1, t, pmax_tri);
    launch_bt_apply(sp_, d_Bv_.get(), true, d_probes_.get(), t, d_sdw_.get(), nullptr, nullptr, d_Zp_.get(), s_);
    slq = Pcg(*bslq, d_Zp_.get(), d_U_.get(), 0, true, true, 0, pmax_tri, cfg.cg_delta_conv);
    if (slq.nan) Fatal("NaN or Inf occurred in the stochastic Lanczos quadrature (log-determinant)");
  }
  Block& bt = *bslq;
  const int L = slq.its_block;
  res.lanczos_steps = L;
  const int tb = bt.t;
  std::vector<double> ah((size_t)L * tb), bh((size_t)L * tb);
  HIP_CHECK(hipMemcpyAsync(ah.data(), bt.a_hist.get(), sizeof(double) * ah.size(), hipMemcpyDeviceToHost, s_));
  if (L > 1)
    HIP_CHECK(hipMemcpyAsync(bh.data(), bt.b_hist.get(), sizeof(double) * (size_t)(L - 1) * tb, hipMemcpyDeviceToHost,
                             s_));
  sa.mode = d_mode_.get();
  sa.dw = d_dw_.get();
  Scalars(sa, sc);   // synchronises the stream
  std::vector<std::vector<double>> Td(t), Ts(t);
  for (int c = 0; c < t; ++c) {   // CG_utils.cpp:200-206 (a_old = 1, b_old = 0 before the first step)
    const int cc = c + n_lead;
    Td[c].resize(L);
    Ts[c].resize(L > 0 ? L - 1 : 0);
    for (int j = 0; j < L; ++j) {
      const double a = ah[(size_t)j * tb + cc];
      const double a_old = j > 0 ? ah[(size_t)(j - 1) * tb + cc] : 1.;
      const double b_old = j > 0 ? bh[(size_t)(j - 1) * tb + cc] : 0.;
      Td[c][j] = 1. / a + b_old / a_old;
      if (j > 0) Ts[c][j - 1] = std::sqrt(b_old) / a_old;
    }
  }
  const double ldet_PI = slq_logdet(Td, Ts, n);
  res.logdet = ldet_PI - sc[kSqLogDinv] + sc[kSqLogDw];
  const double mll_final = mll - 0.5 * res.logdet;
  res.nll = -mll_final;

  if (want_grad) {
    // ---- 4. gradient (likelihoods.h:4951-5206)
    Precond(d_Zp_.get(), d_P_.get(), bt.Xt.get(), t);   // PI_Z = P^-1 Z (:12321-12327)
    if (!gauss) {   // grad_information_wrt_mode_non_zero_: implicit derivative through the mode
      ModeDerivArgs md{};
      md.n = n; md.m = m_; md.t = t; md.lik = lik; md.nbr = d_nbr_.get(); md.Bv = d_Bv_.get(); md.dw = d_dw_.get();
      md.loc = d_mode_.get(); md.U = d_U_.get(); md.P = d_P_.get(); md.dmll = d_dmll_.get();
      launch_mode_deriv(md, s_);
      const PcgResult pv = Pcg(b1, d_dmll_.get(), d_vS_.get(), 1, true, true, cg_max, 0, cfg.cg_delta_conv);
      res.cg_its += pv.its_single;
      if (pv.nan) Warning("NaN or Inf occurred in the conjugate gradient algorithm of the gradient calculation");
    }
    GradColsArgs ga{};
    ga.n = n; ga.m = m_; ga.t = t; ga.nbr = d_nbr_.get(); ga.Bv = d_Bv_.get(); ga.dBv = d_dBv_.get();
    ga.Dinv = d_Dinv_.get(); ga.dD = d_dD_.get(); ga.W = d_W_.get();
    ga.daux = gauss ? -1. / aux : 0.;   // d information / dlog(aux) (likelihoods.h:10967-10976)
    ga.U = d_U_.get(); ga.P = d_P_.get();
    DevBuf<double>& cols = d_out_;
    launch_grad_cols(ga, d_partials_.get(), cols.get(), s_);
    std::vector<double> z((size_t)kGradCols * t);
    HIP_CHECK(hipMemcpyAsync(z.data(), cols.get(), sizeof(double) * z.size(), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    ScalarArgs sg = sa;
    sg.dBv = d_dBv_.get();
    sg.dD = d_dD_.get();
    sg.vS = gauss ? nullptr : d_vS_.get();
    Scalars(sg, sc);
    auto mean = [t](const double* v) {
      double s = 0.;
      for (int c = 0; c < t; ++c) s += v[c];
      return s / t;
    };
    // marginal variance: SigmaI_deriv = -Sigma^-1 (:5036-5038, 12445-12458)
    {
      const double* z1 = z.data();
      const double* zP = z.data() + t;
      const double tr1 = mean(z1), trP = mean(zP);
      const double trD = -sc[kSqTrVar];
      const double c = optimal_c(z1, zP, t, tr1, trP);
      const double dld = tr1 + n + c * trD - c * trP;
      double g = 0.5 * (-sc[kSqQuad] + dld);
      if (!gauss) g += sc[kSqImpVar];   // - vS^T (-Sigma^-1 m)
      res.grad.push_back(g);
    }
    // range (:5040-5063, 12449-12465)
    {
      const double* z1 = z.data() + 2 * t;
      const double* zP = z.data() + 3 * t;
      const double tr1 = mean(z1), trP = mean(zP);
      const double trD = -sc[kSqTrRng];
      const double c = optimal_c(z1, zP, t, tr1, trP);
      const double dld = tr1 + sc[kSqDinvDD] + c * trD - c * trP;
      double g = 0.5 * (2. * sc[kSqDQuadRng] - sc[kSqDDQuad] + dld);
      if (!gauss) g -= sc[kSqImpRng];
      res.grad.push_back(g);
    }
    // gaussian error variance on the log scale (:5166-5200, 10586-10597, 12520-12546)
    if (gauss && want_aux_grad) {
      const double* z1 = z.data() + 4 * t;
      const double* zP = z.data() + 5 * t;
      const double tr1 = mean(z1), trP = mean(zP);
      const double trD = sc[kSqTrDw] * (-1. / aux);
      const double c = optimal_c(z1, zP, t, tr1, trP);
      const double dd = tr1 + c * trD - c * trP;
      res.grad.push_back(sc[kSqRss] * (-0.5 / aux) + 0.5 * n + 0.5 * dd);
    }
  }
  HIP_CHECK(hipEventRecord(ev1_, s_));
  HIP_CHECK(hipEventSynchronize(ev1_));
  CheckSolveError();
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
  res.ms_total = ms;
  if (g_timer.on) {
    std::fprintf(stderr, "[latent timing] total %.1f ms | precond t=1: %d x %.3f ms, t=%d: %d x %.3f ms | "
                 "A t=1: %d x %.3f ms, t=%d: %d x %.3f ms\n", ms, g_timer.cnt[0],
                 g_timer.cnt[0] ? g_timer.ms[0] / g_timer.cnt[0] : 0., t, g_timer.cnt[1],
                 g_timer.cnt[1] ? g_timer.ms[1] / g_timer.cnt[1] : 0., g_timer.cnt[2],
                 g_timer.cnt[2] ? g_timer.ms[2] / g_timer.cnt[2] : 0., t, g_timer.cnt[3],
                 g_timer.cnt[3] ? g_timer.ms[3] / g_timer.cnt[3] : 0.);
    g_timer = PhaseTimer();
  }
  return res;
}

}  // namespace gpb_amd
