// GroupedRE implementation: host planning of Z^T Z (setup) and the iteration logic of the PCG /
// SLQ / stochastic-trace path; every vector operation runs on the device (grouped_kernels.hip and
// the shared block-CG kernels of latent_kernels.h).
#include "grouped.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

#include "dense.h"
#include "fitc.h"
#include "grouped_kernels.h"
#include "latent_kernels.h"
#include "slq_host.h"

namespace gpb_amd {

namespace {
constexpr double kZeroRhsAbs = 1e-100;   // THRESHOLD_ZERO_RHS_CG (utils.h), on sum |rhs|
constexpr int kOut = 4096;   // pinned host / device scalar slots (>= 1024 residual norms, 2 + 2K sums)
constexpr int kDenseMaxM = 60000;   // K >= 2 cholesky: dense M x M factor (3.5 M^2 doubles, ~100 GB at the limit)
}  // namespace

GroupedRE::GroupedRE(int n, const std::vector<std::vector<int>>& levels, hipStream_t s)
    : n_(n), K_((int)levels.size()), s_(s) {
  if (K_ < 1) Fatal("grouped random effects need at least one grouping variable");
  m_.resize(K_);
  cum_.assign(K_ + 1, 0);
  for (int k = 0; k < K_; ++k) {
    int mx = -1;
    for (int i = 0; i < n; ++i) mx = std::max(mx, levels[k][i]);
    m_[k] = mx + 1;
    cum_[k + 1] = cum_[k] + m_[k];
  }
  M_ = cum_[K_];
  // observations per RE level (ascending), and Z^T Z: diagonal counts + off-diagonal cross counts
  std::vector<int> optr(M_ + 1, 0), cnt_i(M_, 0);
  for (int k = 0; k < K_; ++k)
    for (int i = 0; i < n; ++i) ++cnt_i[cum_[k] + levels[k][i]];
  for (int r = 0; r < M_; ++r) optr[r + 1] = optr[r] + cnt_i[r];
  std::vector<int> obs((size_t)n * K_), fill(optr.begin(), optr.end() - 1);
  for (int k = 0; k < K_; ++k)
    for (int i = 0; i < n; ++i) obs[fill[cum_[k] + levels[k][i]]++] = i;
  // off-diagonal entries (r, c), r and c in different effects: sort the n K (K-1) pairs
  std::vector<int64_t> pairs;
  pairs.reserve((size_t)n * K_ * (K_ - 1));
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < K_; ++k)
      for (int l = 0; l < K_; ++l)
        if (k != l) pairs.push_back((int64_t)(cum_[k] + levels[k][i]) * M_ + (cum_[l] + levels[l][i]));
  std::sort(pairs.begin(), pairs.end());
  std::vector<int> rowptr(M_ + 1, 0), split(M_, 0), col;
  std::vector<double> val;
  for (size_t a = 0; a < pairs.size();) {
    size_t b = a;
    while (b < pairs.size() && pairs[b] == pairs[a]) ++b;
    const int r = (int)(pairs[a] / M_), c = (int)(pairs[a] % M_);
    col.push_back(c);
    val.push_back((double)(b - a));
    ++rowptr[r + 1];
    a = b;
  }
  for (int r = 0; r < M_; ++r) rowptr[r + 1] += rowptr[r];
  std::vector<int> blk(M_);
  for (int k = 0; k < K_; ++k)
    for (int r = cum_[k]; r < cum_[k + 1]; ++r) {
      blk[r] = k;
      int e = rowptr[r];
      while (e < rowptr[r + 1] && col[e] < cum_[k]) ++e;
      split[r] = e;
    }
  std::vector<double> cnt(cnt_i.begin(), cnt_i.end());
  rowptr_h_ = rowptr;
  split_h_ = split;
  const size_t nnz = std::max<size_t>(col.size(), 1);
  d_rowptr_.alloc(M_ + 1);
  d_split_.alloc(M_);
  d_col_.alloc(nnz);
  d_val_.alloc(nnz);
  d_blk_.alloc(M_);
  d_cnt_.alloc(M_);
  d_obs_ptr_.alloc(M_ + 1);
  d_obs_.alloc(obs.size());
  HIP_CHECK(hipMemcpyAsync(d_rowptr_.get(), rowptr.data(), sizeof(int) * (M_ + 1), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_split_.get(), split.data(), sizeof(int) * M_, hipMemcpyHostToDevice, s_));
  if (!col.empty()) {
    HIP_CHECK(hipMemcpyAsync(d_col_.get(), col.data(), sizeof(int) * col.size(), hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipMemcpyAsync(d_val_.get(), val.data(), sizeof(double) * val.size(), hipMemcpyHostToDevice, s_));
  }
  HIP_CHECK(hipMemcpyAsync(d_blk_.get(), blk.data(), sizeof(int) * M_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_cnt_.get(), cnt.data(), sizeof(double) * M_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_obs_ptr_.get(), optr.data(), sizeof(int) * (M_ + 1), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(d_obs_.get(), obs.data(), sizeof(int) * obs.size(), hipMemcpyHostToDevice, s_));
  for (auto* b : {&d_D_, &d_sqrtD_, &d_zty_, &d_u_, &d_ztzu_}) b->alloc(M_);
  d_tau_.alloc(K_);
  d_dsum_.alloc(2 * K_);
  d_cum_.alloc(K_ + 1);
  HIP_CHECK(hipMemcpyAsync(d_cum_.get(), cum_.data(), sizeof(int) * (K_ + 1), hipMemcpyHostToDevice, s_));
  d_yty_.alloc(1);
  d_out_.alloc(kOut);
  d_partials_.alloc((size_t)kMaxRedBlocks * 3 * 64 + 16);
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_out_), kOut * sizeof(double), hipHostMallocDefault));
  HIP_CHECK(hipStreamSynchronize(s_));
}

GroupedRE::~GroupedRE() {
  if (h_out_) (void)hipHostFree(h_out_);
}

void GroupedRE::SetY(const double* y) {
  d_y_.alloc(n_);
  HIP_CHECK(hipMemcpyAsync(d_y_.get(), y, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
  launch_gre_zty(M_, d_obs_ptr_.get(), d_obs_.get(), d_y_.get(), d_zty_.get(), s_);
  const double* A[1] = {d_y_.get()};
  const double* B[1] = {d_y_.get()};
  launch_coldots(n_, 1, 1, A, B, d_partials_.get(), d_yty_.get(), s_);
  HIP_CHECK(hipStreamSynchronize(s_));
  y_set_ = true;
}

GroupedRE::Block& GroupedRE::GetBlock(int which, int t, int pmax) {
  std::unique_ptr<Block>& bp = which == 0 ? b1_ : bt_;
  if (!bp) bp.reset(new Block());
  Block& b = *bp;
  if (b.t != t) {
    const size_t mt = (size_t)M_ * t;
    for (auto* buf : {&b.R, &b.Z, &b.H, &b.V, &b.U, &b.S}) buf->alloc(mt);
    b.small.alloc((size_t)6 * t);
    b.t = t;
  }
  if (b.a_hist.size() < (size_t)(pmax + 1) * t) {
    b.a_hist.alloc((size_t)(pmax + 1) * t);
    b.b_hist.alloc((size_t)(pmax + 1) * t);
  }
  if (d_partials_.size() < (size_t)kMaxRedBlocks * 3 * t) d_partials_.alloc((size_t)kMaxRedBlocks * 3 * t);
  return b;
}

const GroupedRE::ChunkPlan& GroupedRE::Plan(int tc) {
  auto it = plans_.find(tc);
  if (it != plans_.end()) return *it->second;
  std::unique_ptr<ChunkPlan> pl(new ChunkPlan());
  const int L = gre_chunk_len(tc);
  for (int kind = 0; kind < 3; ++kind) {   // full, lower, upper entry ranges of every row
    std::vector<int> e0, e1, ptr(M_ + 1, 0);
    for (int r = 0; r < M_; ++r) {
      const int a = kind == 2 ? split_h_[r] : rowptr_h_[r];
      const int b = kind == 1 ? split_h_[r] : rowptr_h_[r + 1];
      for (int e = a; e < b; e += L) {
        e0.push_back(e);
        e1.push_back(std::min(e + L, b));
      }
      ptr[r + 1] = (int)e0.size();
    }
    pl->n[kind] = (int)e0.size();
    const size_t nc = std::max<size_t>(e0.size(), 1);
    pl->e0[kind].alloc(nc);
    pl->e1[kind].alloc(nc);
    pl->ptr[kind].alloc(M_ + 1);
    if (!e0.empty()) {
      HIP_CHECK(hipMemcpyAsync(pl->e0[kind].get(), e0.data(), sizeof(int) * e0.size(), hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipMemcpyAsync(pl->e1[kind].get(), e1.data(), sizeof(int) * e1.size(), hipMemcpyHostToDevice, s_));
    }
    HIP_CHECK(hipMemcpyAsync(pl->ptr[kind].get(), ptr.data(), sizeof(int) * (M_ + 1), hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));   // the host vectors go out of scope
    if (kind == 1 || kind == 2) {
      std::vector<int>& q = kind == 1 ? pl->lower_q : pl->upper_q;
      q.resize(K_ + 1);
      for (int k = 0; k <= K_; ++k) q[k] = ptr[cum_[k]];
    }
  }
  ChunkPlan& ref = *pl;
  plans_[tc] = std::move(pl);
  return ref;
}

GroupedOp GroupedRE::Op(int t) {
  GroupedOp op;
  op.M = M_;
  op.rowptr = d_rowptr_.get();
  op.split = d_split_.get();
  op.col = d_col_.get();
  op.val = d_val_.get();
  op.tc = gre_tc(t);
  const ChunkPlan& pl = Plan(op.tc);
  GreChunks* ch[3] = {&op.full, &op.lower, &op.upper};
  for (int kind = 0; kind < 3; ++kind) {
    ch[kind]->n = pl.n[kind];
    ch[kind]->e0 = pl.e0[kind].get();
    ch[kind]->e1 = pl.e1[kind].get();
    ch[kind]->ptr = pl.ptr[kind].get();
  }
  const size_t need = (size_t)std::max(pl.n[0], std::max(pl.n[1], pl.n[2])) * t + 1;
  if (d_chunk_partials_.size() < need) d_chunk_partials_.alloc(need);
  op.P = d_chunk_partials_.get();
  return op;
}

void GroupedRE::Diag(const double* tau) {
  HIP_CHECK(hipMemcpyAsync(d_tau_.get(), tau, sizeof(double) * K_, hipMemcpyHostToDevice, s_));
  launch_gre_diag(K_, d_cum_.get(), d_cnt_.get(), d_tau_.get(), d_D_.get(), d_sqrtD_.get(), d_dsum_.get(), s_);
}

void GroupedRE::ApplyA(const double* X, double* Y, int t, bool with_sigma_inv) {
  launch_gre_apply(Op(t), with_sigma_inv ? d_D_.get() : d_cnt_.get(), X, Y, t, s_);
}

void GroupedRE::Precond(const double* R, double* Z, double* S, int t) {
  const GroupedOp op = Op(t);
  const ChunkPlan& pl = Plan(op.tc);
  launch_gre_ssor(op, cum_, pl.lower_q, pl.upper_q, d_D_.get(), d_sqrtD_.get(), R, S, Z, t, s_);
}

// CGRandomEffectsVec (block = false; CG_utils.cpp:1100-1230) and CGTridiagRandomEffects (block =
// true; :1232-1400) with the SSOR preconditioner, U initialised to 0.
int GroupedRE::Pcg(Block& b, const double* RHS, double* U, bool block, int pmax, double delta, bool warm) {
  const int t = b.t;
  const size_t mt = (size_t)M_ * t;
  double* rz = b.small.get();
  double* rz_new = rz + t;
  double* hv = rz + 2 * t;
  double* rr = rz + 3 * t;
  double* a = rz + 4 * t;
  double* bb = rz + 5 * t;
  if (!block) {   // rhs de facto 0 (CG_utils.cpp:1127-1131)
    const double* A[1] = {RHS};
    const double* B[1] = {RHS};
    launch_coldots(M_, 1, 1, A, B, d_partials_.get(), d_out_.get(), s_);
    HIP_CHECK(hipMemcpyAsync(h_out_, d_out_.get(), sizeof(double), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    if (std::sqrt(h_out_[0]) * std::sqrt((double)M_) < kZeroRhsAbs) {   // sum|x| <= sqrt(M) ||x||
      HIP_CHECK(hipMemsetAsync(U, 0, sizeof(double) * mt, s_));
      return 0;
    }
  }
  if (warm && !block) {
    ApplyA(U, b.V.get(), t, true);
    launch_gre_residual(mt, RHS, b.V.get(), b.R.get(), s_);
  } else {
    HIP_CHECK(hipMemsetAsync(U, 0, sizeof(double) * mt, s_));
    launch_copy(mt, RHS, b.R.get(), s_);
  }
  Precond(b.R.get(), b.Z.get(), b.S.get(), t);
  launch_copy(mt, b.Z.get(), b.H.get(), s_);
  {
    const double* A[1] = {b.R.get()};
    const double* B[1] = {b.Z.get()};
    launch_coldots(M_, t, 1, A, B, d_partials_.get(), rz, s_);
  }
  pmax = std::min(pmax, M_);
  int its = pmax;
  for (int j = 0; j < pmax; ++j) {
    ApplyA(b.H.get(), b.V.get(), t, true);
    {
      const double* A[1] = {b.H.get()};
      const double* B[1] = {b.V.get()};
      launch_coldots(M_, t, 1, A, B, d_partials_.get(), hv, s_);
    }
    launch_cg_alpha(t, rz, hv, nullptr, a, b.a_hist.get() + (size_t)j * t, s_);
    launch_cg_update(M_, t, a, b.H.get(), b.V.get(), U, b.R.get(), d_partials_.get(), rr, s_);
    HIP_CHECK(hipMemcpyAsync(h_out_, rr, sizeof(double) * t, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    double norm = 0.;
    for (int c = 0; c < t; ++c) norm += std::sqrt(h_out_[c]);
    norm /= t;   // single column: ||r||; block: mean column norm (CG_utils.cpp:1353)
    if (std::isnan(norm) || std::isinf(norm))
      Fatal("There was Nan or Inf value generated in the Conjugate Gradient Method!");
    const bool stop = norm < delta;
    if (stop && !block) return j + 1;
    Precond(b.R.get(), b.Z.get(), b.S.get(), t);
    {
      const double* A[1] = {b.R.get()};
      const double* B[1] = {b.Z.get()};
      launch_coldots(M_, t, 1, A, B, d_partials_.get(), rz_new, s_);
    }
    launch_cg_beta(t, rz_new, rz, nullptr, bb, b.b_hist.get() + (size_t)j * t, s_);
    launch_h_update(M_, t, bb, b.Z.get(), b.H.get(), s_);
    if (stop) {
      its = j + 1;
      break;
    }
  }
  return its;
}

void GroupedRE::CheckMethod(const double* tau, bool iterative) const {
  if (!y_set_) Fatal("response variable y has not been set");
  for (int k = 0; k < K_; ++k)
    if (!(tau[k] > 0.)) Fatal("covariance parameters must be > 0");
  if (iterative && K_ < 2)
    Fatal("Cannot use matrix_inversion_method = 'iterative' if there is only a single-level grouped random effects. "
          "Use matrix_inversion_method = 'cholesky' instead (this is very fast). Iterative methods are for multiple "
          "grouped random effects ");
  if (!iterative && K_ > 1 && M_ > kDenseMaxM)
    Fatal("matrix_inversion_method 'cholesky' with several grouped random effects: %d random effects exceed the "
          "dense factor's limit of %d in gpboost_amd (use 'iterative')", M_, kDenseMaxM);
}

void GroupedRE::DenseFactor() {
  // A = Sigma^-1 + Z^T Z dense (diag(A) = D from Diag), in-place Cholesky, log|A|, the inverse factor
  const int M = M_;
  if (ldM_ == 0) {
    ldM_ = (M + 63) / 64 * 64;
    const size_t mm = (size_t)ldM_ * ldM_;
    dA_.alloc(mm);
    dW_.alloc(mm);
    dLiT_.alloc(mm);
    dX_.alloc((size_t)ldM_ * (ldM_ / 2 + 64));
    d_invdiag_.alloc(M);
    d_tmpM_.alloc(ldM_);
    d_info_.alloc(1);
    HIP_CHECK(hipMemsetAsync(dW_.get(), 0, sizeof(double) * mm, s_));
  }
  const int ld = ldM_;
  HIP_CHECK(hipMemsetAsync(dA_.get(), 0, sizeof(double) * (size_t)ld * ld, s_));
  HIP_CHECK(hipMemsetAsync(d_info_.get(), 0, sizeof(int), s_));
  launch_gre_dense_build(M, ld, d_rowptr_.get(), d_col_.get(), d_val_.get(), d_D_.get(), dA_.get(), s_);
  chol_lower(s_, dA_.get(), dW_.get(), M, ld, d_info_.get());
  launch_logdet_chol(s_, dA_.get(), ld, M, d_out_.get() + kOut - 3);
  trtri_lower(s_, dA_.get(), dW_.get(), dX_.get(), 0, M, ld);
  fitc_lower_t(s_, dW_.get(), M, ld, dLiT_.get());
  launch_gre_inv_diag(M, ld, dW_.get(), d_invdiag_.get(), s_);
  fitc_chol_solve(s_, dW_.get(), dLiT_.get(), d_zty_.get(), M, ld, d_tmpM_.get(), d_u_.get());
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, d_info_.get(), sizeof(int), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipMemcpyAsync(h_out_ + kOut - 3, d_out_.get() + kOut - 3, sizeof(double), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  if (info != 0) Fatal("the matrix Sigma^-1 + Z^T Z is not positive definite");
  dense_logdet_ = h_out_[kOut - 3];
}

// u = A^-1 Z^T y (CalcYAux, re_model_template.h:8965-9003): K == 1 closed form (single_sums: the
// pinned slots receiving sum cnt and sum cnt^2 / D), else SSOR-PCG. Returns the PCG iterations.
int GroupedRE::SolveU(bool iterative, bool warm, const IterativeConfig& cfg, double* single_sums) {
  int its = 0;
  if (!iterative && K_ > 1) {
    DenseFactor();
  } else if (!iterative) {   // A diagonal: u = Z^T y / D
    launch_gre_single(M_, d_zty_.get(), d_cnt_.get(), d_D_.get(), d_u_.get(), d_out_.get() + kOut - 2, s_);
    HIP_CHECK(hipMemcpyAsync(single_sums, d_out_.get() + kOut - 2, sizeof(double) * 2, hipMemcpyDeviceToHost, s_));
  } else {
    Block& b1 = GetBlock(0, 1, std::max(cfg.cg_max_num_it, 1));
    its = Pcg(b1, d_zty_.get(), d_u_.get(), false, std::max(cfg.cg_max_num_it, 1), cfg.cg_delta_conv,
              warm && u_valid_);
  }
  u_valid_ = true;
  return its;
}

void GroupedRE::Blup(const double* tau, bool iterative, bool warm, const IterativeConfig& cfg, double* b,
                     double* var) {
  // PredictTrainingDataRandomEffects, grouped branch (re_model_template.h:4065-4167): posterior means
  // tau_k Z_k^T Psi^-1 y = tau_k (Z^T y - Z^T Z u)_k; K == 1 variances tau (1 - tau (cnt - cnt^2 / D))
  CheckMethod(tau, iterative);
  Diag(tau);
  double* single_sums = h_out_ + kOut - 2;
  SolveU(iterative, warm, cfg, single_sums);
  ApplyA(d_u_.get(), d_ztzu_.get(), 1, false);
  std::vector<double> zty(M_), ztzu(M_), D, cnt;
  HIP_CHECK(hipMemcpyAsync(zty.data(), d_zty_.get(), sizeof(double) * M_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipMemcpyAsync(ztzu.data(), d_ztzu_.get(), sizeof(double) * M_, hipMemcpyDeviceToHost, s_));
  std::vector<double> invdiag;
  if (var != nullptr && K_ > 1) {   // cholesky (iterative is refused by the caller): diag(A^-1)
    invdiag.resize(M_);
    HIP_CHECK(hipMemcpyAsync(invdiag.data(), d_invdiag_.get(), sizeof(double) * M_, hipMemcpyDeviceToHost, s_));
  } else if (var != nullptr) {
    D.resize(M_);
    cnt.resize(M_);
    HIP_CHECK(hipMemcpyAsync(D.data(), d_D_.get(), sizeof(double) * M_, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipMemcpyAsync(cnt.data(), d_cnt_.get(), sizeof(double) * M_, hipMemcpyDeviceToHost, s_));
  }
  HIP_CHECK(hipStreamSynchronize(s_));
  for (int k = 0; k < K_; ++k)
    for (int r = cum_[k]; r < cum_[k + 1]; ++r) {
      b[r] = tau[k] * (zty[r] - ztzu[r]);
      if (var != nullptr && K_ > 1) {
        var[r] = invdiag[r];   // tau + tau^2 (M_aux^T M_aux - Z_j^T Z_j)_rr = (A^-1)_rr (:4122-4139)
      } else if (var != nullptr) {
        const double ma = cnt[r] / std::sqrt(D[r]);   // M_aux (:4088-4091)
        var[r] = tau[k] - tau[k] * tau[k] * (cnt[r] - ma * ma);
      }
    }
}

void GroupedRE::PredCov(int np, const std::vector<int>& idx, bool want_cov, double* out) {
  if (np <= 0) return;
  if (K_ == 1) {   // A^-1 = diag(1/D)
    std::vector<double> D(M_);
    HIP_CHECK(hipMemcpyAsync(D.data(), d_D_.get(), sizeof(double) * M_, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    if (want_cov) {
      for (int q = 0; q < np; ++q)
        for (int p = 0; p < np; ++p)
          out[(size_t)q * np + p] = (idx[p] >= 0 && idx[p] == idx[q]) ? 1. / D[idx[p]] : 0.;
    } else {
      for (int p = 0; p < np; ++p) out[p] = idx[p] >= 0 ? 1. / D[idx[p]] : 0.;
    }
    return;
  }
  if (ldM_ == 0) Fatal("predictive variances need the Cholesky factor (matrix_inversion_method = 'cholesky')");
  const int ld = ldM_;
  DevBuf<int> d_idx(idx.size());
  HIP_CHECK(hipMemcpyAsync(d_idx.get(), idx.data(), sizeof(int) * idx.size(), hipMemcpyHostToDevice, s_));
  if (want_cov) {
    DevBuf<double> E((size_t)ld * np), C((size_t)np * np);
    HIP_CHECK(hipMemsetAsync(E.get(), 0, sizeof(double) * (size_t)ld * np, s_));
    launch_gre_pred_cols(M_, ld, K_, np, d_idx.get(), dW_.get(), E.get(), nullptr, s_);
    gemm_f64(s_, np, np, M_, 1., E.get(), ld, 1, E.get(), ld, 0, 0., C.get(), np);
    HIP_CHECK(hipMemcpyAsync(out, C.get(), sizeof(double) * (size_t)np * np, hipMemcpyDeviceToHost, s_));
  } else {
    DevBuf<double> v(np);
    launch_gre_pred_cols(M_, ld, K_, np, d_idx.get(), dW_.get(), nullptr, v.get(), s_);
    HIP_CHECK(hipMemcpyAsync(out, v.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
  }
  HIP_CHECK(hipStreamSynchronize(s_));
}

void GroupedRE::Fisher(const double* tau, double sigma2, double* FI) {
  const int K = K_, M = M_;
  std::vector<double> F, tr;
  FisherParts(tau, F, tr);
  const int P = 1 + K;
  const double c4 = 0.5 / (sigma2 * sigma2);
  double f00 = (double)n_ - M;
  for (double v : F) f00 += v;
  FI[0] = f00 * c4;
  for (int j = 0; j < K; ++j) {
    double rs = 0.;
    for (int k = 0; k < K; ++k) rs += F[(size_t)j * K + k];
    FI[j + 1] = FI[(size_t)(j + 1) * P] = (tr[j] - rs) / tau[j] * c4;
    for (int k = j; k < K; ++k) {
      const double v = (F[(size_t)j * K + k] + (j == k ? m_[j] - 2. * tr[j] : 0.)) / (tau[j] * tau[k]) * c4;
      FI[(size_t)(j + 1) * P + k + 1] = FI[(size_t)(k + 1) * P + j + 1] = v;
    }
  }
}

void GroupedRE::FisherParts(const double* tau, std::vector<double>& F, std::vector<double>& tr) {
  CheckMethod(tau, false);
  const int K = K_, M = M_;
  Diag(tau);
  F.assign((size_t)K * K, 0.);
  tr.assign(K, 0.);
  if (K == 1) {   // A^-1 = diag(1/D): B_rr = 1 / (tau D_r)
    std::vector<double> D(M);
    HIP_CHECK(hipMemcpyAsync(D.data(), d_D_.get(), sizeof(double) * M, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    for (int r = 0; r < M; ++r) {
      const double b = 1. / (tau[0] * D[r]);
      F[0] += b * b;
      tr[0] += b;
    }
  } else {
    DenseFactor();
    const int ld = ldM_;
    // A^-1 = L^-T L^-1 = LiT LiT^T (the clean transposed factor; L itself is not needed any more)
    gemm_f64(s_, M, M, M, 1., dLiT_.get(), ld, 0, dLiT_.get(), ld, 1, 0., dA_.get(), ld);
    std::vector<double> sc(M);
    for (int k = 0; k < K; ++k)
      for (int r = cum_[k]; r < cum_[k + 1]; ++r) sc[r] = 1. / std::sqrt(tau[k]);
    DevBuf<double> dsc(M), dpart((size_t)M * K), ddiag(M);
    HIP_CHECK(hipMemcpyAsync(dsc.get(), sc.data(), sizeof(double) * M, hipMemcpyHostToDevice, s_));
    launch_gre_fisher_cols(M, ld, K, d_cum_.get(), dsc.get(), dA_.get(), dpart.get(), ddiag.get(), s_);
    std::vector<double> part((size_t)M * K), diag(M);
    HIP_CHECK(hipMemcpyAsync(part.data(), dpart.get(), sizeof(double) * part.size(), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipMemcpyAsync(diag.data(), ddiag.get(), sizeof(double) * M, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    for (int k = 0; k < K; ++k)
      for (int c = cum_[k]; c < cum_[k + 1]; ++c) {
        tr[k] += diag[c];
        for (int j = 0; j < K; ++j) F[(size_t)j * K + k] += part[(size_t)c * K + j];
      }
  }
}

void GroupedRE::Eval(const double* tau, bool want_grad, bool iterative, bool warm, const IterativeConfig& cfg,
                     GroupedParts& out) {
  CheckMethod(tau, iterative);
  out = GroupedParts();
  out.quad.assign(K_, 0.);
  out.trace.assign(K_, 0.);
  Diag(tau);
  int t = 1;
  double* single_sums = h_out_ + kOut - 2;   // pinned, read after the next synchronisation
  out.cg_its = SolveU(iterative, warm, cfg, single_sums);
  // y^T Psi^-1 y = y^T y - (Z^T y)^T u ; the per-effect sums of log D and 1/D
  {
    const double* A[1] = {d_zty_.get()};
    const double* B[1] = {d_u_.get()};
    launch_coldots(M_, 1, 1, A, B, d_partials_.get(), d_out_.get(), s_);
    HIP_CHECK(hipMemcpyAsync(h_out_, d_out_.get(), sizeof(double), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipMemcpyAsync(h_out_ + 1, d_yty_.get(), sizeof(double), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipMemcpyAsync(h_out_ + 2, d_dsum_.get(), sizeof(double) * 2 * K_, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
  }
  out.yTPsiInvy = h_out_[1] - h_out_[0];
  std::vector<double> sum_logD(h_out_ + 2, h_out_ + 2 + K_), sum_Dinv(h_out_ + 2 + K_, h_out_ + 2 + 2 * K_);
  double logdet = 0.;
  if (!iterative && K_ > 1) {
    logdet = dense_logdet_;   // 2 sum log L_ii (re_model_template.h:2780)
  } else if (!iterative) {
    for (int k = 0; k < K_; ++k) logdet += sum_logD[k];   // 2 sum log sqrt(D) (re_model_template.h:2780)
  } else {
    // ---- SLQ: probes r ~ N(0, I) (GenRandVecNormalParallel), P-distributed L D^-1/2 r, block PCG
    t = cfg.num_rand_vec_trace;
    if (t < 1 || t > 1024) Fatal("num_rand_vec_trace = %d outside [1, 1024]", t);
    if (!(probes_saved_ && probes_t_ == t)) {
      std::vector<double> R((size_t)M_ * t);
      gen_probes_normal(M_, t, cfg.seed_rand_vec_trace, probe_run_id_, R.data());
      ++probe_run_id_;
      d_probes_.alloc(R.size());
      HIP_CHECK(hipMemcpyAsync(d_probes_.get(), R.data(), sizeof(double) * R.size(), hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipStreamSynchronize(s_));   // R is pageable and goes out of scope
      probes_t_ = t;
      probes_saved_ = cfg.reuse_rand_vec_trace;
    }
    d_probesP_.alloc((size_t)M_ * t);
    launch_gre_lds_mult(Op(t), d_D_.get(), d_sqrtD_.get(), d_probes_.get(), d_probesP_.get(), t, s_);
    const int pmax = std::max(1, std::min(cfg.cg_max_num_it_tridiag, M_));
    Block& bt = GetBlock(1, t, pmax);
    const int L = Pcg(bt, d_probesP_.get(), bt.U.get(), true, pmax, cfg.cg_delta_conv);
    out.lanczos_steps = L;
    std::vector<double> ah((size_t)L * t), bh((size_t)std::max(L - 1, 1) * t);
    HIP_CHECK(hipMemcpyAsync(ah.data(), bt.a_hist.get(), sizeof(double) * ah.size(), hipMemcpyDeviceToHost, s_));
    if (L > 1)
      HIP_CHECK(hipMemcpyAsync(bh.data(), bt.b_hist.get(), sizeof(double) * (size_t)(L - 1) * t, hipMemcpyDeviceToHost,
                               s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    std::vector<std::vector<double>> Td(t), Ts(t);
    for (int c = 0; c < t; ++c) {   // CG_utils.cpp:1383-1388 (a_old = 1, b_old = 0 before the first step)
      Td[c].resize(L);
      Ts[c].resize(L > 0 ? L - 1 : 0);
      for (int j = 0; j < L; ++j) {
        const double aj = ah[(size_t)j * t + c];
        const double a_old = j > 0 ? ah[(size_t)(j - 1) * t + c] : 1.;
        const double b_old = j > 0 ? bh[(size_t)(j - 1) * t + c] : 0.;
        Td[c][j] = 1. / aj + b_old / a_old;
        if (j > 0) Ts[c][j - 1] = std::sqrt(b_old) / a_old;
      }
    }
    logdet = slq_logdet(Td, Ts, M_);
    for (int k = 0; k < K_; ++k) logdet += sum_logD[k];   // log|P| = 2 sum log(D sqrt(1/D)) (:2848-2851)
  }
  for (int k = 0; k < K_; ++k) logdet += m_[k] * std::log(tau[k]);   // log|Sigma| (:2868-2871)
  out.logdet = logdet;
  if (!want_grad) return;

  // ---- gradient (CalcGradPars_Only_Grouped_REs_Woodbury_GaussLikelihood_Cluster_i, :2242-2391)
  ApplyA(d_u_.get(), d_ztzu_.get(), 1, false);   // Z^T Z u = Z^T y_tilde2
  for (int k = 0; k < K_; ++k) {
    const size_t o = cum_[k];
    const double* A[3] = {d_zty_.get() + o, d_zty_.get() + o, d_ztzu_.get() + o};
    const double* B[3] = {d_zty_.get() + o, d_ztzu_.get() + o, d_ztzu_.get() + o};
    launch_coldots(m_[k], 1, 3, A, B, d_partials_.get(), d_out_.get() + 3 * k, s_);
  }
  HIP_CHECK(hipMemcpyAsync(h_out_, d_out_.get(), sizeof(double) * 3 * K_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  for (int k = 0; k < K_; ++k)
    out.quad[k] = (h_out_[3 * k] - 2. * h_out_[3 * k + 1] + h_out_[3 * k + 2]) * tau[k];
  if (!iterative && K_ > 1) {   // tr(Psi^-1 dPsi_k) = m_k - tr(A^-1_kk) / tau_k (:2279-2296)
    std::vector<double> invdiag(M_);
    HIP_CHECK(hipMemcpyAsync(invdiag.data(), d_invdiag_.get(), sizeof(double) * M_, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    for (int k = 0; k < K_; ++k) {
      double tr = 0.;
      for (int r = cum_[k]; r < cum_[k + 1]; ++r) tr += invdiag[r];
      out.trace[k] = m_[k] - tr / tau[k];
    }
    return;
  }
  if (!iterative) {   // tr(Psi^-1 dPsi_k) = tau_k (sum cnt - sum cnt^2 / D) (:2279-2296)
    out.trace[0] = (single_sums[0] - single_sums[1]) * tau[0];
    return;
  }
  Block& bt = GetBlock(1, t, 1);
  d_PI_.alloc((size_t)M_ * t);
  d_DI_.alloc((size_t)M_ * t);
  Precond(d_probesP_.get(), d_PI_.get(), bt.S.get(), t);               // PI_RV = P^-1 z
  launch_gre_upper(Op(t), d_D_.get(), d_PI_.get(), d_DI_.get(), t, s_);  // DI_L_plus_D_t_PI_RV
  std::vector<double> sums((size_t)3 * t * K_);
  d_sums3_.alloc((size_t)3 * t * K_);   // own scratch: M x t blocks can be smaller than 3 t (M < 3)
  for (int k = 0; k < K_; ++k) {
    const size_t o = (size_t)cum_[k] * t;
    const double* A[3] = {bt.U.get() + o, d_PI_.get() + o, d_DI_.get() + o};
    const double* B[3] = {d_PI_.get() + o, d_DI_.get() + o, d_DI_.get() + o};
    launch_coldots(m_[k], t, 3, A, B, d_partials_.get(), d_sums3_.get() + (size_t)3 * t * k, s_);
  }
  HIP_CHECK(hipMemcpyAsync(sums.data(), d_sums3_.get(), sizeof(double) * sums.size(), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  std::vector<double> z1(t), zP(t);
  for (int k = 0; k < K_; ++k) {
    const double* q = sums.data() + (size_t)3 * t * k;
    const double inv = 1. / tau[k];   // -dSigma^-1 / dlog tau_k on effect k
    double tr1 = 0., trP = 0.;
    for (int c = 0; c < t; ++c) {
      z1[c] = -(q[c] * inv);
      zP[c] = -2. * (q[t + c] * inv) + q[2 * t + c] * inv;
      tr1 += z1[c];
      trP += zP[c];
    }
    tr1 /= t;
    trP /= t;
    const double trD = -(sum_Dinv[k] * inv);
    const double copt = optimal_c(z1.data(), zP.data(), t, tr1, trP);
    out.trace[k] = tr1 + copt * (trD - trP) + m_[k];
  }
}

}  // namespace gpb_amd
