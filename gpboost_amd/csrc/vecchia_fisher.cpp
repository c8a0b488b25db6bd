// VecchiaFisher: the stochastic-trace Fisher information of the Gaussian Vecchia model (vecchia_fisher.h).
#include "vecchia_fisher.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "cov.h"
#include "latent_kernels.h"
#include "slq_host.h"

namespace gpb_amd {

// Y = Do .* (dD .* W - U) over n x t blocks (vecchia_fisher.hip)
void launch_fisher_mix(int n, int t, const double* Do, const double* dD, const double* U, const double* W, double* Y,
                       hipStream_t s);

namespace {
int env_rows(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::max(0, std::atoi(e)) : dflt;
}
}  // namespace

VecchiaFisher::VecchiaFisher(int n, int d, int m, const double* d_X, const int* d_nbr, const std::vector<int>& nbr,
                             hipStream_t stream)
    : n_(n), d_(d), m_(m), s_(stream), d_X_(d_X), d_nbr_(d_nbr) {
  if (m > 64) Fatal("standard deviations for the Vecchia approximation support num_neighbors <= 64, got %d", m);
  if ((int)nbr.size() != n * m) Fatal("VecchiaFisher: neighbour table of %zu entries, expected %d", nbr.size(), n * m);
  // B^T lists (column j -> rows ascending, value slot row * m + r), as LatentVecchia::BuildStructure
  std::vector<int> cnt(n + 1, 0);
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < std::min(i, m); ++r) ++cnt[nbr[(size_t)i * m + r] + 1];
  std::vector<int> tptr(n + 1, 0);
  for (int j = 0; j < n; ++j) tptr[j + 1] = tptr[j] + cnt[j + 1];
  const int nnz = tptr[n];
  std::vector<int> trow(std::max(nnz, 1)), tslot(std::max(nnz, 1)), fill(tptr.begin(), tptr.end() - 1);
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < std::min(i, m); ++r) {
      const int j = nbr[(size_t)i * m + r];
      trow[fill[j]] = i;
      tslot[fill[j]] = i * m + r;
      ++fill[j];
    }
  // the VADU plan over identity storage labels (the model order is the Vecchia order); the same head
  // split as the latent solver (latent.cpp: dense head 2048 rows, LDS segment to 14336)
  std::vector<int> id(n);
  for (int i = 0; i < n; ++i) id[i] = i;
  std::vector<int> nb0(nbr);
  for (auto& v : nb0) v = std::max(v, 0);
  const int K0 = std::min(env_rows("GPBOOST_AMD_DENSE_ROWS", 2048), n);
  const int K = std::max(std::min(env_rows("GPBOOST_AMD_HEAD_ROWS", 14336), n), K0);
  pre_.reset(new VaduPrecond(n, m, s_));
  pre_->Build(nb0.data(), id, id, tptr, trow, tslot, K0, K);
  tptr_.alloc(n + 1);
  trow_.alloc(trow.size());
  tslot_.alloc(tslot.size());
  HIP_CHECK(hipMemcpyAsync(tptr_.get(), tptr.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(trow_.get(), trow.data(), sizeof(int) * trow.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(tslot_.get(), tslot.data(), sizeof(int) * tslot.size(), hipMemcpyHostToDevice, s_));
  for (auto* b : {&Bv_, &dBv0_, &dBv1_}) b->alloc((size_t)n * m);
  for (auto* b : {&Dinv_, &dD0_, &dD1_, &Do_, &mones_}) b->alloc(n);
  const std::vector<double> mones(n, -1.);
  HIP_CHECK(hipMemcpyAsync(mones_.get(), mones.data(), sizeof(double) * n, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

VecchiaFisher::~VecchiaFisher() { pre_.reset(); }

void VecchiaFisher::Fisher(int cov_type, const double* orig, const double* trafo, int t, int seed, uint64_t run_id,
                           double* FI) {
  const int n = n_, m = m_;
  if (t < 1) Fatal("num_rand_vec_trace must be > 0");
  if (!(orig[0] > 0. && orig[1] > 0. && orig[2] > 0.)) Fatal("covariance parameters must be > 0");
  if (t != t_) {
    for (auto* b : {&Z_, &P_, &W_, &T_, &U_, &G_[0], &G_[1], &G_[2]}) b->alloc((size_t)n * t);
    part_.alloc((size_t)kMaxRedBlocks * 3 * t);
    red_.alloc((size_t)3 * t);
    t_ = t;
  }
  // 1. B, D^-1 and their derivatives on the transformed scale (nugget 1)
  LatentFactorArgs fa{};
  fa.X = d_X_; fa.nbr = d_nbr_; fa.n = n; fa.d = d_; fa.m = m;
  fa.var = trafo[1]; fa.phi = trafo[2];
  fa.jitter = 1.;
  fa.nugget = 1.;
  fa.Bv = Bv_.get(); fa.Dinv = Dinv_.get();
  fa.dBv = dBv1_.get(); fa.dD = dD1_.get();
  fa.dBv_var = dBv0_.get(); fa.dD_var = dD0_.get();
  launch_latent_factor(cov_type, fa, s_);
  // 2. Sigma_t z = B^-1 D B^-T z (P) and B^-T z (W) by one VADU application with dw = D^-1
  std::vector<double> Zh((size_t)n * t);
  gen_probes_normal(n, t, seed, run_id, Zh.data());
  HIP_CHECK(hipMemcpyAsync(Z_.get(), Zh.data(), sizeof(double) * Zh.size(), hipMemcpyHostToDevice, s_));
  pre_->Refresh(Bv_.get());
  pre_->SetDiag(Dinv_.get());
  pre_->Apply(Z_.get(), P_.get(), U_.get(), t);
  SparseB B{};
  B.n = n; B.m = m; B.nbr = d_nbr_; B.tptr = tptr_.get(); B.trow = trow_.get(); B.tslot = tslot_.get();
  // B^-T z = D^-1 B (B^-1 D B^-T z): the plan's own B^-T scratch holds only partial sums on its dense-head rows
  launch_b_apply(B, Bv_.get(), true, P_.get(), t, Dinv_.get(), W_.get(), s_);
  // 3. original scale (CalcStdDevCovPar's transf_scale = false, Vecchia_utils.cpp:1353, 1474-1489, 1500-1520)
  const double s2 = orig[0], v1 = orig[1], rho = orig[2];
  const double g = (cov_type == kGaussian ? -2. : -1.) / rho;   // dlog(phi) / drho
  const size_t nm = (size_t)n * m, nt = (size_t)n * t;
  launch_axpby(n, 1. / s2, Dinv_.get(), 0., Dinv_.get(), Do_.get(), s_);          // D_o^-1
  launch_axpby(nm, 1. / v1, dBv0_.get(), 0., dBv0_.get(), dBv0_.get(), s_);       // dB / dsigma1^2
  launch_axpby(n, s2 / v1, dD0_.get(), 0., dD0_.get(), dD0_.get(), s_);           // dD / dsigma1^2
  launch_axpby(nm, g, dBv1_.get(), 0., dBv1_.get(), dBv1_.get(), s_);             // dB / drho
  launch_axpby(n, s2 * g, dD1_.get(), 0., dD1_.get(), dD1_.get(), s_);            // dD / drho
  launch_axpby(nt, s2, P_.get(), 0., P_.get(), P_.get(), s_);                     // Sigma_o z
  // 4. g_0 = B^T D^-1 B z; g_k = B^T D^-1 (dD_k B^-T z - dB_k Sigma z) - dB_k^T B^-T z
  launch_b_apply(B, Bv_.get(), true, Z_.get(), t, Do_.get(), T_.get(), s_);
  launch_bt_apply(B, Bv_.get(), true, T_.get(), t, nullptr, nullptr, nullptr, G_[0].get(), s_);
  const double* dBk[2] = {dBv0_.get(), dBv1_.get()};
  const double* dDk[2] = {dD0_.get(), dD1_.get()};
  for (int k = 0; k < 2; ++k) {
    launch_b_apply(B, dBk[k], false, P_.get(), t, nullptr, U_.get(), s_);                          // dB_k Sigma z
    launch_fisher_mix(n, t, Do_.get(), dDk[k], U_.get(), W_.get(), T_.get(), s_);
    launch_bt_apply(B, dBk[k], false, W_.get(), t, nullptr, nullptr, nullptr, U_.get(), s_);        // dB_k^T W
    // G_k = B^T T - U  (the W .* H term of the transposed product with W = -1)
    launch_bt_apply(B, Bv_.get(), true, T_.get(), t, nullptr, mones_.get(), U_.get(), G_[k + 1].get(), s_);
  }
  if (const char* path = std::getenv("GPBOOST_AMD_FISHER_DUMP")) {
    // diagnostics: the original-scale factor and the probe blocks, raw fp64 in this order after
    // the header (n, m, t as doubles): Bv dBv0 dBv1 (n m each) Do dD0 dD1 (n) Z P W G0 G1 G2 (n t)
    HIP_CHECK(hipStreamSynchronize(s_));
    FILE* f = std::fopen(path, "wb");
    if (!f) Fatal("cannot open %s", path);
    const double hdr[3] = {(double)n, (double)m, (double)t};
    std::fwrite(hdr, sizeof(double), 3, f);
    auto put = [&](const double* d, size_t cnt) {
      std::vector<double> h(cnt);
      HIP_CHECK(hipMemcpy(h.data(), d, sizeof(double) * cnt, hipMemcpyDeviceToHost));
      std::fwrite(h.data(), sizeof(double), cnt, f);
    };
    for (const double* p : {Bv_.get(), dBv0_.get(), dBv1_.get()}) put(p, nm);
    for (const double* p : {Do_.get(), dD0_.get(), dD1_.get()}) put(p, n);
    for (const double* p : {Z_.get(), P_.get(), W_.get(), G_[0].get(), G_[1].get(), G_[2].get()}) put(p, nt);
    std::fclose(f);
  }
  // 5. FI_kl = 1/2 mean_c (g_k . g_l)_c
  const double* A1[3] = {G_[0].get(), G_[0].get(), G_[0].get()};
  const double* B1[3] = {G_[0].get(), G_[1].get(), G_[2].get()};
  const double* A2[3] = {G_[1].get(), G_[1].get(), G_[2].get()};
  const double* B2[3] = {G_[1].get(), G_[2].get(), G_[2].get()};
  std::vector<double> h((size_t)6 * t);
  launch_coldots(n, t, 3, A1, B1, part_.get(), red_.get(), s_);
  HIP_CHECK(hipMemcpyAsync(h.data(), red_.get(), sizeof(double) * 3 * t, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  launch_coldots(n, t, 3, A2, B2, part_.get(), red_.get(), s_);
  HIP_CHECK(hipMemcpyAsync(h.data() + 3 * t, red_.get(), sizeof(double) * 3 * t, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  const int kl[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
  for (int q = 0; q < 6; ++q) {
    double s = 0.;
    for (int c = 0; c < t; ++c) s += h[(size_t)q * t + c];
    const double v = 0.5 * s / t;
    FI[kl[q][0] * 3 + kl[q][1]] = v;
    FI[kl[q][1] * 3 + kl[q][0]] = v;
  }
}

}  // namespace gpb_amd
