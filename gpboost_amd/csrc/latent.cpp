// LatentVecchia implementation: host orchestration of the iterative latent-Vecchia path.
#include "latent.h"

#include <algorithm>
#include <random>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <map>
#include <cstring>

#include "kernels.h"
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

namespace {
int env_rows(const char* name, int def) {
  const char* e = std::getenv(name);
  if (!e) return def;
  char* end = nullptr;
  const long v = std::strtol(e, &end, 10);
  if (end == e || *end != '\0' || v < 0 || v > (1L << 30)) Fatal("%s must be a row count >= 0 (got '%s')", name, e);
  return (int)v;
}
}  // namespace

LatentVecchia::LatentVecchia(int n, int d, int m, const double* d_X, const int* nbr, hipStream_t stream)
    : n_(n), d_(d), m_(m), d_X_(d_X), s_(stream) {
  HIP_CHECK(hipEventCreate(&ev0_));
  HIP_CHECK(hipEventCreate(&ev1_));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_out_), kOutDoubles * sizeof(double), hipHostMallocDefault));
  // PCG verdicts: written by the device straight into host-coherent memory (no copy command on
  // the stream between iterations), polled by the host
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_ctl_), 4 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_hctl_), h_ctl_, 0));
  std::fill(h_ctl_, h_ctl_ + 4, -1);   // two 64-bit verdict slots, no sequence number matches
  // VADU plan split (vadu_precond.h): dense head [0, K0), LDS segment [K0, K), level-scheduled
  // tail. K0 = 2048: the first 2048 rows span 201 of the 388 levels of each solve at n = 100k.
  // K = 14336: 112 KB of segment values per column workgroup (K sweep 12288 / 14336 / 16384:
  // 1.741 / 1.719 / 1.732 ms per application at t = 51 with K0 = 0).
  dense_rows_ = std::min(env_rows("GPBOOST_AMD_DENSE_ROWS", 2048), n);
  head_rows_ = std::max(std::min(env_rows("GPBOOST_AMD_HEAD_ROWS", 14336), n), dense_rows_);
  std::vector<int> nbr_p;
  Relabel(nbr, nbr_p);
  BuildStructure(nbr_p.data());
  for (auto* b : {&d_Bv_, &d_dBv_}) b->alloc((size_t)n * m);
  for (auto* b : {&d_y_, &d_Dinv_, &d_dD_, &d_W_, &d_dw_, &d_sdw_, &d_d1_, &d_mode_, &d_mode_upd_, &d_mode_new_,
                  &d_rhs_, &d_dir_, &d_Adir_, &d_vS_, &d_dmll_})
    b->alloc(n);
  d_out_.alloc(kOutDoubles);
  // InitializeModeAvec at construction (re_model_template.h:6346): a warm start before any
  // evaluation starts from 0
  HIP_CHECK(hipMemsetAsync(d_mode_.get(), 0, sizeof(double) * n, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void LatentVecchia::ResetModeToPrevious() {
  if (!mode_prev_valid_) return;
  launch_copy(n_, d_mode_prev_.get(), d_mode_.get(), s_);
  HIP_CHECK(hipStreamSynchronize(s_));
}

LatentVecchia::~LatentVecchia() {
  pre_.reset();
  if (h_out_) (void)hipHostFree(h_out_);
  if (h_ctl_) (void)hipHostFree(h_ctl_);
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

// Host construction of the B^T lists (in the storage labels of Relabel) and of the VADU
// preconditioner plan over them.
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
  pre_.reset(new VaduPrecond(n, m, s_));
  pre_->Build(nbr, vo_, lab_, tptr, trow, tslot, dense_rows_, head_rows_);

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
  {   // LDS tiles of the t >= 2 operator (TileOp): greedy runs of consecutive storage rows
    auto build = [&](bool trans, TileDev& td) {
      std::vector<int> r0{0}, uoff{0}, urow, fb;
      std::vector<uint16_t> lidx(trans ? std::max(nnz, 1) : (size_t)n * m, 0);
      std::vector<unsigned char> isfb(n, 0);
      std::vector<int> stamp(n, -1), loc(n, 0);
      int tile = 0, umax = 0, i = 0;
      auto range = [&](int r, int& e0, int& e1) {
        e0 = trans ? tptr[r] : r * m;
        e1 = trans ? tptr[r + 1] : r * m + std::min(r, m);
      };
      auto id_of = [&](int e) { return trans ? trow[e] : nbr[e]; };
      while (i < n) {
        int rows = 0, nu = 0;
        const int start = i;
        while (i < n && i - start < kTileRows) {   // the kernel covers kTileRows rows of range per tile
          int e0, e1;
          range(i, e0, e1);
          if (e1 - e0 > kTileUnion) {   // a list that alone overflows the LDS union
            isfb[i] = 1;
            fb.push_back(i);
            ++i;
            continue;
          }
          int add = 0;
          for (int e = e0; e < e1; ++e) add += stamp[id_of(e)] != tile;
          if (rows > 0 && nu + add > kTileUnion) break;
          for (int e = e0; e < e1; ++e) {
            const int id = id_of(e);
            if (stamp[id] != tile) {
              stamp[id] = tile;
              loc[id] = nu++;
              urow.push_back(id);
            }
            lidx[e] = (uint16_t)loc[id];
          }
          ++rows;
          ++i;
        }
        r0.push_back(i);
        uoff.push_back((int)urow.size());
        umax = std::max(umax, nu);
        ++tile;
      }
      td.r0.alloc(r0.size());
      td.uoff.alloc(uoff.size());
      td.urow.alloc(std::max<size_t>(urow.size(), 1));
      td.lidx.alloc(lidx.size());
      td.fb.alloc(std::max<size_t>(fb.size(), 1));
      td.isfb.alloc(n);
      HIP_CHECK(hipMemcpy(td.r0.get(), r0.data(), sizeof(int) * r0.size(), hipMemcpyHostToDevice));
      HIP_CHECK(hipMemcpy(td.uoff.get(), uoff.data(), sizeof(int) * uoff.size(), hipMemcpyHostToDevice));
      if (!urow.empty()) HIP_CHECK(hipMemcpy(td.urow.get(), urow.data(), sizeof(int) * urow.size(), hipMemcpyHostToDevice));
      HIP_CHECK(hipMemcpy(td.lidx.get(), lidx.data(), sizeof(uint16_t) * lidx.size(), hipMemcpyHostToDevice));
      if (!fb.empty()) HIP_CHECK(hipMemcpy(td.fb.get(), fb.data(), sizeof(int) * fb.size(), hipMemcpyHostToDevice));
      HIP_CHECK(hipMemcpy(td.isfb.get(), isfb.data(), n, hipMemcpyHostToDevice));
      td.op.ntile = tile;
      td.op.nfb = (int)fb.size();
      td.op.r0 = td.r0.get();
      td.op.uoff = td.uoff.get();
      td.op.urow = td.urow.get();
      td.op.lidx = td.lidx.get();
      td.op.fb = td.fb.get();
      td.op.isfb = td.isfb.get();
      td.op.umax = umax;
    };
    build(false, tile_b_);
    build(true, tile_bt_);
  }
  {   // t = 1 form of B: ELL, column-major (SparseB). A row's entries in ascending storage index:
      // lane l's r-th gather is then the r-th smallest neighbour of row base + l, so the 64 gathers
      // of one load instruction fall on fewer cache lines than in neighbour (distance) order
      // (GPBOOST_AMD_ELL_UNSORTED: distance order, A/B)
    static const bool unsorted = std::getenv("GPBOOST_AMD_ELL_UNSORTED") != nullptr;
    std::vector<int> eidx((size_t)m * n), eslot((size_t)m * n);
    std::vector<std::pair<int, int>> row(m);
    for (int i = 0; i < n; ++i) {
      const int k = std::min(i, m);
      for (int r = 0; r < k; ++r) row[r] = {nbr[(size_t)i * m + r], i * m + r};
      if (!unsorted) std::sort(row.begin(), row.begin() + k);
      for (int r = 0; r < m; ++r) {
        eidx[(size_t)r * n + i] = r < k ? row[r].first : i;
        eslot[(size_t)r * n + i] = r < k ? row[r].second : -1;
      }
    }
    d_ell_idx_.alloc(eidx.size());
    d_ell_slot_.alloc(eslot.size());
    d_ell_val_.alloc(eidx.size());
    HIP_CHECK(hipMemcpy(d_ell_idx_.get(), eidx.data(), sizeof(int) * eidx.size(), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_ell_slot_.get(), eslot.data(), sizeof(int) * eslot.size(), hipMemcpyHostToDevice));
    sp_.ell_idx = d_ell_idx_.get();
    sp_.ell_val = d_ell_val_.get();
    sp_.vals_of = nullptr;
  }
  if (n < (1 << 24)) {   // t = 1 default form of B^T (SparseB::seg_*): runs of consecutive storage
      // rows holding <= kSegEntries entries (a longer row is a run of its own) and <= kSegRows rows,
      // one wave each; per entry one packed word: source row (bits 0-23), the row's index within
      // the run (bits 24-30) and "last entry of its row" (bit 31) for the wave's segmented sums
    std::vector<int> seg{0};
    std::vector<uint32_t> pk(std::max(nnz, 1), 0);
    int ce = 0, cr = 0;
    for (int j = 0; j < n; ++j) {
      const int len = tptr[j + 1] - tptr[j];
      if (cr > 0 && (ce + len > kSegEntries || cr >= kSegRows)) {
        seg.push_back(j);
        ce = 0;
        cr = 0;
      }
      for (int e = tptr[j]; e < tptr[j + 1]; ++e)
        pk[e] = (uint32_t)trow[e] | ((uint32_t)cr << 24) | (e + 1 == tptr[j + 1] ? 0x80000000u : 0u);
      ce += len;
      ++cr;
    }
    seg.push_back(n);
    d_seg_rb_.alloc(seg.size());
    d_seg_pk_.alloc(pk.size());
    HIP_CHECK(hipMemcpy(d_seg_rb_.get(), seg.data(), sizeof(int) * seg.size(), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_seg_pk_.get(), pk.data(), sizeof(uint32_t) * pk.size(), hipMemcpyHostToDevice));
    // entry-pair layout of the runs: each run's entries start at an even position of a padded copy
    // (pad entries: key 127, value 0), so a lane's two entries are one 8-byte and one 16-byte load
    std::vector<int4> info(seg.size() - 1);
    std::vector<uint32_t> pk2;
    std::vector<int> slot2;
    for (size_t w = 0; w + 1 < seg.size(); ++w) {
      const int a = tptr[seg[w]], b = tptr[seg[w + 1]];
      const int p0 = (int)pk2.size();
      for (int e = a; e < b; ++e) { pk2.push_back(pk[e]); slot2.push_back(tslot[e]); }
      if ((b - a) & 1) { pk2.push_back((uint32_t)kSegRows << 24); slot2.push_back(-1); }
      info[w] = make_int4(seg[w], seg[w + 1], p0, p0 + (b - a));
    }
    seg2_n_ = (int)pk2.size();
    d_seg_info_.alloc(std::max<size_t>(info.size(), 1));
    d_seg_pk2_.alloc(std::max<size_t>(pk2.size(), 2));
    d_seg_slot2_.alloc(std::max<size_t>(slot2.size(), 2));
    d_seg_val2_.alloc(std::max<size_t>(slot2.size(), 2));
    if (!info.empty())
      HIP_CHECK(hipMemcpy(d_seg_info_.get(), info.data(), sizeof(int4) * info.size(), hipMemcpyHostToDevice));
    if (!pk2.empty()) {
      HIP_CHECK(hipMemcpy(d_seg_pk2_.get(), pk2.data(), sizeof(uint32_t) * pk2.size(), hipMemcpyHostToDevice));
      HIP_CHECK(hipMemcpy(d_seg_slot2_.get(), slot2.data(), sizeof(int) * slot2.size(), hipMemcpyHostToDevice));
    }
    sp_.seg_pk2 = d_seg_pk2_.get();
    sp_.seg_val2 = d_seg_val2_.get();
    sp_.seg_rb = d_seg_rb_.get();
    sp_.seg_pk = d_seg_pk_.get();
    sp_.seg_info = d_seg_info_.get();
    sp_.nseg = (int)seg.size() - 1;
  }
}

void LatentVecchia::SetObservations(const std::vector<int>& obs_row) {
  n_obs_ = (int)obs_row.size();
  std::vector<int> ptr(n_ + 1, 0);
  for (int i = 0; i < n_obs_; ++i) {
    const int v = obs_row[i];
    if (v < 0 || v >= n_) Fatal("observation %d maps to latent row %d outside [0, %d)", i, v, n_);
    ++ptr[lab_[v] + 1];
  }
  for (int p = 0; p < n_; ++p) ptr[p + 1] += ptr[p];
  obs_order_.assign(n_obs_, 0);
  std::vector<int> fill(ptr.begin(), ptr.end() - 1);
  for (int i = 0; i < n_obs_; ++i) obs_order_[fill[lab_[obs_row[i]]]++] = i;   // ascending observation index per row
  obs_cnt_.resize(n_);
  for (int p = 0; p < n_; ++p) obs_cnt_[p] = ptr[p + 1] - ptr[p];
  d_optr_.alloc(n_ + 1);
  HIP_CHECK(hipMemcpyAsync(d_optr_.get(), ptr.data(), sizeof(int) * (n_ + 1), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  d_yo_.alloc(n_obs_);
  has_obs_ = true;
}

ObsMap LatentVecchia::Obs() const {
  ObsMap ob;
  if (has_obs_) {
    ob.ptr = d_optr_.get();
    ob.y = d_yo_.get();
    ob.offset = has_off_ ? d_offo_.get() : nullptr;
  }
  return ob;
}

void LatentVecchia::SetY(const double* y_vo) {
  if (has_obs_) {
    std::vector<double> yo(n_obs_);
    for (int e = 0; e < n_obs_; ++e) yo[e] = y_vo[obs_order_[e]];
    HIP_CHECK(hipMemcpyAsync(d_yo_.get(), yo.data(), sizeof(double) * n_obs_, hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    y_set_ = true;
    return;
  }
  std::vector<double> yp(n_);
  for (int p = 0; p < n_; ++p) yp[p] = y_vo[vo_[p]];
  sum_log_y_ = 0.;   // likelihood 'gamma': aux_log_normalizing_constant_ (likelihoods.h:8181-8191)
  for (int p = 0; p < n_; ++p) sum_log_y_ += yp[p] > 0. ? std::log(yp[p]) : 0.;
  HIP_CHECK(hipMemcpyAsync(d_y_.get(), yp.data(), sizeof(double) * n_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  y_set_ = true;
}

void LatentVecchia::SetOffset(const double* off_vo) {
  if (off_vo == nullptr) {
    has_off_ = false;
    return;
  }
  if (has_obs_) {
    std::vector<double> oo(n_obs_);
    for (int e = 0; e < n_obs_; ++e) oo[e] = off_vo[obs_order_[e]];
    d_offo_.alloc(n_obs_);
    HIP_CHECK(hipMemcpyAsync(d_offo_.get(), oo.data(), sizeof(double) * n_obs_, hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    has_off_ = true;
    return;
  }
  std::vector<double> op(n_);
  for (int p = 0; p < n_; ++p) op[p] = off_vo[vo_[p]];
  d_off_.alloc(n_);
  HIP_CHECK(hipMemcpyAsync(d_off_.get(), op.data(), sizeof(double) * n_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  has_off_ = true;
}

void LatentVecchia::GetMode(double* mode_vo) {
  if (!factor_ready_) Fatal("the posterior mode has not been computed (no evaluation yet)");
  std::vector<double> mp(n_);
  HIP_CHECK(hipMemcpyAsync(mp.data(), d_mode_.get(), sizeof(double) * n_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  for (int p = 0; p < n_; ++p) mode_vo[vo_[p]] = mp[p];
}

LatentVecchia::Block& LatentVecchia::GetBlock(int which, int t, int pmax) {
  std::unique_ptr<Block>& bp = which == 0 ? blk1_ : (which == 1 ? blkt_ : blkb_);
  if (!bp) bp.reset(new Block());
  Block& b = *bp;
  if (b.t != t) {
    if (b.t != 0) pre_->DropGraphs();   // captured preconditioner launches hold the old buffers
    const size_t nt = (size_t)n_ * t;
    for (auto* buf : {&b.R, &b.Z, &b.H, &b.V, &b.G, &b.Xt}) buf->alloc(nt);
    b.small.alloc((size_t)6 * t);
    b.act.alloc(t);
    b.ctl.alloc(kPcgCtl);
    b.t = t;
  }
  if (b.a_hist.size() < (size_t)(pmax + 2) * t) {   // + the rows of the iterations queued behind the verdict
    b.a_hist.alloc((size_t)(pmax + 2) * t);
    b.b_hist.alloc((size_t)(pmax + 2) * t);
  }
  const size_t need = (size_t)kMaxRedBlocks * std::max(kGradCols * t, (int)kLatentScalars);
  if (d_partials_.size() < need) d_partials_.alloc(need);
  if (d_out_.size() < (size_t)kGradCols * t) d_out_.alloc((size_t)kGradCols * t);
  return b;
}

void LatentVecchia::SetShard(int rank, int world, Collective* coll) {
  if (world < 1 || rank < 0 || rank >= world) Fatal("invalid rank %d / world_size %d", rank, world);
  if (world > 1 && coll == nullptr) Fatal("the probe-sharded latent path needs a collective");
  rank_ = rank;
  world_ = world;
  coll_ = coll;
  probes_saved_ = false;   // this rank's share is drawn at the next evaluation
  d_gsum_.alloc(1);
}

void LatentVecchia::AllReduceHost(double* v, int count) {
  if (coll_ == nullptr || count <= 0) return;
  if (d_red_.size() < (size_t)count) d_red_.alloc(count);
  HIP_CHECK(hipMemcpyAsync(d_red_.get(), v, sizeof(double) * count, hipMemcpyHostToDevice, s_));
  coll_->AllReduceSum(d_red_.get(), count, s_);
  HIP_CHECK(hipMemcpyAsync(v, d_red_.get(), sizeof(double) * count, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void LatentVecchia::EnsureProbes(const IterativeConfig& cfg) {
  const int t = cfg.num_rand_vec_trace;
  if (probes_saved_ && probes_t_ == t) return;
  if (t < world_) Fatal("num_rand_vec_trace = %d < %d ranks: every rank needs at least one probe column", t, world_);
  t_all_ = t;
  c0_ = (int)((long)t * rank_ / world_);
  c1_ = (int)((long)t * (rank_ + 1) / world_);
  const int tw = probe_cols();   // this rank's block width (padding columns stay 0)
  // GenRandVecNormalParallel (CG_utils.cpp:930-947), drawn once when reuse_rand_vec_trace;
  // column c is seeded by its global index, so a rank draws exactly its share
  std::vector<double> R((size_t)n_ * tw, 0.);
  {   // drawn in Vecchia order (the reference's), stored in the relabelled rows
    std::vector<double> Rv((size_t)n_ * tw, 0.);
    gen_probes_normal_cols(n_, c0_, c1_, tw, cfg.seed_rand_vec_trace, probe_run_id_, Rv.data());
    for (int p = 0; p < n_; ++p)
      std::copy(Rv.begin() + (size_t)vo_[p] * tw, Rv.begin() + (size_t)(vo_[p] + 1) * tw, R.begin() + (size_t)p * tw);
  }
  ++probe_run_id_;
  d_probes_.alloc((size_t)n_ * tw);
  d_Zp_.alloc((size_t)n_ * tw);
  d_U_.alloc((size_t)n_ * tw);
  d_P_.alloc((size_t)n_ * tw);
  HIP_CHECK(hipMemcpyAsync(d_probes_.get(), R.data(), sizeof(double) * R.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  probes_t_ = t;
  probes_saved_ = cfg.reuse_rand_vec_trace;
}

void LatentVecchia::PredVarSim(int nsim, int t, double delta, int cg_max, uint64_t seed, int n_pred, int mp,
                               const int* nbr_vo, const double* d_Bpo, double* acc, double* d_V,
                               std::mt19937* ref_gen) {
  if (!factor_ready_) Fatal("predictive variances need an evaluated latent model (mode and factor)");
  if (world_ > 1) Fatal("latent predictive variances are only available on single-rank models");
  t = std::max(1, std::min({t, nsim, 64}));
  // neighbour indices in storage labels (Z rows)
  std::vector<int> nb((size_t)n_pred * mp);
  for (size_t e = 0; e < nb.size(); ++e) nb[e] = nbr_vo[e] >= 0 && nbr_vo[e] < n_ ? lab_[nbr_vo[e]] : 0;
  DevBuf<int> d_nb(nb.size());
  DevBuf<double> d_acc(n_pred), d_sdi(n_), d_sw(n_), d_e1((size_t)n_ * t), d_e2((size_t)n_ * t), d_rhs((size_t)n_ * t),
      d_z((size_t)n_ * t);
  HIP_CHECK(hipMemcpyAsync(d_nb.get(), nb.data(), sizeof(int) * nb.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemsetAsync(d_acc.get(), 0, sizeof(double) * n_pred, s_));
  launch_sqrt_vec(n_, d_Dinv_.get(), d_sdi.get(), s_);   // D^-1/2
  launch_sqrt_vec(n_, d_W_.get(), d_sw.get(), s_);       // W^1/2 (likelihoods.h:6661: W >= 0 checked there)
  Block& b = GetBlock(2, t, cg_max);
  // ref_gen: the reference's own stream (PredictLaplaceApproxVecchia on one thread, likelihoods.h:6668-6700):
  // rng = mt19937(unif{0 .. 2147483646}(cg_generator_)), per draw a fresh normal_distribution giving
  // z1_j, z2_j interleaved over the latent variables in the model order (host, libstdc++ as the reference)
  std::mt19937 rng;
  std::vector<double> h1, h2;
  if (ref_gen) {
    std::uniform_int_distribution<> unif(0, 2147483646);
    rng.seed((std::mt19937::result_type)unif(*ref_gen));
    h1.assign((size_t)n_ * t, 0.);
    h2.assign((size_t)n_ * t, 0.);
  }
  for (int done = 0; done < nsim; done += t) {
    const int tc = std::min(t, nsim - done);   // the last block's extra columns are zero right-hand sides
    if (ref_gen) {
      std::fill(h1.begin(), h1.end(), 0.);
      std::fill(h2.begin(), h2.end(), 0.);
      for (int c = 0; c < tc; ++c) {
        std::normal_distribution<double> nd(0., 1.);
        for (int j = 0; j < n_; ++j) {
          const size_t e = (size_t)lab_[j] * t + c;
          h1[e] = nd(rng);
          h2[e] = nd(rng);
        }
      }
      HIP_CHECK(hipMemcpyAsync(d_e1.get(), h1.data(), sizeof(double) * h1.size(), hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipMemcpyAsync(d_e2.get(), h2.data(), sizeof(double) * h2.size(), hipMemcpyHostToDevice, s_));
    } else {
      launch_gen_normal(n_, t, seed, 1, done, d_e1.get(), s_);
      launch_gen_normal(n_, t, seed, 2, done, d_e2.get(), s_);
    }
    if (tc < t && !ref_gen) {   // columns >= tc: zero draws (zero right-hand side -> z = 0, no contribution)
      for (int c = tc; c < t; ++c) {
        HIP_CHECK(hipMemset2DAsync(d_e1.get() + c, sizeof(double) * t, 0, sizeof(double), n_, s_));
        HIP_CHECK(hipMemset2DAsync(d_e2.get() + c, sizeof(double) * t, 0, sizeof(double), n_, s_));
      }
    }
    // rhs = B^T D^-1/2 e1 + W^1/2 e2 (likelihoods.h:6711), storage order
    launch_bt_apply(sp_, d_Bv_.get(), true, d_e1.get(), t, d_sdi.get(), d_sw.get(), d_e2.get(), d_rhs.get(), s_);
    const PcgResult pr = Pcg(b, d_rhs.get(), d_z.get(), t, true, true, cg_max, 0, delta);
    if (pr.nan) Fatal("NaN or Inf in the conjugate gradient solves of the predictive-variance simulation");
    if (acc) launch_pred_sq_acc(n_pred, mp, t, d_nb.get(), d_Bpo, d_z.get(), d_acc.get(), s_);
    if (d_V) launch_pred_samples(n_pred, mp, t, tc, d_nb.get(), d_Bpo, d_z.get(), d_V, n_pred, done, s_);
    if (ref_gen) HIP_CHECK(hipStreamSynchronize(s_));   // h1 / h2 are refilled for the next block
  }
  if (acc) HIP_CHECK(hipMemcpyAsync(acc, d_acc.get(), sizeof(double) * n_pred, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void LatentVecchia::BenchOperators(int t, int reps, double* out) {
  if (!factor_ready_) Fatal("BenchOperators needs a previous evaluation (the factor of its parameters)");
  if (t < 1 || reps < 1) Fatal("BenchOperators: t and reps must be >= 1");
  Block& b = GetBlock(2, t, 1);
  const size_t nt = (size_t)n_ * t;
  HIP_CHECK(hipMemsetAsync(b.R.get(), 0, sizeof(double) * nt, s_));   // finite inputs (timing only)
  HIP_CHECK(hipMemsetAsync(b.H.get(), 0, sizeof(double) * nt, s_));
  ApplyA(b.H.get(), b.V.get(), b.G.get(), t);              // warm (and graph capture below)
  pre_->Apply(b.R.get(), b.Z.get(), b.Xt.get(), t);
  float ms = 0.f;
  HIP_CHECK(hipEventRecord(ev0_, s_));
  for (int r = 0; r < reps; ++r) ApplyA(b.H.get(), b.V.get(), b.G.get(), t);
  HIP_CHECK(hipEventRecord(ev1_, s_));
  HIP_CHECK(hipEventSynchronize(ev1_));
  HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
  out[0] = ms / reps;
  HIP_CHECK(hipEventRecord(ev0_, s_));
  for (int r = 0; r < reps; ++r) pre_->Apply(b.R.get(), b.Z.get(), b.Xt.get(), t);
  HIP_CHECK(hipEventRecord(ev1_, s_));
  HIP_CHECK(hipEventSynchronize(ev1_));
  HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
  out[1] = ms / reps;
  if (std::getenv("GPBOOST_AMD_PRECOND_SPLIT")) {
    pre_->TimeParts(b.R.get(), b.Z.get(), b.Xt.get(), t, reps);
    for (int part = 0; part < 2; ++part) {   // the operator's two launches
      HIP_CHECK(hipEventRecord(ev0_, s_));
      for (int r = 0; r < reps; ++r) {
        const bool tiled = t >= 2 && std::getenv("GPBOOST_AMD_SPMV_TILED") != nullptr;
        if (part == 0) {
          if (tiled) launch_b_apply_tiled(sp_, tile_b_.op, d_Bv_.get(), b.H.get(), t, d_Dinv_.get(), b.G.get(), s_);
          else launch_b_apply(sp_, d_Bv_.get(), true, b.H.get(), t, d_Dinv_.get(), b.G.get(), s_);
        } else {
          if (tiled)
            launch_bt_apply_tiled(sp_, tile_bt_.op, d_tval_.get(), b.G.get(), t, d_W_.get(), b.H.get(), b.V.get(), s_);
          else
            launch_bt_apply(sp_, d_Bv_.get(), true, b.G.get(), t, nullptr, d_W_.get(), b.H.get(), b.V.get(), s_);
        }
      }
      HIP_CHECK(hipEventRecord(ev1_, s_));
      HIP_CHECK(hipEventSynchronize(ev1_));
      HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
      std::fprintf(stderr, "[operator parts t=%d] %s %.4f ms\n", t, part ? "bt_apply" : "b_apply ", ms / reps);
    }
  }
  if (std::getenv("GPBOOST_AMD_BENCH_2STREAM") && t >= 2) {   // diagnostics: two column groups, two streams
    const int t0 = (t + 1) / 2, t1 = t - t0;
    DevBuf<double> R0((size_t)n_ * t0), Z0((size_t)n_ * t0), X0((size_t)n_ * t0);
    DevBuf<double> R1((size_t)n_ * t1), Z1((size_t)n_ * t1), X1((size_t)n_ * t1);
    for (auto* buf : {&R0, &R1}) HIP_CHECK(hipMemsetAsync(buf->get(), 0, sizeof(double) * buf->size(), s_));
    hipStream_t s2;
    HIP_CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e_fork, e_join;
    HIP_CHECK(hipEventCreateWithFlags(&e_fork, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&e_join, hipEventDisableTiming));
    pre_->Apply(R0.get(), Z0.get(), X0.get(), t0, s_, 0);
    pre_->Apply(R1.get(), Z1.get(), X1.get(), t1, s2, 1);
    HIP_CHECK(hipStreamSynchronize(s2));
    for (int mode = 0; mode < 2; ++mode) {
      HIP_CHECK(hipEventRecord(ev0_, s_));
      HIP_CHECK(hipEventRecord(e_fork, s_));
      HIP_CHECK(hipStreamWaitEvent(s2, e_fork, 0));
      for (int r = 0; r < reps; ++r) {
        pre_->Apply(R0.get(), Z0.get(), X0.get(), t0, s_, 0);
        pre_->Apply(R1.get(), Z1.get(), X1.get(), t1, mode ? s2 : s_, 1);
      }
      HIP_CHECK(hipEventRecord(e_join, s2));
      HIP_CHECK(hipStreamWaitEvent(s_, e_join, 0));
      HIP_CHECK(hipEventRecord(ev1_, s_));
      HIP_CHECK(hipEventSynchronize(ev1_));
      HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
      std::fprintf(stderr, "[precond 2-group t=%d+%d] %s: %.4f ms per pair of applications\n", t0, t1,
                   mode ? "two streams" : "one stream", ms / reps);
    }
    HIP_CHECK(hipEventDestroy(e_fork));
    HIP_CHECK(hipEventDestroy(e_join));
    HIP_CHECK(hipStreamDestroy(s2));
    pre_->DropGraphs();
  }
  out[2] = (double)tnnz_ + n_;
  out[3] = pre_->launches();
}

// V = (B^T D^-1 B + W) H   (CG_utils.cpp:75, 161-164)
void LatentVecchia::ApplyA(const double* H, double* V, double* G, int t) {
  g_timer.begin(s_);
  static const bool tiled = std::getenv("GPBOOST_AMD_SPMV_TILED") != nullptr;   // A/B: LDS-tiled operator
  if (t >= 2 && tiled && sp_.tval_of == d_Bv_.get()) {
    launch_b_apply_tiled(sp_, tile_b_.op, d_Bv_.get(), H, t, d_Dinv_.get(), G, s_);
    launch_bt_apply_tiled(sp_, tile_bt_.op, d_tval_.get(), G, t, d_W_.get(), H, V, s_);
    g_timer.end(s_, 3);
    return;
  }
  launch_b_apply(sp_, d_Bv_.get(), true, H, t, d_Dinv_.get(), G, s_);
  launch_bt_apply(sp_, d_Bv_.get(), true, G, t, nullptr, d_W_.get(), H, V, s_);
  g_timer.end(s_, t == 1 ? 2 : 3);
}

// Z = P^-1 R, P = B^T (D^-1 + W) B (VADU, CG_utils.cpp:56-60): VaduPrecond's three-part plan,
// replayed from a hipGraph per buffer set.
void LatentVecchia::Precond(const double* R, double* Z, double* Xt, int t) {
  g_timer.begin(s_);
  pre_->Apply(R, Z, Xt, t);
  g_timer.end(s_, t == 1 ? 0 : 1);
}

void LatentVecchia::SetDiag() { pre_->SetDiag(d_dw_.get()); }

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
  out[kSqLogLik] += loglik_const_;   // log_normalizing_constant_ (likelihoods.h:8638)
}

// Spin until the device's stopping check `seq` has landed in the host-coherent words (it is
// written last, after a system-scope fence). A stream that drained without it is an error.
void LatentVecchia::WaitCtl(int seq, int* out) {
  // two slots: checks j and j + 1 may both be in flight
  volatile unsigned long long* hc = reinterpret_cast<volatile unsigned long long*>(h_ctl_) + (seq & 1);
  unsigned long long v = *hc;
  for (long spins = 1; (int)(v & 0xFFFF) != (seq & 0xFFFF); ++spins) {
    if ((spins & ((1 << 16) - 1)) == 0) {
      const hipError_t e = hipStreamQuery(s_);
      if (e != hipSuccess && e != hipErrorNotReady) HIP_CHECK(e);
      v = *hc;
      if (e == hipSuccess && (int)(v & 0xFFFF) != (seq & 0xFFFF)) Fatal("PCG stopping check %d did not report", seq);
    }
    __builtin_ia32_pause();
    v = *hc;
  }
  pcg_unpack(v, out);
}

LatentVecchia::PcgResult LatentVecchia::Pcg(Block& b, const double* RHS, double* U, int n_single, bool init_zero,
                                             bool u_is_zero, int pmax_single, int pmax_block, double delta,
                                             int n_valid, int nblock_all) {
  const int t = b.t;
  if (n_valid < 0) n_valid = t;
  const bool gblock = coll_ != nullptr && nblock_all > 0;   // block rule on the all-rank norm sum
  const size_t nt = (size_t)n_ * t;
  PcgResult res;
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
  // activity mask and stopping state on the device; single columns with a zero right-hand
  // side start stopped at u = 0 (CG_utils.cpp:42-45, also inside a fused block)
  const double* rr0 = nullptr;
  if (n_single > 0 && t > 1) {
    const double* A[1] = {b.R.get()};
    const double* Bm[1] = {b.R.get()};
    launch_coldots(n_, t, 1, A, Bm, d_partials_.get(), b.rr(), s_);
    rr0 = b.rr();
  }
  launch_pcg_init(t, n_valid, n_single, pmax_single, pmax_block, kZeroRhsSq, rr0, b.act.get(), b.ctl.get(), s_);
  Precond(b.R.get(), b.Z.get(), b.Xt.get(), t);
  launch_copy(nt, b.Z.get(), b.H.get(), s_);
  {
    const double* A[1] = {b.R.get()};
    const double* Bm[1] = {b.Z.get()};
    launch_coldots(n_, t, 1, A, Bm, d_partials_.get(), b.rz(), s_);
  }
  // Iteration j is enqueued whole (operator, update, stopping check, preconditioner, beta), then
  // the host waits for the stopping check of iteration j - 1: the queue always holds a whole
  // iteration, so the GPU never waits for the host to submit the ~200 launches of a
  // preconditioner application. Once every column has stopped, the masked updates leave U and
  // the coefficient histories up to its_* unchanged, so the at most two iterations already
  // queued behind the verdict are harmless (a_hist / b_hist carry two spare rows for them).
  int ctl[kPcgCtl];
  {
    HIP_CHECK(hipMemcpyAsync(h_out_, b.ctl.get(), sizeof(int) * kPcgCtl, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    std::memcpy(ctl, h_out_, sizeof(int) * kPcgCtl);
  }
  for (int j = 0; ctl[kCtlActS] || ctl[kCtlActB]; ++j) {
    if (j >= std::max(pmax_single, pmax_block) + 2) Fatal("PCG: stopping rule did not end the iteration");
    ApplyA(b.H.get(), b.V.get(), b.G.get(), t);
    {
      const double* A[1] = {b.H.get()};
      const double* Bm[1] = {b.V.get()};
      launch_coldots(n_, t, 1, A, Bm, d_partials_.get(), b.hv(), s_);
    }
    launch_cg_alpha(t, b.rz(), b.hv(), b.act.get(), b.a(), b.a_hist.get() + (size_t)j * t, s_);
    launch_cg_update(n_, t, b.a(), b.H.get(), b.V.get(), U, b.R.get(), d_partials_.get(), b.rr(), s_);
    if (gblock) {   // every rank runs the same iterations, so the collectives pair up
      launch_pcg_block_sum(n_valid, n_single, b.rr(), d_gsum_.get(), s_);
      coll_->AllReduceSum(d_gsum_.get(), 1, s_);
    }
    const int seq = ++pcg_seq_;
    launch_pcg_check(j, t, n_single, pmax_single, pmax_block, delta, b.rr(), gblock ? d_gsum_.get() : nullptr,
                     nblock_all, b.act.get(), b.ctl.get(), d_hctl_ + (seq & 1) * 2, seq, s_);
    Precond(b.R.get(), b.Z.get(), b.Xt.get(), t);
    {
      const double* A[1] = {b.R.get()};
      const double* Bm[1] = {b.Z.get()};
      launch_coldots(n_, t, 1, A, Bm, d_partials_.get(), b.rz_new(), s_);
    }
    launch_cg_beta(t, b.rz_new(), b.rz(), b.act.get(), b.b(), b.b_hist.get() + (size_t)j * t, s_);
    launch_h_update(n_, t, b.b(), b.Z.get(), b.H.get(), s_);
    if (j == 0) continue;   // verdict of iteration j - 1 (see above)
    WaitCtl(seq - 1, ctl);
    if (ctl[kCtlNan]) break;
  }
  if (!ctl[kCtlNan]) WaitCtl(pcg_seq_, ctl);   // the last check enqueued (its counters are final)
  if (ctl[kCtlNan]) {
    HIP_CHECK(hipStreamSynchronize(s_));
    res.nan = true;
  }
  res.its_single = ctl[kCtlItsS];
  res.its_block = ctl[kCtlItsB];
  return res;
}

LatentResult LatentVecchia::Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                                 bool want_grad, bool want_aux_grad, double* grad_f_vo, ModeStart start) {
  if (use_chol_) return EvalChol(cov_type, lik, trafo, aux, cfg, want_grad, want_aux_grad, grad_f_vo, start);
  if (!y_set_) Fatal("response variable y has not been set");
  if (!(trafo[0] > 0. && trafo[1] > 0.)) Fatal("covariance parameters must be > 0");
  if (lik == kLikGaussian && !(aux > 0.)) Fatal("the error variance (aux_pars) must be > 0");
  if (lik == kLikGamma && want_grad && want_aux_grad && has_obs_)
    Fatal("estimating the shape of likelihood 'gamma' with gp_approx = 'vecchia' and repeated coordinates is not "
          "supported by gpboost_amd (set estimate_aux_pars = false)");
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
  pre_->Refresh(d_Bv_.get());   // preconditioner plan values, dense head inverse
  launch_gather(tnnz_, d_tslot_.get(), d_Bv_.get(), d_tval_.get(), s_);   // B^T operator values, list order
  if (seg2_n_ > 0) launch_gather(seg2_n_, d_seg_slot2_.get(), d_Bv_.get(), d_seg_val2_.get(), s_);   // paired runs
  sp_.tval_of = d_Bv_.get();
  launch_gather(n * m_, d_ell_slot_.get(), d_Bv_.get(), d_ell_val_.get(), s_);   // t = 1 form of B
  sp_.vals_of = d_Bv_.get();
  factor_ready_ = true;

  Block& b1 = GetBlock(0, 1, std::max(cfg.cg_max_num_it, 1));
  if (std::getenv("GPBOOST_AMD_BENCH_PRECOND")) {   // diagnostics: preconditioner cost alone
    NewtonPrepArgs np{};
    np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
    np.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
    np.obs = Obs();
    np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get(); np.W_update = 1; np.dw = d_dw_.get();
    HIP_CHECK(hipMemsetAsync(d_mode_.get(), 0, sizeof(double) * n, s_));
    launch_newton_prep(np, s_);
    SetDiag();
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
      std::fprintf(stderr, "[precond bench] t=%d: %.3f ms per application (%d launches)\n", tt, pm / 20,
                   pre_->launches());
    }
  }
  ScalarArgs sa{};
  sa.n = n; sa.m = m_; sa.lik = lik; sa.aux = aux;
  sa.nbr = d_nbr_.get(); sa.Bv = d_Bv_.get(); sa.Dinv = d_Dinv_.get(); sa.y = d_y_.get();
  sa.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
  sa.obs = Obs();

  // ---- 2. mode finding (likelihoods.h:2780-3000): from 0 (InitializeModeAvec) or from the previous
  // evaluation's mode (mode_previous_value_ kept for a reset)
  if (start == ModeStart::kZero) {
    HIP_CHECK(hipMemsetAsync(d_mode_.get(), 0, sizeof(double) * n, s_));
  } else if (start == ModeStart::kWarm) {
    d_mode_prev_.alloc(n);
    launch_copy(n, d_mode_.get(), d_mode_prev_.get(), s_);
    mode_prev_valid_ = true;
  }
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
      if (lik == kLikPoisson || lik == kLikGamma) launch_cap_mode_change(n, d_mode_.get(), d_mode_new_.get(), s_);
      sa.mode = d_mode_new_.get();
      Scalars(sa, sc);
      mll_new = sc[kSqLogLik] - 0.5 * sc[kSqQuad];
      if (mll_new < mll + kCArmijo * lr * gdd || std::isnan(mll_new) || std::isinf(mll_new)) lr *= 0.5;
      else break;
    }
    std::swap(d_mode_, d_mode_new_);
    res.newton_its = it + 1;
    if (std::isnan(mll_new) || std::isinf(mll_new))
      throw LatentNan("NaN or Inf occurred in the mode finding algorithm for the Laplace approximation");
    const double dc = cfg.delta_conv_mode_finding;
    const bool term = (it == 0) ? std::fabs(mll_new - mll) < dc * std::fabs(mll) : (mll_new - mll) < dc * std::fabs(mll);
    mll = mll_new;
    return term;
  };
  EnsureProbes(cfg);
  const int tw = probe_cols();          // this rank's probe block width (t at world 1)
  const int tl = c1_ - c0_;             // its real probe columns (the rest is padding)
  const int nb_all = coll_ ? t : 0;     // block column count over all ranks (collective stop rule)
  if (gauss) {
    // Gaussian: W = 1/aux does not depend on the mode, so the single Newton step's solve
    // (Sigma^-1 + W)^-1 (y / aux) and the SLQ block solve the same system. Both run as one
    // PCG over 1 + t columns: column 0 keeps the single-vector stopping rule, columns 1..t
    // the block rule (each column's iterates are exactly those of a separate run).
    NewtonPrepArgs np{};
    np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
    np.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
    np.obs = Obs();
    np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get(); np.W_update = 1;
    np.rhs = d_rhs_.get(); np.dw = d_dw_.get(); np.sdw = d_sdw_.get();
    launch_newton_prep(np, s_);
    SetDiag();
    n_lead = 1;
    const int tf = tw + 1;
    bslq = &GetBlock(1, tf, std::max(pmax_tri, cg_max));
    d_rhsf_.alloc((size_t)n * tf);
    d_Uf_.alloc((size_t)n * tf);
    // z_i = B^T (D^-1 + W)^(1/2) r_i into columns 1..tw, y / aux into column 0
    launch_bt_apply(sp_, d_Bv_.get(), true, d_probes_.get(), tw, d_sdw_.get(), nullptr, nullptr, d_Zp_.get(), s_);
    launch_pack_columns(n, tw, d_Zp_.get(), tw, 0, d_rhsf_.get(), tf, 1, s_);
    launch_pack_columns(n, 1, d_rhs_.get(), 1, 0, d_rhsf_.get(), tf, 0, s_);
    slq = Pcg(*bslq, d_rhsf_.get(), d_Uf_.get(), 1, true, true, cg_max, pmax_tri, cfg.cg_delta_conv, 1 + tl, nb_all);
    if (slq.nan) throw LatentNan("NaN or Inf occurred in the conjugate gradient algorithm (mode finding / log-determinant)");
    res.cg_its = slq.its_single;
    launch_pack_columns(n, 1, d_Uf_.get(), tf, 0, d_mode_upd_.get(), 1, 0, s_);
    launch_pack_columns(n, tw, d_Uf_.get(), tf, 1, d_U_.get(), tw, 0, s_);
    line_search_and_check(0, 0.);
    {   // first derivative at the mode (likelihoods.h:3008; used by the gradient wrt F)
      NewtonPrepArgs nd{};
      nd.n = n; nd.lik = lik; nd.aux = aux; nd.y = d_y_.get(); nd.loc = d_mode_.get(); nd.mode = d_mode_.get();
      nd.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
      nd.obs = Obs();
      nd.Dinv = d_Dinv_.get(); nd.d1 = d_d1_.get(); nd.W = d_W_.get(); nd.W_update = 0;
      launch_newton_prep(nd, s_);
    }
  } else {
    // ---- 2. mode finding (likelihoods.h:2780-3000)
    bool upd_zero = true;
    const int newton_its = start == ModeStart::kKeep ? 0 : maxit;   // kKeep: the mode as it stands
    for (int it = 0; it < newton_its; ++it) {
      NewtonPrepArgs np{};
      np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
    np.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
    np.obs = Obs();
      np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get();
      np.W_update = 1;
      np.rhs = d_rhs_.get();
      np.dw = d_dw_.get();
      launch_newton_prep(np, s_);
      SetDiag();
      const PcgResult pr = Pcg(b1, d_rhs_.get(), d_mode_upd_.get(), 1, it == 0, upd_zero, cg_max, 0, cfg.cg_delta_conv);
      res.cg_its += pr.its_single;
      upd_zero = pr.zero_rhs;
      if (pr.nan) throw LatentNan("NaN or Inf occurred in the conjugate gradient algorithm during mode finding");
      // Armijo (likelihoods.h:2957-2966)
      launch_axpby(n, 1., d_mode_upd_.get(), -1., d_mode_.get(), d_dir_.get(), s_);
      ApplyA(d_dir_.get(), d_Adir_.get(), b1.G.get(), 1);
      const double gdd = Dot1(d_dir_.get(), d_Adir_.get());
      if (line_search_and_check(it, gdd)) break;
    }
    {   // derivative / information at the mode, VADU diagonal and its square root (:3000-3005, 12163-12166)
      NewtonPrepArgs np{};
      np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
    np.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
    np.obs = Obs();
      np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get();
      np.W_update = info_changes ? 1 : 0;
      np.dw = d_dw_.get();
      np.sdw = d_sdw_.get();
      launch_newton_prep(np, s_);
      SetDiag();
    }
    // ---- 3. SLQ block (likelihoods.h:3018-3045, 12155-12212): z_i = B^T (D^-1 + W)^(1/2) r_i
    bslq = &GetBlock(1, tw, pmax_tri);
    launch_bt_apply(sp_, d_Bv_.get(), true, d_probes_.get(), tw, d_sdw_.get(), nullptr, nullptr, d_Zp_.get(), s_);
    slq = Pcg(*bslq, d_Zp_.get(), d_U_.get(), 0, true, true, 0, pmax_tri, cfg.cg_delta_conv, tl, nb_all);
    if (slq.nan) throw LatentNan("NaN or Inf occurred in the stochastic Lanczos quadrature (log-determinant)");
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
  std::vector<std::vector<double>> Td(tl), Ts(tl);
  for (int c = 0; c < tl; ++c) {   // CG_utils.cpp:200-206 (a_old = 1, b_old = 0 before the first step)
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
  double ldet_PI;
  if (coll_ == nullptr) {
    ldet_PI = slq_logdet(Td, Ts, n);
  } else {   // every rank's per-probe terms at their global columns, summed in column order
    const std::vector<double> mine = slq_terms(Td, Ts);
    std::vector<double> all(t, 0.);
    std::copy(mine.begin(), mine.end(), all.begin() + c0_);
    AllReduceHost(all.data(), t);
    double ld = 0.;
    for (int c = 0; c < t; ++c) ld += all[c];
    ldet_PI = ld * n / t;
  }
  res.logdet = ldet_PI - sc[kSqLogDinv] + sc[kSqLogDw];
  const double mll_final = mll - 0.5 * res.logdet;
  res.nll = -mll_final;

  if (want_grad) {
    // ---- 4. gradient (likelihoods.h:4951-5206)
    Precond(d_Zp_.get(), d_P_.get(), bt.Xt.get(), tw);   // PI_Z = P^-1 Z (:12321-12327)
    if (!gauss) {   // grad_information_wrt_mode_non_zero_: implicit derivative through the mode
      ModeDerivArgs md{};
      md.n = n; md.m = m_; md.t = tw; md.lik = lik; md.aux = aux; md.nbr = d_nbr_.get(); md.Bv = d_Bv_.get(); md.dw = d_dw_.get();
      md.loc = d_mode_.get(); md.U = d_U_.get(); md.P = d_P_.get(); md.dmll = d_dmll_.get();
      md.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
      md.y = has_obs_ ? nullptr : d_y_.get();
      md.obs = Obs();
      md.t_valid = tl; md.t_all = t;
      if (coll_ == nullptr) {
        md.stage = 0;
        launch_mode_deriv(md, s_);
      } else {   // row moments over all ranks' probes: two all-reduces of n x 2
        d_mom_.alloc((size_t)2 * n);
        d_mom2_.alloc((size_t)2 * n);
        md.mom = d_mom_.get();
        md.mom2 = d_mom2_.get();
        for (int st = 1; st <= 3; ++st) {
          md.stage = st;
          launch_mode_deriv(md, s_);
          if (st < 3) coll_->AllReduceSum(st == 1 ? d_mom_.get() : d_mom2_.get(), 2 * n, s_);
        }
      }
      const PcgResult pv = Pcg(b1, d_dmll_.get(), d_vS_.get(), 1, true, true, cg_max, 0, cfg.cg_delta_conv);
      res.cg_its += pv.its_single;
      if (pv.nan) Warning("NaN or Inf occurred in the conjugate gradient algorithm of the gradient calculation");
    }
    GradColsArgs ga{};
    ga.n = n; ga.m = m_; ga.t = tw; ga.nbr = d_nbr_.get(); ga.Bv = d_Bv_.get(); ga.dBv = d_dBv_.get();
    ga.Dinv = d_Dinv_.get(); ga.dD = d_dD_.get(); ga.W = d_W_.get();
    ga.daux = gauss ? -1. / aux : 0.;   // d information / dlog(aux) (likelihoods.h:10967-10976)
    ga.obs_ptr = has_obs_ ? d_optr_.get() : nullptr;   // per observation: x the row's count
    ga.U = d_U_.get(); ga.P = d_P_.get();
    DevBuf<double>& cols = d_out_;
    launch_grad_cols(ga, d_partials_.get(), cols.get(), s_);
    std::vector<double> z((size_t)kGradCols * t, 0.);
    {   // per-column sums [q][c]; probe-sharded: this rank's columns at their global index, summed over ranks
      std::vector<double> zl((size_t)kGradCols * tw);
      HIP_CHECK(hipMemcpyAsync(zl.data(), cols.get(), sizeof(double) * zl.size(), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      for (int q = 0; q < kGradCols; ++q)
        for (int c = 0; c < tl; ++c) z[(size_t)q * t + c0_ + c] = zl[(size_t)q * tw + c];
      AllReduceHost(z.data(), (int)z.size());
    }
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
    if (grad_f_vo != nullptr && has_obs_)
      Fatal("the gradient wrt the fixed effects of a latent model with repeated coordinates is not supported by "
            "gpboost_amd");
    if (grad_f_vo != nullptr) {   // wrt the fixed effects F (likelihoods.h:5337-5367)
      d_gradf_.alloc(n);
      launch_grad_f(n, d_d1_.get(), gauss ? nullptr : d_dmll_.get(), d_W_.get(), gauss ? nullptr : d_vS_.get(),
                    d_gradf_.get(), s_);
      std::vector<double> gp(n);
      HIP_CHECK(hipMemcpyAsync(gp.data(), d_gradf_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      for (int p = 0; p < n; ++p) grad_f_vo[vo_[p]] = gp[p];
    }
    // gamma shape on the log scale (:5139-5202, 10508-10524, 10856-10869)
    if (lik == kLikGamma && want_aux_grad) {
      DevBuf<double> rec((size_t)3 * n), red(3);
      launch_gamma_aux_rec(n, aux, d_y_.get(), has_off_ ? d_off_.get() : nullptr, d_mode_.get(), d_W_.get(),
                           d_dmll_.get(), d_d1_.get(), d_vS_.get(), rec.get(), s_);
      launch_sum_blocks(rec.get(), n, 3, red.get(), s_);
      double h[3];
      HIP_CHECK(hipMemcpyAsync(h, red.get(), sizeof(h), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double neg = aux * (h[0] - n * (std::log(aux) + 1. - digamma_asa103(aux)) - sum_log_y_);
      res.grad.push_back(neg + 0.5 * h[1] + h[2]);
    }
    // gaussian error variance on the log scale (:5166-5200, 10586-10597, 12520-12546)
    if (gauss && want_aux_grad) {
      const double* z1 = z.data() + 4 * t;
      const double* zP = z.data() + 5 * t;
      const double tr1 = mean(z1), trP = mean(zP);
      const double trD = sc[kSqTrDw] * (-1. / aux);
      const double c = optimal_c(z1, zP, t, tr1, trP);
      const double dd = tr1 + c * trD - c * trP;
      res.grad.push_back(sc[kSqRss] * (-0.5 / aux) + 0.5 * (has_obs_ ? n_obs_ : n) + 0.5 * dd);
    }
  }
  HIP_CHECK(hipEventRecord(ev1_, s_));
  HIP_CHECK(hipEventSynchronize(ev1_));
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
