// Fisher information of the covariance parameters of the Gaussian Vecchia model, for their standard
// deviations (GPB_GetCovPar(calc_std_dev = true)).
//
// Reference path replaced:
//   CalcStdDevCovPar              re_model_template.h:9775-9789 (original-scale factor and derivatives:
//                                 CalcCovFactor(false, sigma^2), CalcGradientVecchia(false, sigma^2, true))
//   CalcFisherInformation_Vecchia re_model_template.h:9238-9307, the default stochastic-trace form
//                                 (use_stochastic_trace_for_Fisher_information_Vecchia_ = true, :5533): probes z
//                                 (n x t, GenRandVecNormalParallel(seed_rand_vec_trace, cg_generator_counter_)),
//                                 g_0 = Sigma^-1 z = B^T D^-1 B z,
//                                 g_k = B^T D^-1 (-dB_k Sigma z + dD_k B^-T z) - dB_k^T B^-T z   (k = sigma1^2, rho),
//                                 FI_kl = 1/2 mean over the columns of g_k . g_l
// The reference forms these with Eigen sparse triangular solves (TriangularSolve, one row at a time).
//
// This build: the factor and its two derivatives from one row kernel on the transformed scale (the
// latent factor kernel in its nugget form, latent_factor.hip), rescaled to the original scale on the
// device (B is scale-free; D_o = sigma^2 D, dB_o / dsigma1^2 = dB / dlog(var) / sigma1^2, dD_o / dsigma1^2 =
// dD / dlog(var) sigma^2 / sigma1^2, d / drho = dlog(phi) / drho d / dlog(phi), dD also times sigma^2);
// Sigma z from ONE application of the VADU plan (vadu_precond.h: B^-1 diag(1/dw) B^-T with dw = D^-1 —
// dense head, LDS segment and level-scheduled tail solves over all t columns at once) and B^-T z = D^-1 B
// (Sigma z) from it by one sparse product, the
// sparse products over probe-interleaved n x t blocks (sparse_kernels.hip), the column dot products by the
// deterministic two-pass reduction. The 3 x 3 inverse is on the host (re_model: StdDevCovPars).
//
// HBM layout (Vecchia order, identity storage labels): B values and derivatives n x m beside the neighbour
// table, t-column blocks row-major n x t (X[i t + c]).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "common.h"
#include "vadu_precond.h"

namespace gpb_amd {

class VecchiaFisher {
 public:
  // d_X: device n x d coordinates (Vecchia order); d_nbr / nbr: the same n x m neighbour table on the
  // device and the host (row i holds min(i, m) entries).
  VecchiaFisher(int n, int d, int m, const double* d_X, const int* d_nbr, const std::vector<int>& nbr,
                hipStream_t stream);
  ~VecchiaFisher();
  // FI (3 x 3, row-major, [sigma^2, sigma1^2, rho]) at the original-scale parameters orig; trafo: the same
  // on the transformed scale (TransformCovPars); t probes from (seed, run_id).
  void Fisher(int cov_type, const double* orig, const double* trafo, int t, int seed, uint64_t run_id, double* FI);

 private:
  int n_, d_, m_;
  hipStream_t s_;
  const double* d_X_;
  const int* d_nbr_;
  std::unique_ptr<VaduPrecond> pre_;
  DevBuf<int> tptr_, trow_, tslot_;
  DevBuf<double> Bv_, dBv0_, dBv1_;    // n x m: B, dB / dsigma1^2, dB / drho
  DevBuf<double> Dinv_, dD0_, dD1_, Do_, mones_;   // mones_: n times -1
  DevBuf<double> Z_, P_, W_, T_, U_, G_[3];   // n x t
  DevBuf<double> part_, red_;
  int t_ = 0;
};

}  // namespace gpb_amd
