// Dense Gaussian-process likelihood on the GPU (gp_approx = "none"):
// Psi = Sigma/sigma2 + I built in HBM, blocked fp64 Cholesky with MFMA trailing updates,
// Psi^-1 for the gradient traces. Reference: re_model_template.h:5902-5904 (CalcChol),
// :5987-6007 (CalcPsiInv), :1798-1818 (dense gradient), :2875-2880 (nll).
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"

namespace gpb_amd {

class DenseSolver {
 public:
  DenseSolver(int n, int d, const double* d_X, hipStream_t stream);
  ~DenseSolver();
  // sums = [logdet, q, s1_var, s1_range, s2_var, s2_range] (same contract as the Vecchia rows):
  // s1_k = -1/2 y_aux^T dPsi_k y_aux, s2_k = tr(dPsi_k Psi^-1).
  // kernel_ms[0] = Cholesky time, kernel_ms[1] = whole device evaluation.
  void Eval(int cov_type, double var, double phi, const double* d_y, bool want_grad, double* sums, double* kernel_ms);

 private:
  void Potrf();
  void Trtri(int a, int b);

  int n_, d_, ld_;
  const double* d_X_;
  hipStream_t stream_;
  DevBuf<double> A_, W_, T_, vec_, red_;
  DevBuf<int> info_;
  double* h_red_ = nullptr;
  hipEvent_t ev_[3] = {nullptr, nullptr, nullptr};
};

// host helper shared by all paths (re_model.cpp)
void combine_partials(const double* s, int n, double sigma2_in, int profile, double* nll, double* grad,
                      double* sigma2_out);

}  // namespace gpb_amd
