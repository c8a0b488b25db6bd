// Dense path kernels (placeholder until the blocked MFMA Cholesky lands).
#include "dense.h"
#include "kernels.h"

namespace gpb_amd {

DenseSolver::DenseSolver(int n, int d, const double* d_X, hipStream_t stream)
    : n_(n), d_(d), ld_(n), d_X_(d_X), stream_(stream) {}
DenseSolver::~DenseSolver() {}
void DenseSolver::Eval(int, double, double, const double*, bool, double*, double*) {
  Fatal("dense GPU path not available in this build yet");
}

}  // namespace gpb_amd
