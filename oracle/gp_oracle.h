/* ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
 *
 * CPU restatement of the reference GPBoost GP-likelihood hot path, used ONLY as
 * the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * The product (libgpboost_amd.so) never links, loads or calls this code.
 *
 * Parity pinning: tests/test_oracle_golden.py checks every function here against
 * (a) the golden values hard-coded in the reference's own R tests and
 * (b) fixtures produced by the reference itself (oracle/_ref/ref_harness, built
 *     from /root/reference by oracle/Makefile; tests/golden/make_golden.py).
 *
 * Conventions: fp64 throughout, int32 indices. "Vecchia order" = data after the
 * random permutation of CreateREComponentsVecchia (Vecchia_utils.cpp:1094-1103).
 * Covariance parameters are on the reference's "transformed scale"
 * (cov_fcts.h:438-493): pars = (sigma2, sigma1^2/sigma2, phi).
 */
#ifndef GP_ORACLE_H_
#define GP_ORACLE_H_

#ifdef __cplusplus
extern "C" {
#endif

/* covariance kernel codes (shared numbering with include/gpboost_amd.h) */
enum { ORC_MATERN05 = 0, ORC_MATERN15 = 1, ORC_MATERN25 = 2, ORC_GAUSSIAN = 3 };

/* cov_fcts.h:438-493 TransformCovPars: orig (sigma2, sigma1^2, rho) -> trafo */
void orc_transform_cov_pars(int cov_type, const double* orig, double* trafo);

/* Vecchia_utils.cpp:1094-1095: identity, then std::shuffle with std::mt19937(seed)
 * when ordering == "random". perm[i] = original index of the i-th point. */
void orc_vecchia_order(int n, int seed, int random_ordering, int* perm);

/* Vecchia_utils.cpp:732-1058 find_nearest_neighbors_Vecchia_fast ("nearest"):
 * coords_vo row-major n x d in Vecchia order. nbr: n x m, row i holds
 * k_i = min(i, m) indices (ascending distance), rest -1. */
void orc_find_neighbors(const double* coords_vo, int n, int d, int m, int* nbr);
// Prediction ("order_obs_first_cond_obs_only"): neighbours of rows [n_obs, n_all) among the
// observed rows, and the predictive mean / variance (gp_oracle.cpp cites the reference lines).
void orc_find_neighbors_pred(const double* x_all, int n_obs, int n_all, int d, int m, int* nbr);
int orc_vecchia_predict(const double* x_all, const double* y_obs, const int* nbr, int n_obs, int n_pred, int d,
                        int m, int t, const double* pars, int predict_response, double* mean, double* var);

/* Exact Gaussian Vecchia nll + gradient (Vecchia_utils.cpp:1307-1632,
 * re_model_template.h:1748-1791, 2646-2881, 8885-9120).
 * mode 0: gradient wrt log of all trafo pars incl. nugget (include_error_var=true),
 *         nll at pars[0].
 * mode 1: the L-BFGS objective unit (optim_utils.h:243-364): sigma2 profiled out
 *         (= yT Psi^-1 y / n), gradient wrt log(pars[1:]) only.
 * Outputs: nll, grad (length 3 in mode 0, 2 in mode 1), sigma2_out; optional
 * Dinv (n) and Bvals (n x m, B(i, nbr) = -A_i, 0-padded) if non-NULL. */
int orc_vecchia_nll_grad(const double* coords_vo, const double* y_vo, const int* nbr,
                         int n, int d, int m, int cov_type, const double* pars, int mode,
                         double* nll, double* grad, double* sigma2_out,
                         double* Dinv, double* Bvals);

/* Per-row-range partial sums of the same quantity (for the multi-rank sharding
 * test): rows [r0, r1). sums = [logdet, q, s1_1..s1_P, s2_1..s2_P, qnug] with
 * P = 2 (var, range); see DESIGN.md "reduction contract". */
int orc_vecchia_partials(const double* coords_vo, const double* y_vo, const int* nbr,
                         int n, int d, int m, int cov_type, const double* pars,
                         int r0, int r1, double* sums);

/* Dense Gaussian GP nll + gradient (re_model_template.h:5902, 5987-6007, 1798-1818,
 * 2875-2880). coords row-major n x d (original order). Same mode semantics. */
int orc_dense_nll_grad(const double* coords, const double* y, int n, int d,
                       int cov_type, const double* pars, int mode,
                       double* nll, double* grad, double* sigma2_out);

/* ---- latent Vecchia + iterative methods (gp_oracle_iter.cpp) ---- */
enum { ORC_LIK_GAUSSIAN = 0, ORC_LIK_BERNOULLI_LOGIT = 1 };

/* Latent Vecchia factor (Vecchia_utils.cpp:1307-1632, gauss_likelihood = false):
 * trafo = (sigma1^2, phi). Bv/dBv: n x m row-major, B(i, nbr[i][r]) and its derivative wrt
 * log(phi) (0-padded); Dinv, dD (= dD/dlog phi): n. Returns 0 or -1 (not SPD). */
int orc_latent_vecchia_factor(const double* coords_vo, const int* nbr, int n, int d, int m, int cov_type,
                              const double* trafo, double* Bv, double* dBv, double* Dinv, double* dD);

/* GenRandVecNormalParallel (CG_utils.cpp:930-947): R column-major n x t. */
void orc_gen_probes(int n, int t, int seed, unsigned long long run_id, double* R);

/* Laplace-approximated nll and gradient for the latent Vecchia model with iterative
 * methods and the VADU preconditioner (likelihoods.h:2765-3076, 4951-5206, 12069-12546;
 * CG_utils.cpp:21-217, 930-1041). Mode starts at 0; probes use run_id 0 (first draw,
 * reuse_rand_vec_trace). trafo = (sigma1^2, phi); aux = gaussian error variance.
 * grad = [d/dlog sigma1^2, d/dlog phi, (gaussian) d/dlog aux]. info (optional, 4):
 * newton iterations, total mode-finding CG iterations, Lanczos steps, log|Sigma W + I|. */
int orc_latent_vecchia_iterative(const double* coords_vo, const double* y_vo, const int* nbr, int n, int d, int m,
                                 int cov_type, const double* trafo, int likelihood, double aux, int t, int seed,
                                 double cg_delta_conv, int cg_max_num_it, int cg_max_num_it_tridiag, int want_grad,
                                 double* nll, double* grad, double* info);

#ifdef __cplusplus
}
#endif
#endif
