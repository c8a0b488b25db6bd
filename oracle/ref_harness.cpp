// ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
//
// Probe harness for the *reference* GPBoost implementation. It is compiled
// (by oracle/Makefile) directly against the reference sources where they lie
// under /root/reference — nothing is copied into this repository — and its
// binary goes to oracle/_ref/ (git-ignored). It is used only by
// tests/golden/make_golden.py (to produce the committed golden fixtures) and by
// bench.py's cpu_baseline leg (kind "reference").
//
// The public C API of the reference has no gradient entry point
// (include/LightGBM/c_api.h:1500 returns only the nll), so this harness calls
// REModelTemplate exactly as the L-BFGS objective does
// (include/GPBoost/optim_utils.h:243-364):
//   TransformCovPars (re_model_template.h:7189)
//   CalcCovFactorOrModeAndNegLL (re_model_template.h:2582)
//   ProfileOutSigma2 (:2407) + EvalNegLogLikelihoodOnlyUpdateNuggetVariance (:2888)
//   CalcGradPars (:1748)
//
// Input file (little-endian): int32 n, int32 d, double coords[n*d] (column-major),
// double y[n]. Options on argv (key=value). Output: one JSON object on stdout.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <map>
#include <chrono>
#include <algorithm>
#include <memory>
#include <mutex>
#include <thread>
#include <fstream>

// Pull in every system / third-party header first with normal access control,
// then open up only the GPBoost class internals (members such as
// nearest_neighbors_ are needed for the golden index fixtures).
#include <sstream>
#include <iostream>
#include <iomanip>
#include <complex>
#include <random>
#include <set>
#include <unordered_map>
#include <unordered_set>
#include <functional>
#include <numeric>
#include <limits>
#include <cmath>
#include <Eigen/Dense>
#include <Eigen/Sparse>
#include <Eigen/IterativeLinearSolvers>
#include <LightGBM/utils/log.h>
#include <LightGBM/utils/common.h>
#include <LightGBM/meta.h>
#include <LBFGSpp/BFGSMat.h>
#define private public
#define protected public
#include <GPBoost/re_model_template.h>
#undef private
#undef protected

using namespace GPBoost;

static std::map<std::string, std::string> parse_args(int argc, char** argv) {
  std::map<std::string, std::string> a;
  for (int i = 2; i < argc; ++i) {
    std::string s(argv[i]);
    auto p = s.find('=');
    if (p == std::string::npos) continue;
    a[s.substr(0, p)] = s.substr(p + 1);
  }
  return a;
}

static std::string get(const std::map<std::string, std::string>& a, const char* k, const char* def) {
  auto it = a.find(k);
  return it == a.end() ? std::string(def) : it->second;
}

static std::vector<double> parse_list(const std::string& s) {
  std::vector<double> v;
  size_t st = 0;
  while (st < s.size()) {
    size_t e = s.find(',', st);
    if (e == std::string::npos) e = s.size();
    v.push_back(std::atof(s.substr(st, e - st).c_str()));
    st = e + 1;
  }
  return v;
}

static void print_vec(const char* name, const double* v, int n, bool comma = true) {
  std::printf("\"%s\": [", name);
  for (int i = 0; i < n; ++i) std::printf("%s%.17g", i ? ", " : "", v[i]);
  std::printf("]%s\n", comma ? "," : "");
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: ref_harness input.bin key=value ...\n");
    return 2;
  }
  auto args = parse_args(argc, argv);
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) { std::perror("open"); return 2; }
  int32_t n = 0, d = 0;
  if (std::fread(&n, 4, 1, f) != 1 || std::fread(&d, 4, 1, f) != 1) return 2;
  std::vector<double> coords((size_t)n * d), y(n);
  if (std::fread(coords.data(), 8, coords.size(), f) != coords.size()) return 2;
  if (std::fread(y.data(), 8, y.size(), f) != y.size()) return 2;
  // optional linear regression covariates: int32 p, double X[n*p] (column-major)
  int32_t p_cov = 0;
  std::vector<double> Xcov;
  if (std::fread(&p_cov, 4, 1, f) == 1 && p_cov > 0) {
    Xcov.resize((size_t)n * p_cov);
    if (std::fread(Xcov.data(), 8, Xcov.size(), f) != Xcov.size()) return 2;
  }
  // optional fixed effects F (offset of the location parameter): int32 1, double F[n]
  int32_t has_fe = 0;
  std::vector<double> fe;
  if (std::fread(&has_fe, 4, 1, f) == 1 && has_fe == 1) {
    fe.resize(n);
    if (std::fread(fe.data(), 8, fe.size(), f) != fe.size()) return 2;
  }
  const double* fe_ptr = fe.empty() ? nullptr : fe.data();
  // optional grouped random effects: int32 K, int32 labels[n * K] (effect-major); the reference
  // takes NUL-terminated label strings, effect-major (c_api.h:1324-1327)
  int32_t num_re_group = 0;
  std::string re_group_data;
  if (std::fread(&num_re_group, 4, 1, f) == 1 && num_re_group > 0) {
    std::vector<int32_t> lab((size_t)n * num_re_group);
    if (std::fread(lab.data(), 4, lab.size(), f) != lab.size()) return 2;
    for (int32_t v : lab) {
      re_group_data += std::to_string(v);
      re_group_data.push_back('\0');
    }
  } else {
    num_re_group = 0;
  }
  std::fclose(f);

  const std::string cov_fct = get(args, "cov_fct", "exponential");
  const double shape = std::atof(get(args, "shape", "0.5").c_str());
  const std::string gp_approx = get(args, "gp_approx", "none");
  const int num_neighbors = std::atoi(get(args, "num_neighbors", "30").c_str());
  const std::string ordering = get(args, "ordering", "random");
  const std::string likelihood = get(args, "likelihood", "gaussian");
  const std::string mim = get(args, "matrix_inversion_method", "cholesky");
  const int seed = std::atoi(get(args, "seed", "0").c_str());
  const int threads = std::atoi(get(args, "threads", "-1").c_str());
  const std::vector<double> cov_pars_orig = parse_list(get(args, "cov_pars", "0.1,1.6,0.2"));
  const std::string mode = get(args, "mode", "eval");   // eval | lbfgs | fit | stddev
  const int reps = std::atoi(get(args, "reps", "1").c_str());
  const int dump_nn = std::atoi(get(args, "dump_nn", "0").c_str());
  const std::string aux = get(args, "aux_pars", "");
  // FITC (gp_approx = "fitc"): inducing points (re_model_template.h:6931-7073)
  const int num_ind_points = std::atoi(get(args, "num_ind_points", "0").c_str());
  const double cover_tree_radius = std::atof(get(args, "cover_tree_radius", "1").c_str());
  const std::string ind_points_selection = get(args, "ind_points_selection", "kmeans++");

  Log::ResetLogLevelRE(LogLevelRE::Warning);
  auto t0 = std::chrono::steady_clock::now();
  // GPB_HARNESS_GROUPED: the sparse instantiation the REModel facade picks for models without GPs
  // (re_model.cpp:65-76); grouped random effects only (num_gp = 0)
#ifdef GPB_HARNESS_GROUPED
  typedef REModelTemplate<sp_mat_rm_t, chol_sp_mat_rm_t> Model;
  if (num_re_group <= 0) { std::fprintf(stderr, "grouped harness needs group data\n"); return 2; }
  std::unique_ptr<Model> m(new Model(
      n, nullptr, re_group_data.data(), num_re_group, nullptr, nullptr, 0, nullptr,
      0, nullptr, 0, nullptr, 0, cov_fct.c_str(), shape, gp_approx.c_str(),
      -1., 0., num_neighbors, ordering.c_str(), 0, 1., "kmeans++",
      likelihood.c_str(), 0., mim.c_str(), seed, threads, false, false, nullptr, 1.));
#else
  typedef REModelTemplate<den_mat_t, chol_den_mat_t> Model;
  // grouped random effects beside the GP (combined model, gp_approx = "none"): the same label input
  std::unique_ptr<Model> m(new Model(
      n, nullptr, num_re_group > 0 ? re_group_data.data() : nullptr, num_re_group, nullptr, nullptr, 0, nullptr,
      1, coords.data(), d, nullptr, 0, cov_fct.c_str(), shape, gp_approx.c_str(),
      -1., 0., num_neighbors, ordering.c_str(), num_ind_points, cover_tree_radius, ind_points_selection.c_str(),
      likelihood.c_str(), 0., mim.c_str(), seed, threads, false, false, nullptr, 1.));
#endif
  auto t1 = std::chrono::steady_clock::now();
  double t_construct = std::chrono::duration<double>(t1 - t0).count();

  if (args.count("cg_delta_conv") || args.count("num_rand_vec_trace")) {
    // same defaults as re_model_template.h:5364-5380 unless overridden
    const double cg_delta_conv = std::atof(get(args, "cg_delta_conv", "1e-2").c_str());
    const int t = std::atoi(get(args, "num_rand_vec_trace", "50").c_str());
    const int cg_max = std::atoi(get(args, "cg_max_num_it", "1000").c_str());
#ifdef GPB_HARNESS_GROUPED
    const std::string prec = get(args, "cg_preconditioner_type", "ssor");
#else
    const std::string prec = get(args, "cg_preconditioner_type", "vadu");
#endif
    const int no_index[1] = {-1};   // SetOptimConfig reads estimate_cov_par_index[0] (re_model_template.h:810)
    m->SetOptimConfig(0.1, 0.5, 1000, 1e-6, true, 0, "lbfgs", 2, "relative_change_in_log_likelihood",
                      0.1, 0.5, "lbfgs", cg_max, cg_max, cg_delta_conv, t, true, prec.c_str(),
                      std::atoi(get(args, "seed_rand_vec_trace", "1").c_str()), -1,
                      std::atoi(get(args, "estimate_aux", "1").c_str()) != 0, no_index, 6, 1e-8);
  }
  const bool gauss = m->gauss_likelihood_;
  if (!aux.empty()) {
    std::vector<double> av = parse_list(aux);
    m->SetAuxPars(av.data());
  }
  m->SetY(y.data());

  if (mode == "fit") {
    // GPB_OptimCovPar as the REModel facade runs it (re_model.cpp:339-401): initial values from
    // init_cov_pars (original scale, SetOptimConfig re_model.cpp:264-279) or FindInitCovPar
    // (InitializeCovParsIfNotDefined re_model.cpp:1142-1164), then OptimLinRegrCoefCovPar with the
    // Python package's default optimizer settings (basic.py:4510-4533: lr_cov = -1,
    // delta_rel_conv = -1, maxit = 1000, m_lbfgs = -1 -> C++ defaults; optimizer "lbfgs").
    const int no_index[1] = {-1};
    // optimizer / use_nesterov_acc / acc_rate_cov / momentum_offset / convergence_criterion: the internal
    // optimizers' settings (GPB_SetOptimConfig's arguments), defaults as the Python package's
    const std::string optimizer = get(args, "optimizer", "lbfgs");
    const std::string crit = get(args, "convergence_criterion", "relative_change_in_log_likelihood");
    m->SetOptimConfig(std::atof(get(args, "lr_cov", "-1").c_str()),
                      std::atof(get(args, "acc_rate_cov", "0.5").c_str()),
                      std::atoi(get(args, "maxit", "1000").c_str()),
                      std::atof(get(args, "delta_rel_conv", "-1").c_str()),
                      std::atoi(get(args, "use_nesterov_acc", "1").c_str()) != 0, 0, optimizer.c_str(),
                      std::atoi(get(args, "momentum_offset", "2").c_str()), crit.c_str(), 0.1, 0.5, "",
                      std::atoi(get(args, "cg_max_num_it", "1000").c_str()),
                      std::atoi(get(args, "cg_max_num_it", "1000").c_str()),
                      std::atof(get(args, "cg_delta_conv", "1e-2").c_str()),
                      std::atoi(get(args, "num_rand_vec_trace", "50").c_str()), true,
#ifdef GPB_HARNESS_GROUPED
                      "ssor",
#else
                      "vadu",
#endif
                      std::atoi(get(args, "seed_rand_vec_trace", "1").c_str()), -1,
                      std::atoi(get(args, "estimate_aux", "1").c_str()) != 0, no_index,
                      std::atoi(get(args, "m_lbfgs", "-1").c_str()), -1.);
    if (!aux.empty()) {
      std::vector<double> av = parse_list(aux);
      m->SetAuxPars(av.data());
    }
    m->SetY(y.data());
    vec_t cp(m->num_cov_par_);
    const std::string init = get(args, "init_cov_pars", "");
    if (!init.empty()) {
      std::vector<double> iv = parse_list(init);
      vec_t io = Eigen::Map<const vec_t>(iv.data(), (int)iv.size());
      m->TransformCovPars(io, cp);
    } else {
      m->FindInitCovPar(y.data(), fe_ptr, cp.data());
    }
    vec_t init_orig;
    m->TransformBackCovPars(cp, init_orig);
    int num_it = 0;
    std::vector<double> coef(std::max(p_cov, 1), 0.);
    auto a = std::chrono::steady_clock::now();
    // REModel::OptimCovPar / OptimLinRegrCoefCovPar (re_model.cpp:339-469)
    m->OptimLinRegrCoefCovPar(y.data(), p_cov > 0 ? Xcov.data() : nullptr, p_cov, cp.data(),
                              p_cov > 0 ? coef.data() : nullptr, num_it, cp.data(), nullptr, fe_ptr,
                              true, false, false, false, false);
    auto b = std::chrono::steady_clock::now();
    vec_t fit_orig;
    m->TransformBackCovPars(cp, fit_orig);
    std::printf("{\n\"n\": %d, \"d\": %d,\n", n, d);
    print_vec("init_cov_pars", init_orig.data(), (int)init_orig.size());
    print_vec("cov_pars", fit_orig.data(), (int)fit_orig.size());
    if (p_cov > 0) {
      print_vec("coef", coef.data(), p_cov);
      std::vector<double> sd_coef(p_cov), sd_cov(m->num_cov_par_);
      m->CalculateStandardErrorsCoefs(cp.data(), sd_coef.data());   // GetCoef(calc_std_dev), re_model.cpp:836-870
      print_vec("coef_std_dev", sd_coef.data(), p_cov);
      if (gp_approx == "none") {
        m->CalculateStandardErrorsCovPars(cp.data(), sd_cov.data());
        print_vec("cov_pars_std_dev", sd_cov.data(), (int)sd_cov.size());
      }
    }
    if (m->NumAuxPars() > 0) print_vec("aux_pars", m->GetAuxPars(), m->NumAuxPars());
    std::printf("\"nll\": %.17g,\n", m->neg_log_likelihood_);
    std::printf("\"num_it\": %d, \"num_ll_evaluations\": %d,\n", num_it, m->num_ll_evaluations_);
    std::printf("\"fit_time\": %.9g, \"t_construct\": %.9g,\n\"ok\": true\n}\n",
                std::chrono::duration<double>(b - a).count(), t_construct);
    return 0;
  }

  if (mode == "boost") {
    // The covariance update of R consecutive GPBoost boosting rounds as the boosting objective runs
    // it (regression_objective.hpp:153-182, objective_function.cpp:149-156): per round the score
    // F_r = scale_r * F (F from the input file), then
    //   Gaussian: g = F_r - y; REModel::OptimCovPar(g, NULL, true, reuse); CalcGradient(g, NULL, false)
    //   latent:   REModel::OptimCovPar(NULL, F_r, true, reuse); CalcGradient(grad, F_r, false)
    // REModel::OptimCovPar (re_model.cpp:339-401) = InitializeCovParsIfNotDefined(y, F) (when y is
    // given) + OptimLinRegrCoefCovPar(y, NULL, 0, cov_pars_, NULL, num_it, cov_pars_, NULL, F, true,
    // true, reuse, false, false); CalcGradient = CalcGradientF(y, F, false, cov_pars_) (:667-680).
    if (fe.empty()) { std::fprintf(stderr, "boost mode needs the fixed effects F in the input\n"); return 2; }
    const std::vector<double> scales = parse_list(get(args, "scales", "0.5,1,1.5"));
    const bool reuse = get(args, "reuse", "1") == "1";
    const int no_index[1] = {-1};
    m->SetOptimConfig(-1., 0.5, 1000, -1., true, 0, "lbfgs", 2, "relative_change_in_log_likelihood", 0.1, 0.5, "",
                      std::atoi(get(args, "cg_max_num_it", "1000").c_str()),
                      std::atoi(get(args, "cg_max_num_it", "1000").c_str()),
                      std::atof(get(args, "cg_delta_conv", "1e-2").c_str()),
                      std::atoi(get(args, "num_rand_vec_trace", "50").c_str()), true, "vadu",
                      std::atoi(get(args, "seed_rand_vec_trace", "1").c_str()), -1, true, no_index, -1, -1.);
    vec_t cp(m->num_cov_par_);
    bool initialized = false;
    if (!gauss) {   // objective_function.cpp:154-156: SetY(label); InitializeCovParsIfNotDefined(NULL, NULL)
      m->SetY(y.data());
      m->FindInitCovPar(nullptr, nullptr, cp.data());
      initialized = true;
    }
    std::printf("{\n\"n\": %d, \"d\": %d,\n\"rounds\": [\n", n, d);
    for (size_t r = 0; r < scales.size(); ++r) {
      std::vector<double> F(n), g(n);
      for (int i = 0; i < n; ++i) F[i] = scales[r] * fe[i];
      int num_it = 0;
      if (gauss) {
        for (int i = 0; i < n; ++i) g[i] = F[i] - y[i];
        if (!initialized) { m->FindInitCovPar(g.data(), nullptr, cp.data()); initialized = true; }
        m->OptimLinRegrCoefCovPar(g.data(), nullptr, 0, cp.data(), nullptr, num_it, cp.data(), nullptr, nullptr,
                                  true, true, reuse, false, false);
        m->CalcGradientF(g.data(), nullptr, false, cp);
      } else {
        m->OptimLinRegrCoefCovPar(nullptr, nullptr, 0, cp.data(), nullptr, num_it, cp.data(), nullptr, F.data(),
                                  true, true, reuse, false, false);
        m->CalcGradientF(g.data(), F.data(), false, cp);
      }
      vec_t co;
      m->TransformBackCovPars(cp, co);
      std::printf("{");
      print_vec("cov_pars", co.data(), (int)co.size());
      std::printf("\"num_it\": %d, \"nll\": %.17g,\n", num_it, m->neg_log_likelihood_);
      print_vec("grad_f", g.data(), n, false);
      std::printf("}%s\n", r + 1 < scales.size() ? "," : "");
    }
    std::printf("],\n\"ok\": true\n}\n");
    return 0;
  }

  vec_t orig = Eigen::Map<const vec_t>(cov_pars_orig.data(), (int)cov_pars_orig.size());
  vec_t trafo;
  m->TransformCovPars(orig, trafo);

  if (mode == "grad_f") {
    // REModel::CalcGradient -> CalcGradientF (re_model_template.h:3021-3043) at cov_pars: Gaussian:
    // input y, output Psi^-1 y / sigma2; non-Gaussian: the gradient wrt F at the mode (F = fe)
    if (!gauss)
      for (const auto& c : m->unique_clusters_) m->likelihood_[c]->InitializeModeAvec();
    std::vector<double> g(y);
    m->CalcGradientF(g.data(), fe_ptr, true, trafo);
    std::printf("{\n\"n\": %d, \"d\": %d,\n", n, d);
    print_vec("grad_f", g.data(), n);
    std::printf("\"ok\": true\n}\n");
    return 0;
  }

  if (mode == "pred_train") {
    // GPB_PredictREModelTrainingDataRandomEffects at cov_pars (re_model.cpp -> PredictTrainingDataRandomEffects):
    // one block of n means per random-effect component (grouped: K), then the variances (calc_var)
    const int ncomp = std::max(1, (int)num_re_group);
    const bool calc_var = gauss && get(args, "calc_var", "1") == "1";
    std::vector<double> out((size_t)2 * n * ncomp, 0.);
    m->PredictTrainingDataRandomEffects(trafo.data(), nullptr, y.data(), out.data(), true, nullptr, calc_var);
    std::printf("{\n\"n\": %d, \"d\": %d,\n", n, d);
    print_vec("mean", out.data(), n * ncomp);
    if (calc_var) print_vec("var", out.data() + (size_t)n * ncomp, n * ncomp);
    std::printf("\"ok\": true\n}\n");
    return 0;
  }

  if (mode == "predict") {
    // GPB_SetPredictionData + GPB_PredictREModel at cov_pars (re_model.cpp:927-1000 -> Predict
    // re_model_template.h:3146): prediction coordinates from the file `pred` (int32 np, double
    // coords[np * d] column-major); outputs the predictive mean and (predict_var) variances.
    // Grouped models (num_re_group > 0): the file holds int32 np, then int32 labels[np * K]
    // (effect-major), passed as the NUL-separated label strings of re_group_data_pred.
    FILE* fp = std::fopen(get(args, "pred", "").c_str(), "rb");
    if (!fp) { std::perror("open pred"); return 2; }
    int32_t np = 0;
    if (std::fread(&np, 4, 1, fp) != 1 || np <= 0) return 2;
    // (combined GP + grouped models: double coords[np * d] first, then the labels)
    std::vector<double> xp((size_t)np * d);
    std::string re_group_pred;
    if (d > 0 && std::fread(xp.data(), 8, xp.size(), fp) != xp.size()) return 2;
    if (num_re_group > 0) {
      std::vector<int32_t> lab((size_t)np * num_re_group);
      if (std::fread(lab.data(), 4, lab.size(), fp) != lab.size()) return 2;
      for (int32_t v : lab) {
        re_group_pred += std::to_string(v);
        re_group_pred.push_back('\0');
      }
    }
    std::fclose(fp);
    const bool pcov = get(args, "predict_cov", "0") == "1";
    const bool pvar = !pcov && get(args, "predict_var", "0") == "1";
    const bool presp = get(args, "predict_response", "0") == "1";
    const std::string ptype = get(args, "vecchia_pred_type", "");
    if (d > 0)
      m->SetPredictionData(np, nullptr, nullptr, nullptr, xp.data(), nullptr, nullptr,
                           ptype.empty() ? nullptr : ptype.c_str(),
                           std::atoi(get(args, "num_neighbors_pred", "-1").c_str()),
                           std::atof(get(args, "cg_delta_conv_pred", "-1").c_str()),
                           std::atoi(get(args, "nsim_var_pred", "-1").c_str()), -1);
    std::vector<double> out((size_t)np + (pcov ? (size_t)np * np : (size_t)np), 0.);
    m->Predict(trafo.data(), y.data(), np, out.data(), true, pcov, pvar, presp, nullptr, nullptr, nullptr,
               num_re_group > 0 ? re_group_pred.data() : nullptr, nullptr, d > 0 ? xp.data() : nullptr,
               nullptr, false, fe_ptr, nullptr);
    std::printf("{\n\"n\": %d, \"d\": %d, \"np\": %d,\n", n, d, np);
    print_vec("mean", out.data(), np);
    if (pvar) print_vec("var", out.data() + np, np);
    if (pcov) print_vec("cov", out.data() + np, np * np);
    std::printf("\"ok\": true\n}\n");
    return 0;
  }

  if (mode == "stddev") {
    // GPB_GetCovPar(calc_std_dev = true) at cov_pars: CalculateStandardErrorsCovPars
    // (re_model_template.h:1634-1660 -> CalcStdDevCovPar :9775-9789), transformed-scale input
    vec_t sd(m->num_cov_par_);
    m->CalculateStandardErrorsCovPars(trafo.data(), sd.data());
    std::printf("{\n\"n\": %d, \"d\": %d,\n", n, d);
    print_vec("cov_pars", orig.data(), (int)orig.size());
    print_vec("std_dev", sd.data(), (int)sd.size());
    std::printf("\"ok\": true\n}\n");
    return 0;
  }

  double nll = 0., sigma2 = gauss ? trafo[0] : 1.;
  vec_t grad, gb;
  std::vector<double> times;
  for (int r = 0; r < reps; ++r) {
    vec_t cp = trafo;
    if (!gauss) {
      for (const auto& c : m->unique_clusters_) m->likelihood_[c]->InitializeModeAvec();
    }
    auto a = std::chrono::steady_clock::now();
    m->CalcCovFactorOrModeAndNegLL(cp, fe_ptr);
    nll = m->neg_log_likelihood_;
    if (gauss && mode == "lbfgs") {
      sigma2 = m->ProfileOutSigma2();
      cp[0] = sigma2;
      m->EvalNegLogLikelihoodOnlyUpdateNuggetVariance(sigma2, nll);
      m->CalcGradPars(cp, sigma2, true, false, grad, gb, false, false, nullptr, false);
    }
    else if (gauss) {
      m->CalcGradPars(cp, cp[0], true, false, grad, gb, true, false, nullptr, false);
    }
    else {
      m->CalcGradPars(cp, 1., true, false, grad, gb, false, false, fe_ptr, false);
    }
    auto b = std::chrono::steady_clock::now();
    times.push_back(std::chrono::duration<double>(b - a).count());
  }
  std::vector<double> ts = times;
  std::sort(ts.begin(), ts.end());

  std::printf("{\n");
  std::printf("\"n\": %d, \"d\": %d,\n", n, d);
  std::printf("\"gauss\": %s,\n", gauss ? "true" : "false");
  std::printf("\"nll\": %.17g,\n", nll);
  std::printf("\"sigma2\": %.17g,\n", sigma2);
  print_vec("cov_pars_trafo", trafo.data(), (int)trafo.size());
  print_vec("grad", grad.data(), (int)grad.size());
  print_vec("times", times.data(), (int)times.size());
  std::printf("\"median_time\": %.9g,\n", ts[ts.size() / 2]);
  std::printf("\"t_construct\": %.9g,\n", t_construct);
  if (gauss && gp_approx == "vecchia") {
    std::printf("\"yTPsiInvy\": %.17g, \"log_det_Psi\": %.17g,\n", m->yTPsiInvy_, m->log_det_Psi_);
  }
  const bool vif = gp_approx == "full_scale_vecchia" || gp_approx == "vif";
  if (gp_approx == "fitc" || vif) {
    if (gauss) std::printf("\"yTPsiInvy\": %.17g, \"log_det_Psi\": %.17g,\n", m->yTPsiInvy_, m->log_det_Psi_);
    const den_mat_t& ip = m->gp_coords_ip_mat_;
    std::vector<double> ipv((size_t)ip.rows() * ip.cols());
    for (int i = 0; i < (int)ip.rows(); ++i)
      for (int q = 0; q < (int)ip.cols(); ++q) ipv[(size_t)i * ip.cols() + q] = ip(i, q);
    print_vec("ind_points", ipv.data(), (int)ipv.size());
  }
  if ((gp_approx == "vecchia" || gp_approx == "vecchia_latent" || vif) && dump_nn) {
    const auto& perm = m->data_indices_per_cluster_[m->unique_clusters_[0]];
    std::printf("\"perm\": [");
    for (size_t i = 0; i < perm.size(); ++i) std::printf("%s%d", i ? "," : "", perm[i]);
    std::printf("],\n");
    const auto& nn = m->nearest_neighbors_[m->unique_clusters_[0]][0];
    std::printf("\"neighbors\": [");
    for (size_t i = 0; i < nn.size(); ++i) {
      std::printf("%s[", i ? "," : "");
      for (size_t j = 0; j < nn[i].size(); ++j) std::printf("%s%d", j ? "," : "", nn[i][j]);
      std::printf("]");
    }
    std::printf("],\n");
    // D^-1 diagonal (Vecchia order)
    const sp_mat_t& Dinv = m->D_inv_[m->unique_clusters_[0]][0];
    vec_t dd = Dinv.diagonal();
    print_vec("D_inv", dd.data(), (int)dd.size());
    // B rows: dense values per row in neighbor order
    const sp_mat_t& B = m->B_[m->unique_clusters_[0]][0];
    std::printf("\"B_rows\": [");
    for (size_t i = 0; i < nn.size(); ++i) {
      std::printf("%s[", i ? "," : "");
      for (size_t j = 0; j < nn[i].size(); ++j) std::printf("%s%.17g", j ? "," : "", B.coeff((int)i, nn[i][j]));
      std::printf("]");
    }
    std::printf("],\n");
  }
  std::printf("\"ok\": true\n}\n");
  return 0;
}
