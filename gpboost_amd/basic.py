"""Python host mirror of the reference ``gpboost.GPModel`` for the likelihood path.

Same constructor arguments, argument checking and error behaviour as the reference
(python-package/gpboost/basic.py:4054-6620, ``GPModel.__init__`` :4062,
``neg_log_likelihood`` :5284), calling the MI355X library through the same C ABI
(include/gpboost_amd.h) with ctypes. There is no CPU fallback: if the HIP library
is missing or no GPU is visible, construction raises ``GPBoostError``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GPBOOST_AMD_VARIANT=<name> selects an in-tree A/B build of the same sources
# (gpboost_amd/lib/ab/libgpboost_amd_<name>.so, see build.py) for kernel experiments.
_VARIANT = os.environ.get("GPBOOST_AMD_VARIANT", "")
LIB_PATH = (os.path.join(_HERE, "lib", "ab", f"libgpboost_amd_{_VARIANT}.so") if _VARIANT
            else os.path.join(_HERE, "lib", "libgpboost_amd.so"))


_HostReduceFn = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_void_p)


class GPBoostError(Exception):
    """Error thrown by the library (reference basic.py:136-145)."""


def _load_lib():
    if not os.path.exists(LIB_PATH):
        raise GPBoostError(f"HIP library not built: {LIB_PATH} (run python -m gpboost_amd.build)")
    lib = ctypes.CDLL(LIB_PATH)
    lib.LGBM_GetLastError.restype = ctypes.c_char_p
    D = ctypes.POINTER(ctypes.c_double)
    lib.GPB_EvalNegLogLikelihoodGrad.argtypes = [ctypes.c_void_p, D, D, D, ctypes.c_int, D, D, D]
    lib.GPB_CombinePartials.argtypes = [D, ctypes.c_int32, ctypes.c_double, ctypes.c_int, D, D, D]
    I = ctypes.POINTER(ctypes.c_int)
    c = ctypes
    lib.GPB_SetOptimConfig.argtypes = [c.c_void_p, D, c.c_double, c.c_double, c.c_int, c.c_double, c.c_bool, c.c_int,
                                       c.c_bool, c.c_char_p, c.c_int, c.c_char_p, c.c_int, D, c.c_double, c.c_double,
                                       c.c_char_p, c.c_int, c.c_int, c.c_double, c.c_int, c.c_bool, c.c_char_p,
                                       c.c_int, c.c_int, D, c.c_bool, I, c.c_int, c.c_double]
    lib.GPB_SetDistributedHostReduce.argtypes = [c.c_void_p, c.c_int, c.c_int, _HostReduceFn, c.c_void_p]
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _load_lib()
    return _LIB


def _safe_call(ret: int):
    """reference basic.py:136-145"""
    if ret != 0:
        raise GPBoostError(lib().LGBM_GetLastError().decode("utf-8"))


def c_str(s: str | None):
    return ctypes.c_char_p(s.encode("utf-8")) if s is not None else None


def _dp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _as1d(x, name: str) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    if not np.all(np.isfinite(a)):
        raise ValueError(f"'{name}' contains NaN or Inf")
    return a


class GPModel:
    """Gaussian process model (reference ``gpboost.GPModel``), likelihood evaluation subset."""

    _SUPPORTED_APPROX = ("none", "vecchia", "vecchia_latent", "fitc")

    def __init__(self, likelihood="gaussian", group_data=None, group_rand_coef_data=None,
                 ind_effect_group_rand_coef=None, drop_intercept_group_rand_effect=None, gp_coords=None,
                 gp_rand_coef_data=None, cov_function="matern", cov_fct_shape=1.5, gp_approx="none",
                 num_parallel_threads=None, GPU_use=True, matrix_inversion_method="default", weights=None,
                 likelihood_learning_rate=1., cov_fct_taper_range=1., cov_fct_taper_shape=1., num_neighbors=None,
                 vecchia_ordering="random", ind_points_selection="kmeans++", num_ind_points=None,
                 cover_tree_radius=1., seed=0, cluster_ids=None, num_data=None, likelihood_additional_param=None,
                 free_raw_data=False, model_file=None, model_dict=None, vecchia_approx=None,
                 vecchia_pred_type=None, num_neighbors_pred=None):
        self.handle = None
        if group_rand_coef_data is not None:
            raise GPBoostError("grouped random coefficients are out of scope for gpboost_amd")
        if gp_rand_coef_data is not None:
            raise GPBoostError("GP random coefficients are out of scope for gpboost_amd")
        if model_file is not None or model_dict is not None:
            raise GPBoostError("model loading is out of scope for gpboost_amd")
        if group_data is not None:   # grouped random effects, optionally beside one dense GP (gp_approx "none")
            self._init_grouped(group_data, likelihood, matrix_inversion_method, seed, cluster_ids, weights,
                               gp_coords, cov_function, cov_fct_shape, gp_approx)
            return
        if gp_coords is None:
            raise ValueError("Either 'group_data' or 'gp_coords' must be provided")
        if vecchia_approx is not None and vecchia_approx:
            gp_approx = "vecchia"
        coords = np.asarray(gp_coords, dtype=np.float64)
        if coords.ndim == 1:
            coords = coords.reshape(-1, 1)
        self.num_data = coords.shape[0]
        self.dim_coords = coords.shape[1]
        self.gp_approx = gp_approx
        self.cov_function = cov_function
        self.cov_fct_shape = float(cov_fct_shape)
        vif = gp_approx in ("full_scale_vecchia", "vif", "VIF")
        if num_neighbors is None:   # the reference's defaults (re_model_template.h:288-297, 320-330)
            num_neighbors = 30 if vif else 20
        if num_ind_points is None:
            num_ind_points = 200 if vif else 500
        self.num_neighbors = int(num_neighbors)
        self.likelihood = likelihood
        coords_cm = np.ascontiguousarray(coords.T).reshape(-1)  # column-major, as the reference passes it
        cluster = None
        if cluster_ids is not None:
            cluster = np.ascontiguousarray(np.asarray(cluster_ids), dtype=np.int32)
        handle = ctypes.c_void_p()
        _safe_call(lib().GPB_CreateREModel(
            ctypes.c_int32(self.num_data),
            _ip(cluster) if cluster is not None else None,
            None, ctypes.c_int32(0), None, None, ctypes.c_int32(0), None,
            ctypes.c_int32(1), _dp(coords_cm), ctypes.c_int(self.dim_coords), None, ctypes.c_int32(0),
            c_str(cov_function), ctypes.c_double(self.cov_fct_shape), c_str(gp_approx),
            ctypes.c_double(cov_fct_taper_range), ctypes.c_double(cov_fct_taper_shape),
            ctypes.c_int(self.num_neighbors), c_str(vecchia_ordering), ctypes.c_int(num_ind_points),
            ctypes.c_double(cover_tree_radius), c_str(ind_points_selection), c_str(likelihood),
            ctypes.c_double(likelihood_additional_param or 0.), c_str(matrix_inversion_method),
            ctypes.c_int(seed), ctypes.c_int(num_parallel_threads or -1), ctypes.c_bool(GPU_use),
            ctypes.c_bool(weights is not None), None, ctypes.c_double(likelihood_learning_rate),
            ctypes.byref(handle)))
        self.handle = handle
        self.num_group_re = 0
        self._post_init()

    def _init_grouped(self, group_data, likelihood, matrix_inversion_method, seed, cluster_ids, weights,
                      gp_coords=None, cov_function="matern", cov_fct_shape=1.5, gp_approx="none"):
        """Grouped random effects (reference basic.py GPModel.__init__ group_data handling): labels are
        converted to strings and passed column-major as NUL-terminated C strings. With gp_coords: the
        combined model with one GP component (gp_approx "none")."""
        g = np.asarray(group_data)
        if g.ndim == 1:
            g = g.reshape(-1, 1)
        if g.ndim != 2 or g.shape[0] == 0:
            raise ValueError("'group_data' must be a vector or a matrix with one row per observation")
        self.num_data, self.num_group_re = g.shape
        self.gp_approx = "none"
        self.likelihood = likelihood
        self.dim_coords = 0
        self.num_neighbors = 0
        self.cov_function = None
        self.cov_fct_shape = 0.
        self.has_gp = gp_coords is not None
        coords_cm = None
        if self.has_gp:
            coords = np.asarray(gp_coords, dtype=np.float64)
            if coords.ndim == 1:
                coords = coords.reshape(-1, 1)
            if coords.shape[0] != self.num_data:
                raise ValueError("Incorrect number of data points in 'gp_coords'")
            self.dim_coords = coords.shape[1]
            self.cov_function = cov_function
            self.cov_fct_shape = float(cov_fct_shape)
            self.gp_approx = gp_approx
            coords_cm = np.ascontiguousarray(coords.T).reshape(-1)
        labels = g.astype(np.dtype(str)).flatten(order="F")
        buf = ctypes.create_string_buffer(b"\0".join(s.encode() for s in labels) + b"\0")
        cluster = None
        if cluster_ids is not None:
            cluster = np.ascontiguousarray(np.asarray(cluster_ids), dtype=np.int32)
        handle = ctypes.c_void_p()
        _safe_call(lib().GPB_CreateREModel(
            ctypes.c_int32(self.num_data), _ip(cluster) if cluster is not None else None,
            buf, ctypes.c_int32(self.num_group_re), None, None, ctypes.c_int32(0), None,
            ctypes.c_int32(1 if self.has_gp else 0), _dp(coords_cm) if self.has_gp else None,
            ctypes.c_int(self.dim_coords), None, ctypes.c_int32(0),
            c_str(cov_function if self.has_gp else "exponential"),
            ctypes.c_double(self.cov_fct_shape if self.has_gp else 0.5), c_str(self.gp_approx),
            ctypes.c_double(1.), ctypes.c_double(1.),
            ctypes.c_int(0), c_str("random"), ctypes.c_int(0), ctypes.c_double(1.), c_str("kmeans++"),
            c_str(likelihood), ctypes.c_double(0.), c_str(matrix_inversion_method), ctypes.c_int(seed),
            ctypes.c_int(-1), ctypes.c_bool(True), ctypes.c_bool(weights is not None), None, ctypes.c_double(1.),
            ctypes.byref(handle)))
        self.handle = handle
        self._post_init()

    def _post_init(self):
        self.has_covariates = False
        self.num_covariates = 0
        k = ctypes.c_int(0)
        _safe_call(lib().GPB_GetNumCovPars(self.handle, ctypes.byref(k)))
        self.num_cov_pars = k.value
        _safe_call(lib().GPB_GetNumAuxPars(self.handle, ctypes.byref(k)))
        self.num_aux_pars = k.value
        # reference basic.py:4510-4533 (parameters of the likelihood path only)
        self.params = {"cg_max_num_it": 1000, "cg_max_num_it_tridiag": 1000, "cg_delta_conv": 1e-2,
                       "num_rand_vec_trace": 50, "reuse_rand_vec_trace": True, "seed_rand_vec_trace": 1,
                       "cg_preconditioner_type": None, "init_aux_pars": None, "estimate_aux_pars": True,
                       "delta_conv_mode_finding": -1.,
                       # covariance-parameter optimizer (reference basic.py:4510-4533 defaults)
                       "optimizer_cov": None, "init_cov_pars": None, "maxit": 1000, "delta_rel_conv": -1.,
                       "lr_cov": -1., "m_lbfgs": -1, "trace": False,
                       "convergence_criterion": "relative_change_in_log_likelihood",
                       "acc_rate_cov": 0.5, "use_nesterov_acc": True, "nesterov_schedule_version": 0,
                       "momentum_offset": 2, "estimate_cov_par_index": None}

    def __del__(self):
        try:
            if self.handle is not None and _LIB is not None:
                _LIB.GPB_REModelFree(self.handle)
        except Exception:
            pass

    # ------------------------------------------------------------------ reference API
    def _call(self, ret: int):
        """_safe_call, then re-raise an exception of a host all-reduce callback (set_distributed_host):
        the callback fills the buffer with NaN on failure, so the library stops with an error."""
        err = getattr(self, "_host_reduce_error", None)
        if err is not None:
            self._host_reduce_error = None
            raise GPBoostError(f"the host all-reduce callback failed: {err!r}") from err
        _safe_call(ret)

    def _check_y(self, y):
        if y is None:
            return None
        y = _as1d(y, "y")
        if y.shape[0] != self.num_data:
            raise ValueError("Incorrect number of data points in 'y'")
        return y

    def _check_cov_pars(self, cov_pars):
        cp = _as1d(cov_pars, "cov_pars")
        if cp.shape[0] != self.num_cov_pars:
            raise ValueError("'cov_pars' does not contain the correct number of parameters")
        return cp

    def set_optim_params(self, params=None):
        """Store likelihood-path and optimizer settings through GPB_SetOptimConfig (reference
        basic.py:5380-5540). Covariance-parameter optimizers: "lbfgs" (the reference default),
        "gradient_descent" (Nesterov: use_nesterov_acc, acc_rate_cov, momentum_offset,
        nesterov_schedule_version) and "fisher_scoring" (Gaussian likelihood, no covariates);
        convergence_criterion as the reference's. Keys of the coefficient optimizers are accepted and
        have no effect."""
        if params:
            for key, val in params.items():
                if key == "init_aux_pars" and val is not None:
                    val = _as1d(val, "params['init_aux_pars']")
                    if val.shape[0] != self.num_aux_pars:
                        raise ValueError("params['init_aux_pars'] does not contain the correct number of parameters")
                if key == "init_cov_pars" and val is not None:
                    val = _as1d(val, "params['init_cov_pars']")
                    if val.shape[0] != self.num_cov_pars:
                        raise ValueError("params['init_cov_pars'] does not contain the correct number of parameters")
                self.params[key] = val
        p = self.params
        aux = p["init_aux_pars"]
        init = p["init_cov_pars"]
        no_index = np.array([-1], dtype=np.int32)
        if p["estimate_cov_par_index"] is not None:   # reference basic.py: int32 array of num_cov_pars entries
            no_index = np.asarray(p["estimate_cov_par_index"], dtype=np.int32).reshape(-1)
            if no_index.shape[0] != self.num_cov_pars:
                raise ValueError("params['estimate_cov_par_index'] does not contain the correct number of parameters")
        _safe_call(lib().GPB_SetOptimConfig(
            self.handle, _dp(init) if init is not None else None, float(p["lr_cov"]), float(p["acc_rate_cov"]),
            int(p["maxit"]), float(p["delta_rel_conv"]), bool(p["use_nesterov_acc"]),
            int(p["nesterov_schedule_version"]), bool(p["trace"]), c_str(p["optimizer_cov"]), int(p["momentum_offset"]),
            c_str(p["convergence_criterion"]), 0, None, 0.1, 0.5, None,
            int(p["cg_max_num_it"]), int(p["cg_max_num_it_tridiag"]), float(p["cg_delta_conv"]),
            int(p["num_rand_vec_trace"]), bool(p["reuse_rand_vec_trace"]),
            p["cg_preconditioner_type"].encode() if p["cg_preconditioner_type"] else None,
            int(p["seed_rand_vec_trace"]), -1, _dp(aux) if aux is not None else None,
            bool(p["estimate_aux_pars"]), no_index.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), int(p["m_lbfgs"]),
            float(p["delta_conv_mode_finding"])))

    def fit(self, y, X=None, params=None, offset=None, fixed_effects=None):
        """Estimate the covariance parameters (and, with X, the linear regression coefficients) by
        maximising the (approximate marginal) likelihood (reference basic.py:5067-5275 ->
        GPB_OptimCovPar, or GPB_OptimLinRegrCoefCovPar when X is given: GLS coefficients)."""
        if fixed_effects is not None:
            raise GPBoostError("The argument 'fixed_effects' is discontinued. Use the renamed equivalent argument 'offset' instead")
        y = self._check_y(y)
        off = None
        if offset is not None:
            off = _as1d(offset, "offset")
            if off.shape[0] != self.num_data:
                raise ValueError("Incorrect number of data points in 'offset'")
        self.set_optim_params(params)
        if X is None:
            self.has_covariates = False
            self._call(lib().GPB_OptimCovPar(self.handle, _dp(y), _dp(off) if off is not None else None))
        else:
            Xa = np.asarray(X, dtype=np.float64)
            if Xa.ndim == 1:
                Xa = Xa.reshape(-1, 1)
            if Xa.shape[0] != self.num_data:
                raise ValueError("Incorrect number of data points in 'X'")
            if not np.all(np.isfinite(Xa)):
                raise ValueError("'X' contains NaN or Inf")
            self.num_covariates = Xa.shape[1]
            self.has_covariates = True
            xcol = np.ascontiguousarray(Xa.T).reshape(-1)   # column-major, as the reference passes it
            self._call(lib().GPB_OptimLinRegrCoefCovPar(self.handle, _dp(y), _dp(xcol), ctypes.c_int(self.num_covariates),
                                                        _dp(off) if off is not None else None))
        self.model_fitted = True
        return self

    def get_coef(self, std_err=False):
        """Linear regression coefficients (GPB_GetCoef); std_err=True: 2 x p [coefficients; std. devs.]
        (reference basic.py:5630-5660)."""
        if not getattr(self, "has_covariates", False):
            raise GPBoostError("Model does not have covariates for a linear predictor")
        p = self.num_covariates
        out = np.zeros(2 * p if std_err else p)
        _safe_call(lib().GPB_GetCoef(self.handle, _dp(out), ctypes.c_bool(std_err)))
        return out.reshape(2, -1) if std_err else out

    def predict_training_data_random_effects(self, predict_var=False):
        """Predicted training-data random effects (GPB_PredictREModelTrainingDataRandomEffects,
        reference basic.py:6316-6367): (n,) means, or (n, 2) [mean, variance] with predict_var; grouped
        models: (n, K) means per effect, or (n, 2K) [means..., variances...]."""
        k = max(1, getattr(self, "num_group_re", 0))
        out = np.zeros((2 if predict_var else 1) * k * self.num_data)
        _safe_call(lib().GPB_PredictREModelTrainingDataRandomEffects(self.handle, None, None, _dp(out), None,
                                                                     ctypes.c_bool(bool(predict_var))))
        if getattr(self, "num_group_re", 0):
            return out.reshape(-1, self.num_data).T.copy()
        return out.reshape(2, -1).T.copy() if predict_var else out

    def _get_string(self, fn):
        buf = ctypes.create_string_buffer(256)
        k = ctypes.c_int(0)
        _safe_call(fn(self.handle, buf, ctypes.byref(k)))
        return buf.value.decode()

    def get_optim_params(self):
        """Optimizer settings incl. the names the library reports (reference basic.py:5544-5581:
        GPB_GetOptimizerCovPars / GetOptimizerCoef / GetCGPreconditionerType / GetInitCovPar /
        GetInitAuxPars)."""
        params = dict(self.params)
        params["optimizer_cov"] = self._get_string(lib().GPB_GetOptimizerCovPars)
        params["optimizer_coef"] = self._get_string(lib().GPB_GetOptimizerCoef)
        params["cg_preconditioner_type"] = self._get_string(lib().GPB_GetCGPreconditionerType)
        init = self.get_init_cov_pars()
        if init is not None:
            params["init_cov_pars"] = init
        if self.num_aux_pars > 0:
            a = np.zeros(self.num_aux_pars)
            _safe_call(lib().GPB_GetInitAuxPars(self.handle, _dp(a)))
            if np.any(a != -1.):
                params["init_aux_pars"] = a
        return params

    def get_response_data(self):
        out = np.zeros(self.num_data)
        _safe_call(lib().GPB_GetResponseData(self.handle, _dp(out)))
        return out

    def get_covariate_data(self):
        out = np.zeros(self.num_data * self.num_covariates)
        _safe_call(lib().GPB_GetCovariateData(self.handle, _dp(out)))
        return out.reshape(self.num_covariates, self.num_data).T.copy()

    def can_calculate_standard_errors_cov_pars(self):
        out = ctypes.c_int(0)
        _safe_call(lib().GPB_CanCalculateStandardErrorsCovPars(self.handle, ctypes.byref(out)))
        return bool(out.value)

    def get_init_cov_pars(self):
        """Initial covariance parameters of the last fit (original scale; GPB_GetInitCovPar), or
        None when none were given or determined (reference basic.py:5564-5570)."""
        out = np.zeros(self.num_cov_pars)
        _safe_call(lib().GPB_GetInitCovPar(self.handle, _dp(out)))
        return None if np.all(out == -1.) else out

    def cov_par_names(self):
        """Parameter names as the reference labels them (error term only for the Gaussian likelihood)."""
        if getattr(self, "num_group_re", 0):
            return (["Error_term"] + [f"Group_{k + 1}" for k in range(self.num_group_re)] +
                    (["GP_var", "GP_range"] if getattr(self, "has_gp", False) else []))
        return (["Error_term"] if self.num_cov_pars == 3 else []) + ["GP_var", "GP_range"]

    def summary(self, std_err=False):
        """Print a summary of the fitted parameters (reference basic.py:5709-5770, GP models):
        log-likelihood, AIC and BIC after a fit, covariance parameters (with standard deviations
        when std_err, Gaussian models with gp_approx "none" / "vecchia") and auxiliary parameters."""
        import pandas as pd
        cp = self.get_cov_pars(std_err=std_err)
        rows = cp if std_err else cp.reshape(1, -1)
        print("=====================================================")
        print("Model summary:")
        print("Nb. observations: " + str(self.num_data))
        if getattr(self, "model_fitted", False):
            ll = -self.get_current_neg_log_likelihood()
            npar = self.num_cov_pars
            aic = 2 * npar - 2 * ll
            bic = npar * np.log(self.num_data) - 2 * ll
            out = pd.DataFrame([[round(ll, 2), round(aic, 2), round(bic, 2)]], columns=["Log-lik", "AIC", "BIC"])
            print(out.to_string(index=False))
            print("-----------------------------------------------------")
        print("Covariance parameters (random effects):")
        print(pd.DataFrame(rows.T, index=self.cov_par_names(),
                           columns=["Param.", "Std. dev."] if std_err else ["Param."]).round(4).to_string())
        if self.num_aux_pars:
            aux, name = self.get_aux_pars()
            print("-----------------------------------------------------")
            print("Additional parameters:")
            print(pd.DataFrame(aux.reshape(-1, 1), index=[name or "aux"], columns=["Param."]).round(4).to_string())
        print("=====================================================")

    def get_num_optim_iter(self):
        """Number of optimizer iterations of the last fit (GPB_GetNumIt)."""
        k = ctypes.c_int(0)
        _safe_call(lib().GPB_GetNumIt(self.handle, ctypes.byref(k)))
        return k.value

    def get_aux_pars(self):
        out = np.zeros(max(self.num_aux_pars, 1))
        name = ctypes.create_string_buffer(128)
        _safe_call(lib().GPB_GetAuxPars(self.handle, _dp(out), name))
        return out[: self.num_aux_pars], name.value.decode()

    def neg_log_likelihood(self, cov_pars, y, fixed_effects=None, aux_pars=None):
        """Negative log-likelihood at ``cov_pars`` (original scale), reference basic.py:5284."""
        y = self._check_y(y)
        cp = self._check_cov_pars(cov_pars)
        if aux_pars is not None:   # reference basic.py:5334-5335
            self.set_optim_params({"init_aux_pars": aux_pars})
        fe = None
        if fixed_effects is not None:
            fe = _as1d(fixed_effects, "fixed_effects")
            if fe.shape[0] != self.num_data:
                raise ValueError("Length of 'fixed_effects' is not correct ")
        negll = ctypes.c_double(0)
        self._call(lib().GPB_EvalNegLogLikelihood(self.handle, _dp(y) if y is not None else None, _dp(cp),
                                                  _dp(fe) if fe is not None else None, ctypes.byref(negll)))
        return negll.value

    def get_current_neg_log_likelihood(self):
        v = ctypes.c_double(0)
        _safe_call(lib().GPB_GetCurrentNegLogLikelihood(self.handle, ctypes.byref(v)))
        return v.value

    def get_cov_pars(self, std_err=False):
        """Covariance parameters (original scale); std_err=True: 2 x P array [parameters; standard
        deviations] (reference basic.py get_cov_pars: a two-row table; dense Gaussian models only)."""
        out = np.zeros(2 * self.num_cov_pars if std_err else self.num_cov_pars)
        _safe_call(lib().GPB_GetCovPar(self.handle, _dp(out), ctypes.c_bool(std_err)))
        return out.reshape(2, -1) if std_err else out

    # ------------------------------------------------------------------ extensions
    def neg_log_likelihood_and_grad(self, cov_pars, y=None, profile_sigma2=False, fixed_effects=None):
        """nll and gradient in one device evaluation (include/gpboost_amd.h GPB_EvalNegLogLikelihoodGrad).

        profile_sigma2=False: gradient wrt log of all transformed covariance parameters.
        profile_sigma2=True : the reference's L-BFGS objective unit (sigma2 profiled out).
        Returns (nll, grad, sigma2)."""
        y = self._check_y(y)
        fe = _as1d(fixed_effects, "fixed_effects") if fixed_effects is not None else None
        # per-model argument buffers and their ctypes pointers, made once: an L-BFGS loop calls
        # this every iteration and the device evaluation itself takes well under a millisecond
        if getattr(self, "_eval_bufs", None) is None:
            bufs = dict(cp=np.zeros(self.num_cov_pars), negll=np.zeros(1),
                        grad=np.zeros(self.num_cov_pars + self.num_aux_pars), s2=np.zeros(1))
            self._eval_bufs = (bufs, {k: _dp(v) for k, v in bufs.items()})
        bufs, ptrs = self._eval_bufs
        cp = bufs["cp"]
        v = np.asarray(cov_pars, dtype=np.float64).reshape(-1)
        if v.shape[0] != self.num_cov_pars:
            raise ValueError("'cov_pars' does not contain the correct number of parameters")
        cp[:] = v
        if not np.isfinite(cp).all():
            raise ValueError("'cov_pars' contains NaN or Inf")
        negll, grad, s2 = bufs["negll"], bufs["grad"], bufs["s2"]
        grad.fill(np.nan)
        self._call(lib().GPB_EvalNegLogLikelihoodGrad(
            self.handle, _dp(y) if y is not None else None, ptrs["cp"], _dp(fe) if fe is not None else None,
            int(bool(profile_sigma2)), ptrs["negll"], ptrs["grad"], ptrs["s2"]))
        if profile_sigma2:
            g = grad[: self.num_cov_pars - 1]
        elif self.num_aux_pars and self.params["estimate_aux_pars"]:
            g = grad[: self.num_cov_pars + self.num_aux_pars]
        else:
            g = grad[: self.num_cov_pars]
        return float(negll[0]), g.copy(), float(s2[0])

    def calc_gradient_f(self, y=None, fixed_effects=None, calc_cov_factor=True):
        """Gradient of the (approximate marginal) negative log-likelihood wrt the fixed effects F at the
        current covariance parameters (GPB_CalcGradientF = the reference's REModel::CalcGradient, the
        GPBoost algorithm's boosting gradient). Gaussian likelihood: y = F - label, returns
        Psi^-1 y / sigma^2; latent models: F = fixed_effects, returns -dlog p/dF + implicit terms.
        calc_cov_factor=False (after optim_cov_par_boosting) keeps the last evaluation's Laplace mode."""
        if y is not None:
            out = _as1d(y, "y").copy()
        else:
            out = np.zeros(self.num_data)
        fe = _as1d(fixed_effects, "fixed_effects") if fixed_effects is not None else None
        self._call(lib().GPB_CalcGradientF(self.handle, _dp(out), _dp(fe) if fe is not None else None,
                                           ctypes.c_bool(calc_cov_factor)))
        return out

    def optim_cov_par_boosting(self, y=None, fixed_effects=None, reuse_learning_rates=True):
        """The covariance update of one GPBoost boosting round (GPB_OptimCovParBoosting = the reference's
        REModel::OptimCovPar(y, F, called_in_GPBoost_algorithm=True, reuse_learning_rates_gp_model),
        regression_objective.hpp:164, 178). Gaussian: y = F - label, fixed_effects None; latent models:
        y None (the label set before) and fixed_effects = the current score F."""
        yy = _as1d(y, "y") if y is not None else None
        fe = _as1d(fixed_effects, "fixed_effects") if fixed_effects is not None else None
        self._call(lib().GPB_OptimCovParBoosting(self.handle, _dp(yy) if yy is not None else None,
                                                 _dp(fe) if fe is not None else None, ctypes.c_bool(True),
                                                 ctypes.c_bool(reuse_learning_rates)))
        self.model_fitted = True
        return self

    def inducing_points(self):
        """The inducing points of a gp_approx = "fitc" model, (m, d) (GPB_GetInducingPoints)."""
        m = ctypes.c_int32(0)
        self._call(lib().GPB_GetInducingPoints(self.handle, ctypes.byref(m), None))
        out = np.zeros((m.value, self.dim_coords))
        self._call(lib().GPB_GetInducingPoints(self.handle, ctypes.byref(m), _dp(out)))
        return out

    def last_iteration_info(self):
        """[newton iterations, CG iterations, Lanczos steps, log|Sigma W + I|] of the last latent evaluation."""
        out = np.zeros(4)
        _safe_call(lib().GPB_GetLastIterationInfo(self.handle, _dp(out)))
        return out

    def cholesky_plan_info(self):
        """Statistics of the sparse Cholesky plan of a latent Vecchia model with matrix_inversion_method =
        "cholesky" (include/gpboost_amd.h GPB_GetCholeskyPlanInfo)."""
        out = np.zeros(9)
        _safe_call(lib().GPB_GetCholeskyPlanInfo(self.handle, _dp(out)))
        keys = ["supernodes", "levels", "nnz_L", "front_doubles", "factor_flops", "max_front", "max_supernode",
                "analyze_ms", "last_factor_ms"]
        return {k: float(v) for k, v in zip(keys, out)}

    def latent_vecchia_factor(self, cov_pars):
        cp = self._check_cov_pars(cov_pars)
        m = min(self.num_neighbors, self.num_data - 1)
        dinv, dd = np.zeros(self.num_data), np.zeros(self.num_data)
        b, db = np.zeros((self.num_data, m)), np.zeros((self.num_data, m))
        _safe_call(lib().GPB_GetLatentVecchiaFactor(self.handle, _dp(cp), _dp(dinv), _dp(b), _dp(dd), _dp(db)))
        return dict(Dinv=dinv, B=b, dD=dd, dB=db)

    def vecchia_partials(self, cov_pars, row_begin: int, row_end: int):
        cp = self._check_cov_pars(cov_pars)
        out = np.zeros(6)
        _safe_call(lib().GPB_EvalVecchiaPartials(self.handle, _dp(cp), ctypes.c_int32(row_begin),
                                                 ctypes.c_int32(row_end), _dp(out)))
        return out

    def vecchia_structure(self):
        perm = np.zeros(self.num_data, dtype=np.int32)
        m = min(self.num_neighbors, self.num_data - 1)
        nbr = np.zeros((self.num_data, m), dtype=np.int32)
        _safe_call(lib().GPB_GetVecchiaStructure(self.handle, _ip(perm), _ip(nbr)))
        return perm, nbr

    def vecchia_factor(self, cov_pars):
        cp = self._check_cov_pars(cov_pars)
        m = min(self.num_neighbors, self.num_data - 1)
        dinv = np.zeros(self.num_data)
        b = np.zeros((self.num_data, m))
        _safe_call(lib().GPB_GetVecchiaFactor(self.handle, _dp(cp), _dp(dinv), _dp(b)))
        return dinv, b

    def last_kernel_ms(self):
        out = np.zeros(2)
        _safe_call(lib().GPB_GetLastKernelTimes(self.handle, _dp(out)))
        return out

    def bench_latent_operators(self, t: int, reps: int = 20):
        """(ms per A application, ms per preconditioner application, nnz(B), launches per preconditioner application)."""
        out = np.zeros(4)
        _safe_call(lib().GPB_BenchLatentOperators(self.handle, ctypes.c_int(t), ctypes.c_int(reps), _dp(out)))
        return out

    def set_prediction_data(self, vecchia_pred_type=None, num_neighbors_pred=None, cg_delta_conv_pred=None,
                            nsim_var_pred=None, rank_pred_approx_matrix_lanczos=None, group_data_pred=None,
                            group_rand_coef_data_pred=None, gp_coords_pred=None, gp_rand_coef_data_pred=None,
                            cluster_ids_pred=None, X_pred=None):
        """Prediction settings and data (reference basic.py:6095-6190, GPB_SetPredictionData): the data is
        saved in the model for predict(use_saved_data=True) (gp_coords_pred / X_pred for GP models,
        group_data_pred for grouped random effects)."""
        if any(v is not None for v in (group_rand_coef_data_pred, gp_rand_coef_data_pred, cluster_ids_pred)):
            raise GPBoostError("set_prediction_data: random coefficients and clusters are not supported by gpboost_amd")
        num_data_pred = 0
        gbuf = xcol = xpc = None
        if group_data_pred is not None:
            g = np.asarray(group_data_pred)
            if g.ndim == 1:
                g = g.reshape(-1, 1)
            if g.shape[1] != getattr(self, "num_group_re", 0):
                raise ValueError("Number of grouped random effects in group_data_pred is not correct")
            num_data_pred = g.shape[0]
            labels = g.astype(np.dtype(str)).flatten(order="F")
            gbuf = ctypes.create_string_buffer(b"\0".join(s.encode() for s in labels) + b"\0")
        if gp_coords_pred is not None:
            xp = np.asarray(gp_coords_pred, dtype=np.float64)
            if xp.ndim == 1:
                xp = xp.reshape(-1, 1)
            if xp.shape[1] != self.dim_coords:
                raise ValueError("Incorrect dimension / number of coordinates (=features) in gp_coords_pred")
            if num_data_pred and xp.shape[0] != num_data_pred:
                raise ValueError("Incorrect number of data points in gp_coords_pred")
            num_data_pred = xp.shape[0]
            xcol = np.ascontiguousarray(xp.T.reshape(-1))
        if X_pred is not None:
            Xp = np.asarray(X_pred, dtype=np.float64)
            if Xp.ndim == 1:
                Xp = Xp.reshape(-1, 1)
            if num_data_pred and Xp.shape[0] != num_data_pred:
                raise ValueError("Incorrect number of data points in X_pred")
            num_data_pred = Xp.shape[0]
            xpc = np.ascontiguousarray(Xp.T).reshape(-1)
        _safe_call(lib().GPB_SetPredictionData(
            self.handle, ctypes.c_int32(num_data_pred), None, gbuf, None, _dp(xcol) if xcol is not None else None,
            None, _dp(xpc) if xpc is not None else None, c_str(vecchia_pred_type),
            ctypes.c_int(int(num_neighbors_pred) if num_neighbors_pred is not None else -1),
            ctypes.c_double(float(cg_delta_conv_pred) if cg_delta_conv_pred is not None else -1.),
            ctypes.c_int(int(nsim_var_pred) if nsim_var_pred is not None else -1),
            ctypes.c_int(int(rank_pred_approx_matrix_lanczos) if rank_pred_approx_matrix_lanczos is not None else -1)))
        if num_data_pred > 0:
            self.prediction_data_is_set = True
            self.num_data_pred = num_data_pred

    def predict(self, predict_response=True, predict_var=False, predict_cov_mat=False, y=None, cov_pars=None,
                group_data_pred=None, group_rand_coef_data_pred=None, gp_coords_pred=None,
                gp_rand_coef_data_pred=None, cluster_ids_pred=None, X_pred=None, use_saved_data=False, offset=None,
                offset_pred=None, fixed_effects=None, fixed_effects_pred=None, vecchia_pred_type=None,
                num_neighbors_pred=None):
        """Predictions at new coordinates (reference basic.py:5778-6093, GPB_PredictREModel): returns
        {"mu": mean, "cov": covariance or None, "var": variances or None}. Exact Gaussian Vecchia
        models (vecchia_pred_type "order_obs_first_cond_obs_only") and latent Vecchia models
        ("latent_order_obs_first_cond_obs_only": Laplace mode, simulated iterative variances,
        bernoulli_logit response probabilities by adaptive Gauss-Hermite quadrature)."""
        if use_saved_data:   # reference basic.py:6035-6038: the data saved by set_prediction_data
            if not getattr(self, "prediction_data_is_set", False):
                raise ValueError("No data has been set for making predictions. Call set_prediction_data first")
            return self._predict_saved(predict_var, predict_cov_mat, predict_response, y, cov_pars, offset,
                                       offset_pred, fixed_effects, fixed_effects_pred)
        if getattr(self, "num_group_re", 0):
            return self._predict_grouped(group_data_pred, predict_var, predict_cov_mat, predict_response, y, cov_pars,
                                         offset, offset_pred, fixed_effects, fixed_effects_pred, gp_coords_pred)
        if vecchia_pred_type is not None or num_neighbors_pred is not None:
            self.set_prediction_data(vecchia_pred_type=vecchia_pred_type, num_neighbors_pred=num_neighbors_pred)
        if any(v is not None for v in (group_data_pred, group_rand_coef_data_pred, gp_rand_coef_data_pred,
                                       cluster_ids_pred)):
            raise GPBoostError("predictions with grouped random effects, random coefficients or clusters are not "
                               "supported by gpboost_amd for GP models")
        xpc = None
        if X_pred is not None:
            Xp = np.asarray(X_pred, dtype=np.float64)
            if Xp.ndim == 1:
                Xp = Xp.reshape(-1, 1)
            xpc = np.ascontiguousarray(Xp.T).reshape(-1)
        if gp_coords_pred is None:
            raise ValueError("'gp_coords_pred' is missing")
        xp = np.asarray(gp_coords_pred, dtype=np.float64)
        if xp.ndim == 1:
            xp = xp.reshape(-1, 1)
        if xp.shape[1] != self.dim_coords:
            raise ValueError("Incorrect number of covariates (columns) in 'gp_coords_pred'")
        if not np.all(np.isfinite(xp)):
            raise ValueError("'gp_coords_pred' contains NaN or Inf")
        n_pred = xp.shape[0]
        xcol = np.ascontiguousarray(xp.T.reshape(-1))   # column-major, as the reference passes it
        yv = self._check_y(y)
        if offset is not None:
            fixed_effects = offset if fixed_effects is None else np.asarray(fixed_effects) + np.asarray(offset)
        if offset_pred is not None:
            fixed_effects_pred = offset_pred if fixed_effects_pred is None else (
                np.asarray(fixed_effects_pred) + np.asarray(offset_pred))
        fe = _as1d(fixed_effects, "fixed_effects") if fixed_effects is not None else None
        fep = _as1d(fixed_effects_pred, "fixed_effects_pred") if fixed_effects_pred is not None else None
        cp = self._check_cov_pars(cov_pars) if cov_pars is not None else None
        size = n_pred + (n_pred * n_pred if predict_cov_mat else (n_pred if predict_var else 0))
        out = np.zeros(size)
        _safe_call(lib().GPB_PredictREModel(
            self.handle, _dp(yv) if yv is not None else None, ctypes.c_int32(n_pred), _dp(out),
            ctypes.c_bool(bool(predict_cov_mat)), ctypes.c_bool(bool(predict_var)),
            ctypes.c_bool(bool(predict_response)), None, None, None, _dp(xcol), None,
            _dp(cp) if cp is not None else None, _dp(xpc) if xpc is not None else None, ctypes.c_bool(bool(use_saved_data)),
            _dp(fe) if fe is not None else None, _dp(fep) if fep is not None else None))
        mu = out[:n_pred].copy()
        cov = out[n_pred:].reshape(n_pred, n_pred).T.copy() if predict_cov_mat else None
        var = out[n_pred:].copy() if (predict_var and not predict_cov_mat) else None
        if predict_cov_mat and predict_var:
            var = np.diag(cov).copy()
        return {"mu": mu, "cov": cov, "var": var}

    def _predict_saved(self, predict_var, predict_cov_mat, predict_response, y, cov_pars, offset, offset_pred,
                       fixed_effects, fixed_effects_pred):
        """GPB_PredictREModel(use_saved_data = true): every data argument NULL, num_data_pred that of the
        saved data (re_model_template.h:3168-3206)."""
        n_pred = self.num_data_pred
        yv = self._check_y(y)
        if offset is not None:
            fixed_effects = offset if fixed_effects is None else np.asarray(fixed_effects) + np.asarray(offset)
        if offset_pred is not None:
            fixed_effects_pred = offset_pred if fixed_effects_pred is None else (
                np.asarray(fixed_effects_pred) + np.asarray(offset_pred))
        fe = _as1d(fixed_effects, "fixed_effects") if fixed_effects is not None else None
        fep = _as1d(fixed_effects_pred, "fixed_effects_pred") if fixed_effects_pred is not None else None
        cp = self._check_cov_pars(cov_pars) if cov_pars is not None else None
        size = n_pred + (n_pred * n_pred if predict_cov_mat else (n_pred if predict_var else 0))
        out = np.zeros(size)
        _safe_call(lib().GPB_PredictREModel(
            self.handle, _dp(yv) if yv is not None else None, ctypes.c_int32(n_pred), _dp(out),
            ctypes.c_bool(bool(predict_cov_mat)), ctypes.c_bool(bool(predict_var)),
            ctypes.c_bool(bool(predict_response)), None, None, None, None, None,
            _dp(cp) if cp is not None else None, None, ctypes.c_bool(True),
            _dp(fe) if fe is not None else None, _dp(fep) if fep is not None else None))
        mu = out[:n_pred].copy()
        cov = out[n_pred:].reshape(n_pred, n_pred).T.copy() if predict_cov_mat else None
        var = out[n_pred:].copy() if (predict_var and not predict_cov_mat) else None
        return {"mu": mu, "cov": cov, "var": var}

    def _predict_grouped(self, group_data_pred, predict_var, predict_cov_mat, predict_response, y, cov_pars, offset,
                         offset_pred, fixed_effects, fixed_effects_pred, gp_coords_pred=None):
        """Predictions of a grouped random effects model at new group labels (GPB_PredictREModel
        with re_group_data_pred): means = sum over the effects of the training posterior mean of the
        label's level (0 for a level not seen in training); with predict_var / predict_cov_mat
        (matrix_inversion_method = "cholesky") the predictive variances / covariance matrix."""
        if group_data_pred is None:
            raise ValueError("'group_data_pred' is missing")
        g = np.asarray(group_data_pred)
        if g.ndim == 1:
            g = g.reshape(-1, 1)
        if g.shape[1] != self.num_group_re:
            raise ValueError("Incorrect number of columns in 'group_data_pred'")
        n_pred = g.shape[0]
        labels = g.astype(np.dtype(str)).flatten(order="F")
        buf = ctypes.create_string_buffer(b"\0".join(s.encode() for s in labels) + b"\0")
        yv = self._check_y(y)
        if offset is not None:
            fixed_effects = offset if fixed_effects is None else np.asarray(fixed_effects) + np.asarray(offset)
        if offset_pred is not None:
            fixed_effects_pred = offset_pred if fixed_effects_pred is None else (
                np.asarray(fixed_effects_pred) + np.asarray(offset_pred))
        fe = _as1d(fixed_effects, "fixed_effects") if fixed_effects is not None else None
        fep = _as1d(fixed_effects_pred, "fixed_effects_pred") if fixed_effects_pred is not None else None
        cp = self._check_cov_pars(cov_pars) if cov_pars is not None else None
        xcol = None
        if gp_coords_pred is not None:
            xp = np.asarray(gp_coords_pred, dtype=np.float64)
            if xp.ndim == 1:
                xp = xp.reshape(-1, 1)
            if xp.shape[0] != n_pred:
                raise ValueError("'gp_coords_pred' and 'group_data_pred' have different numbers of rows")
            if xp.shape[1] != self.dim_coords:
                raise ValueError("'gp_coords_pred' must have %d columns (the dimension of 'gp_coords')" % self.dim_coords)
            xcol = np.ascontiguousarray(xp.T).reshape(-1)
        size = n_pred + (n_pred * n_pred if predict_cov_mat else (n_pred if predict_var else 0))
        out = np.zeros(size)
        _safe_call(lib().GPB_PredictREModel(
            self.handle, _dp(yv) if yv is not None else None, ctypes.c_int32(n_pred), _dp(out),
            ctypes.c_bool(bool(predict_cov_mat)), ctypes.c_bool(bool(predict_var)),
            ctypes.c_bool(bool(predict_response)), None, buf, None, _dp(xcol) if xcol is not None else None, None,
            _dp(cp) if cp is not None else None, None, ctypes.c_bool(False),
            _dp(fe) if fe is not None else None, _dp(fep) if fep is not None else None))
        mu = out[:n_pred].copy()
        cov = out[n_pred:].reshape(n_pred, n_pred).T.copy() if predict_cov_mat else None
        var = out[n_pred:].copy() if (predict_var and not predict_cov_mat) else None
        return {"mu": mu, "cov": cov, "var": var}

    def set_distributed(self, rank: int, world_size: int, comm_id: bytes | None):
        """Join an RCCL communicator (GPB_SetDistributed): exact Vecchia shards rows, latent
        Vecchia (iterative) shards the probe columns."""
        buf = ctypes.create_string_buffer(comm_id, len(comm_id)) if comm_id is not None else None
        _safe_call(lib().GPB_SetDistributed(self.handle, ctypes.c_int(rank), ctypes.c_int(world_size), buf))

    def set_distributed_host(self, rank: int, world_size: int, allreduce):
        """Same partition as set_distributed, with the cross-rank sums done by
        ``allreduce(x: np.ndarray)`` (in place, e.g. a gloo all-reduce) instead of RCCL
        (GPB_SetDistributedHostReduce): a test transport for several ranks on one GPU."""
        self._host_reduce_error = None

        def _cb(buf, count, _user):
            arr = np.ctypeslib.as_array(buf, shape=(count,))
            try:
                allreduce(arr)
            except BaseException as e:   # ctypes would print and drop it: record it and poison the sums
                if self._host_reduce_error is None:
                    self._host_reduce_error = e
                arr[:] = np.nan
        self._host_reduce = _HostReduceFn(_cb)   # keep the trampoline alive with the model
        _safe_call(lib().GPB_SetDistributedHostReduce(self.handle, ctypes.c_int(rank), ctypes.c_int(world_size),
                                                      self._host_reduce, None))


def comm_create_id() -> bytes:
    n = lib().GPB_CommIdSize()
    buf = ctypes.create_string_buffer(n)
    _safe_call(lib().GPB_CommCreateId(buf))
    return buf.raw


def partition_rows(num_data: int, world_size: int, rank: int):
    b = ctypes.c_int32(0)
    e = ctypes.c_int32(0)
    _safe_call(lib().GPB_PartitionRows(ctypes.c_int32(num_data), ctypes.c_int(world_size), ctypes.c_int(rank),
                                       ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


def combine_partials(sums, num_data: int, sigma2: float, profile_sigma2: bool):
    s = _as1d(sums, "sums")
    nll = np.zeros(1)
    grad = np.zeros(3)
    s2 = np.zeros(1)
    _safe_call(lib().GPB_CombinePartials(_dp(s), num_data, sigma2, int(bool(profile_sigma2)), _dp(nll), _dp(grad),
                                         _dp(s2)))
    return float(nll[0]), (grad[:2] if profile_sigma2 else grad).copy(), float(s2[0])
