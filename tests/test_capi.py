"""CPU: the C-ABI library loads, exports every symbol include/gpboost_amd.h declares,
host-side logic (row partition, partial-sum assembly) matches the oracle, and the
product fails loudly (no CPU fallback) when no GPU is visible."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gpboost_amd.h")


def _declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"GPBOOST_AMD_EXPORT\s+[\w\s\*]+?\b((?:GPB|LGBM)_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from gpboost_amd import basic
    if not os.path.exists(basic.LIB_PATH):
        from gpboost_amd import build
        build.build(verbose=False)
    return basic.lib()


def test_header_declares_reference_entry_points():
    syms = _declared_symbols()
    for s in ["GPB_CreateREModel", "GPB_REModelFree", "GPB_SetOptimConfig", "GPB_EvalNegLogLikelihood",
              "LGBM_GetLastError", "LGBM_RegisterLogCallback", "GPB_EvalNegLogLikelihoodGrad"]:
        assert s in syms


def _declared_arity():
    txt = open(HEADER).read()
    out = {}
    for m in re.finditer(r"GPBOOST_AMD_EXPORT\s+[\w\s\*]+?\b((?:GPB|LGBM)_\w+)\s*\(([^;]*?)\)\s*;", txt, re.S):
        args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = len(args)
    return out


def test_all_reference_entry_points_declared_and_exported(lib):
    """The drop-in boundary covers every GPB_* function of the reference C API
    (tests/golden/reference_c_api.json, recorded from include/LightGBM/c_api.h by
    tests/golden/make_capi_names.py) with the same parameter count."""
    import json
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_c_api.json")))["functions"]
    assert len(ref) == 29
    arity = _declared_arity()
    for f in ref:
        assert f["name"] in arity, f"{f['name']} (c_api.h:{f['line']}) not declared in include/gpboost_amd.h"
        assert arity[f["name"]] == f["nargs"], (f["name"], arity[f["name"]], f["nargs"])
        assert hasattr(lib, f["name"]), f"{f['name']} not exported"


def _declared_types():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_capi_names",
                                                  os.path.join(ROOT, "tests", "golden", "make_capi_names.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)   # defines param_type only (reads no reference file)
    txt = open(HEADER).read()
    out = {}
    for m in re.finditer(r"GPBOOST_AMD_EXPORT\s+([\w\s\*]+?)\b((?:GPB|LGBM)_\w+)\s*\(([^;]*?)\)\s*;", txt, re.S):
        args = [a for a in m.group(3).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(2)] = (m.group(1).strip(), [mod.param_type(a) for a in args])
    return out


def test_reference_entry_points_have_the_same_parameter_types():
    """Type-level ABI check: every GPB_* entry point returns int and takes the reference's parameter
    types in the reference's order (handles normalised to void*, as both headers typedef them)."""
    import json
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_c_api.json")))["functions"]
    decl = _declared_types()
    for f in ref:
        ret, types = decl[f["name"]]
        assert ret == "int", (f["name"], ret)
        assert types == f["types"], (f["name"], f"c_api.h:{f['line']}", types, f["types"])


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in _declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_partition_rows(lib):
    from gpboost_amd import partition_rows
    for n in [1, 7, 100, 100_003]:
        for w in [1, 2, 3, 8]:
            blocks = [partition_rows(n, w, r) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            for (a, b), (c, _) in zip(blocks, blocks[1:]):
                assert b == c and b >= a
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("profile", [False, True])
def test_combine_partials_matches_oracle(lib, synth2000, profile):
    from gpboost_amd import combine_partials
    from oracle import oracle as O
    X, Y = synth2000
    perm, xv, nb = O.vecchia_setup(X, 30, 0, True)
    tp = O.transform(0, [0.1, 1.0, 0.1])
    sums = O.vecchia_partials(xv, Y[perm], nb, 0, tp, 0, 2000)
    nll, g, s2 = combine_partials(sums, 2000, tp[0], profile)
    ref = O.vecchia_nll_grad(xv, Y[perm], nb, 0, tp, int(profile))
    assert abs(nll - ref["nll"]) <= 1e-12 * abs(ref["nll"])
    np.testing.assert_allclose(g, ref["grad"], rtol=1e-12)


def test_error_convention(lib):
    """-1 + LGBM_GetLastError message, never a crash (reference c_api.cpp:54-58)."""
    from gpboost_amd import GPBoostError, GPModel
    with pytest.raises((GPBoostError, ValueError)):
        GPModel(gp_coords=np.zeros((10, 2)), cov_function="wendland", gp_approx="vecchia")


def test_no_cpu_fallback_without_gpu(lib):
    import os
    import torch
    if torch.cuda.is_available() or os.path.exists("/dev/kfd"):   # a GPU box (torch may not see the card)
        pytest.skip("GPU visible")
    from gpboost_amd import GPBoostError, GPModel
    with pytest.raises(GPBoostError, match="no HIP device"):
        GPModel(gp_coords=np.random.rand(50, 2), cov_function="exponential", gp_approx="vecchia", num_neighbors=5)
