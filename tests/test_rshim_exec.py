"""Executes the R boundary (rshim/sparseRGPs_sgp.c) on a mock R runtime (tests/r_api/mock_rt.c).

R is absent from this image, so the shim runs against a small executable
stand-in for the R C API it uses: SEXPs with type/length/dim/names, R's coercions (logical NA
of matrix() -> NaN), Rf_error as a longjmp back to the .Call frame, a PROTECT stack that is
checked for balance after every routine, captured REprintf output, registration through the
shim's own R_init_sparseRGPs, and external-pointer finalizers.  Every routine is called by its
registered name with the registered arity, as R's .Call does.

CPU: the registry, the transforms, every per-pair routine (sgp_kernel_pair / sgp_dkernel_pair
are host code) against the oracle's closed forms, and every error / 0x0 path of the fillers
(reference behaviour: src/covariance_functionsC.cpp:161-168,
src/covariance_function_derivativesC.cpp:420, 520, 545-551), none of which touches a GPU.
GPU: the four matrix fillers against tests/golden/fills.npz (1e-12) and the fused routines
(sgp_R_eval / _eval_laplace / _predict / _posterior_u / _knot_gradient / _candidates /
_eval_full / contexts) against the golden fixtures and the oracle (1e-6, the north-star bar).
"""
import json
import math
import os
import shutil

import numpy as np
import pytest

from oracle import sgp_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
SGP = os.path.join(ROOT, "sparsergps_amd", "lib", "libsgp.so")


@pytest.fixture(scope="module")
def R():
    from r_api import mockr
    if not os.path.exists(SGP):
        pytest.skip("libsgp.so not built")
    if not os.path.exists(mockr.LIB) and shutil.which("gcc") is None:
        pytest.skip("gcc not available to build the mock runtime")
    mockr.build()
    r = mockr.MockR()
    yield r
    r.reset()


_GPU_DONE = []


def _err(R, name, *args):
    from r_api.mockr import RError
    with pytest.raises(RError) as e:
        R.call(name, *args)
    return str(e.value)


# ------------------------------------------------------------------------------ CPU
def test_registration(R):
    fix = json.load(open(os.path.join(GOLD, "rcpp_registry.json")))
    assert R.n_routines == 37          # 20 reference routines + 17 fused
    assert [tuple(e) for e in R.routines[:20]] == [tuple(e) for e in fix["call_entries"]]
    assert R.L.mock_dynamic_symbols() == 0             # R_useDynamicSymbols(dll, FALSE)


def test_transforms(R):
    x = np.array([-1.5, 0.0, 2.25])
    np.testing.assert_allclose(R.call("_sparseRGPs_real_to_pos", x).py(), np.exp(x), rtol=1e-15)
    np.testing.assert_allclose(R.call("_sparseRGPs_pos_to_real", np.exp(x)).py(), x,
                               rtol=1e-15, atol=1e-15)
    np.testing.assert_allclose(R.call("_sparseRGPs_real_to_pos", R.int_([1, 2])).py(),
                               np.exp([1.0, 2.0]), rtol=1e-15)
    ub, lb = np.array([4.0, 5.0, 6.0]), np.array([-1.0, 0.0, 1.0])
    got = R.call("_sparseRGPs_real_to_bounded", x, ub, lb).py()
    np.testing.assert_allclose(got, (ub * np.exp(x) + lb) / (np.exp(x) + 1), rtol=1e-15)
    # Rcpp sugar: the result has length(ub); no recycling of shorter operands
    assert R.call("_sparseRGPs_real_to_bounded", x, ub[:2], lb).py().shape == (2,)
    assert "length(ub)" in _err(R, "_sparseRGPs_real_to_bounded", x, ub, lb[:2])


CP = {"sigma": 1.3, "l": 1.7, "tau": 0.4}
CPA = {"sigma": 0.9, "l1": 0.8, "l2": 1.5, "l3": 2.2, "tau": 0.3}
LN = ["l1", "l2", "l3"]
X1, X2 = np.array([0.3, 1.9, -0.7]), np.array([1.1, 0.4, 0.2])


def _o_pair(fun, a, b, cp, *extra):
    return fun(a[None, :], b[None, :], cp, *extra)[0, 0]


def test_pair_kernels(R):
    for kname, f in (("_sparseRGPs_cov_fun_sqrd_expC", "sqexp"), ("_sparseRGPs_cov_fun_expC", "exp")):
        got = R.call(kname, X1, X2, CP).py()
        assert got.shape == (1,)
        ref = _o_pair(O.make_cov_matC, X1, X2, CP, f, 0.0)
        assert abs(got[0] - ref) <= 1e-14 * abs(ref)
    got = R.call("_sparseRGPs_cov_fun_sqrd_exp_ardC", X1, X2, CPA, LN).py()[0]
    ref = _o_pair(O.make_cov_mat_ardC, X1, X2, CPA, "ard", 0.0, LN)
    assert abs(got - ref) <= 1e-14 * abs(ref)


@pytest.mark.parametrize("x2", [X2, X1], ids=["distinct", "coincident"])
def test_pair_derivatives(R, x2):
    cases = [("_sparseRGPs_dsqexp_dsigmaC", "sqexp", "sigma", ()),
             ("_sparseRGPs_dsqexp_dlC", "sqexp", "l", ()),
             ("_sparseRGPs_dsqexp_dtauC", "sqexp", "tau", ()),
             ("_sparseRGPs_dexp_dsigmaC", "exp", "sigma", ()),   # L2 distance (Q12)
             ("_sparseRGPs_dexp_dlC", "exp", "l", ()),
             ("_sparseRGPs_dexp_dtauC", "exp", "tau", ())]
    for name, f, p, _ in cases:
        out = R.call(name, X1, x2, CP).py()
        assert list(out) == ["derivative", "trans_par", "inv_trans_par"]
        ref = _o_pair(O.dsig_dthetaC, X1, x2, CP, f, p) if (p != "tau" or f == "sqexp") else \
            (2 * CP["tau"] ** 2 if np.array_equal(X1, x2) else 0.0)
        assert abs(out["derivative"][0] - ref) <= 1e-14 * max(abs(ref), 1e-300), (name, out, ref)
        assert out["trans_par"][0] == pytest.approx(math.log(CP[p]), rel=1e-15)
        assert out["inv_trans_par"][0] == pytest.approx(math.exp(CP[p]), rel=1e-15)
    # d*_dtauC read only cov_par$tau (covariance_function_derivativesC.cpp:148)
    only_tau = R.call("_sparseRGPs_dsqexp_dtauC", X1, x2, {"tau": 0.4}).py()["derivative"][0]
    assert only_tau == (2 * 0.4 ** 2 if np.array_equal(X1, x2) else 0.0)
    out = R.call("_sparseRGPs_dsqexp_dsigma_ardC", X1, x2, CPA, LN).py()
    ref = _o_pair(O.dsig_dtheta_ardC, X1, x2, CPA, "ard", "sigma", LN)
    assert abs(out["derivative"][0] - ref) <= 1e-14 * abs(ref)
    for comp in (1, 2, 3):
        out = R.call("_sparseRGPs_dsqexp_dl_ardC", X1, x2, CPA, LN, float(comp)).py()
        ref = _o_pair(O.dsig_dtheta_ardC, X1, x2, CPA, "ard", f"l{comp}", LN)
        assert abs(out["derivative"][0] - ref) <= 1e-14 * max(abs(ref), 1e-300)
        assert out["trans_par"][0] == pytest.approx(math.log(CPA[f"l{comp}"]), rel=1e-15)
    assert "comp 4" in _err(R, "_sparseRGPs_dsqexp_dl_ardC", X1, x2, CPA, LN, 4.0)


def test_knot_derivatives(R):
    lb, ub = np.array([-2.0, -1.0, -3.0]), np.array([3.0, 4.0, 2.0])
    for name, cp, extra in (("_sparseRGPs_dsqexp_dx2C", CP, ()),
                            ("_sparseRGPs_dsqexp_dx2_ardC", CPA, (LN,))):
        out = R.call(name, X1, X2, cp, lb, ub, *extra).py()
        l = np.array([cp["l"]] * 3) if "l" in cp else np.array([cp[k] for k in LN])
        k = cp["sigma"] ** 2 * math.exp(-np.sum(((X1 - X2) / l) ** 2) / 2)
        t = np.log((X2 - lb) / (ub - X2))
        dxdt = np.exp(t) * (ub - lb) / (np.exp(t) + 1) ** 2
        np.testing.assert_allclose(out["derivative"], (X1 - X2) / l ** 2 * k * dxdt, rtol=1e-14)
        np.testing.assert_allclose(out["trans_par"], t, rtol=1e-14)
        np.testing.assert_allclose(out["inv_trans_par"], (ub * np.exp(X2) + lb) / (np.exp(X2) + 1),
                                   rtol=1e-14)
        assert "at least 3" in _err(R, name, X1, X2, cp, lb[:2], ub, *extra)


def test_filler_messages_and_errors_without_device(R):
    x = np.arange(12, dtype=float).reshape(4, 3) / 3
    xp = x[:2] + 0.5
    na = R.na_matrix()
    # invalid covariance function: Rcerr message + 0x0 (covariance_functionsC.cpp:161-168)
    for args in (("_sparseRGPs_make_cov_matC", x, na, CP, "bogus", 1e-6),
                 ("_sparseRGPs_make_cov_mat_ardC", x, na, CPA, "sqexp", 1e-6, LN),
                 ("_sparseRGPs_dsig_dthetaC", x, na, CP, "bogus", "sigma"),
                 ("_sparseRGPs_dsig_dtheta_ardC", x, xp, CPA, "exp", "sigma", LN)):
        out = R.call(*args)
        assert out.dim == (0, 0) and R.eprint == "Error: invalid covariance function", args
    # unknown parameter names (covariance_function_derivativesC.cpp:420, 545-551)
    assert R.call("_sparseRGPs_dsig_dthetaC", x, xp, CP, "sqexp", "bogus").dim == (0, 0)
    assert R.eprint == "Error: invalid parameter name for chosen covariance function"
    assert R.call("_sparseRGPs_dsig_dthetaC", x, na, CP, "sqexp", "bogus").dim == (0, 0)
    assert R.eprint == "Error: invalid covariance function"
    assert R.call("_sparseRGPs_dsig_dthetaC", x, na, CP, "exp", "bogus").dim == (0, 0)
    assert R.eprint == "Error"
    assert R.call("_sparseRGPs_dsig_dtheta_ardC", x, xp, CPA, "ard", "l9", LN).dim == (0, 0)
    assert R.eprint == "Error: invalid parameter name for chosen covariance function"
    # exp cross mode, tau (and unknown names): a zero n x n' matrix (quirk Q13, l.520)
    for p in ("tau", "bogus"):
        z = R.call("_sparseRGPs_dsig_dthetaC", x, xp, CP, "exp", p).py()
        assert z.shape == (4, 2) and not z.any() and R.eprint == ""
    # a missing cov_par name is Rcpp's index error, raised before any device work
    for args in (("_sparseRGPs_make_cov_matC", x, na, {"sigma": 1.0, "tau": 0.1}, "sqexp", 1e-6),
                 ("_sparseRGPs_cov_fun_sqrd_expC", X1, X2, {"sigma": 1.0}),
                 ("_sparseRGPs_dsig_dtheta_ardC", x, xp, {"sigma": 1.0, "l1": 1.0}, "ard",
                  "sigma", LN)):
        assert _err(R, *args).startswith("Index out of bounds: [index='l")
    assert "no elements" in _err(R, "_sparseRGPs_make_cov_matC", x, np.zeros(0), CP, "sqexp", 0.0)
    assert "differ in length" in _err(R, "_sparseRGPs_cov_fun_sqrd_expC", X1, X2[:2], CP)
    # the fused routines reject anything that is not a context
    assert "not an sgp context" in _err(R, "sgp_R_eval", 1.0, 0.0, "sqexp", [1.0, 1.0, 0.5],
                                        x, 1e-6, 0.0)
    # visible devices (0 here: no GPU), and the multi-device context's device list is checked
    # before any device call
    from sparsergps_amd import _lib
    n = _lib.C.c_int(0)
    if _lib.lib().sgp_device_count(_lib.C.byref(n)) != 0 or n.value == 0:
        assert R.call("sgp_R_device_count").py()[0] == 0
    y4 = np.zeros(4)
    assert "non-negative integers" in _err(R, "sgp_R_ctx_create", x, y4, y4, 8.0, [0.0, -1.0])
    assert "non-negative integers" in _err(R, "sgp_R_ctx_create", x, y4, y4, 8.0, [0.5])
    assert "at most 64" in _err(R, "sgp_R_ctx_create", x, y4, y4, 8.0, [0.0] * 65)


def test_every_host_routine_ran(R):
    """After the CPU tests above every host-only routine (transforms, per-pair kernels and
    derivatives) has been called through mock_call."""
    host = [n for n, _ in R.routines
            if not (n.startswith("sgp_R_") or "cov_mat" in n or "dsig_" in n)]
    assert len(host) == 16
    if not {"_sparseRGPs_real_to_pos", "_sparseRGPs_dsqexp_dx2C",
            "_sparseRGPs_dsqexp_dl_ardC"} <= R.called:
        pytest.skip("only a subset of this module's CPU tests ran")
    missing = [n for n in host if n not in R.called]
    assert not missing, missing


# ------------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def gR(R):
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return R


@pytest.mark.gpu
def test_fills_match_golden(gR):
    R = gR
    z = np.load(os.path.join(GOLD, "fills.npz"))
    x, xp = z["x"], z["xp"]
    checked = 0
    for key in z.files:
        if key in ("x", "xp"):
            continue
        parts = key.split("_")
        mode = parts[-1]
        xpred = R.na_matrix() if mode == "sym" else xp
        f = parts[1]
        if parts[0] == "cov":
            out = (R.call("_sparseRGPs_make_cov_mat_ardC", x, xpred, CPA, "ard", 1e-6, LN)
                   if f == "ard" else
                   R.call("_sparseRGPs_make_cov_matC", x, xpred, CP, f, 1e-6))
        else:
            p = parts[2]
            out = (R.call("_sparseRGPs_dsig_dtheta_ardC", x, xpred, CPA, "ard", p, LN)
                   if f == "ard" else
                   R.call("_sparseRGPs_dsig_dthetaC", x, xpred, CP, f, p))
        got = out.py()
        np.testing.assert_allclose(got, z[key], rtol=1e-12, atol=1e-300, err_msg=key)
        checked += 1
    assert checked == 28
    _GPU_DONE.append("test_fills_match_golden")


@pytest.mark.gpu
def test_vi_fitc_routines(gR):
    R = gR
    z = np.load(os.path.join(GOLD, "gauss_c3_small.npz"))
    X, U, y, mu, th = z["X"], z["U"], z["y"], z["mu"], z["theta"]
    cf, delta, m, d = str(z["cov_fun"]), float(z["delta"]), z["U"].shape[0], X.shape[1]
    cp = dict(zip([str(s) for s in z["names"]], th))
    ctx = R.call("sgp_R_ctx_create", X, y, mu, float(m + 1), None)
    for meth, key in ((0, "vi"), (1, "fitc")):
        out = R.call("sgp_R_eval", ctx, float(meth), cf, th, U, delta, 0.0).py()
        assert abs(out["objective"][0] - z[f"{key}_obj"]) <= 1e-6 * abs(z[f"{key}_obj"])
        np.testing.assert_allclose(out["gradient"], z[f"{key}_grad"], rtol=1e-6, atol=1e-8)
        obj_only = R.call("sgp_R_eval", ctx, float(meth), cf, th, U, delta, 2.0).py()["objective"]
        r_det = R.call("sgp_R_eval", ctx, float(meth), cf, th, U, delta, 1.0).py()["objective"]
        assert obj_only[0] == pytest.approx(out["objective"][0], rel=1e-12)
        assert r_det[0] == pytest.approx(out["objective"][0], rel=1e-9)
    # knot posterior after a VI evaluation (vi_functions.R:1161-1180)
    R.call("sgp_R_eval", ctx, 0.0, cf, th, U, delta, 0.0)
    muu = np.full(m, 0.1)
    post = R.call("sgp_R_posterior_u", ctx, muu).py()
    um, uv = O.vi_posterior_u(cp, cf, U, X, y, mu, muu, delta)
    np.testing.assert_allclose(post["u_mean"], um, rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(post["u_var"], uv, rtol=1e-6, atol=1e-8)
    # knot gradient (xu_opt = "simultaneous"), row-major, reference factor and bounds
    R.call("sgp_R_enable_knot_grad", ctx, R.lgl(True))
    R.call("sgp_R_eval", ctx, 0.0, cf, th, U, delta, 0.0)
    kg = R.call("sgp_R_knot_gradient", ctx, None, float(m), float(d)).py()
    ref = O.delbo_dcov_par(cp, cf, U, X, y, mu, delta, dcov_fun_dknot=cf)["knot_gradient"]
    np.testing.assert_allclose(kg, np.asarray(ref), rtol=1e-6, atol=1e-8)
    R.call("sgp_R_enable_knot_grad", ctx, R.lgl(False))
    # OAT candidate scoring: ELBO at [U; cand_t] per candidate
    cand = np.random.default_rng(3).uniform(0, 10, (3, d))
    sc = R.call("sgp_R_candidates", ctx, 0.0, cf, th, U, delta, cand, 1.0, 1e-5, 10.0).py()
    for t in range(3):
        ref = O.elbo_eval(cp, cf, np.vstack([U, cand[t]]), X, y, mu, delta)
        assert abs(sc[t] - ref) <= 1e-6 * abs(ref)
    # new y / mu on the same rows
    y2 = y[::-1].copy()
    R.call("sgp_R_set_data", ctx, y2, mu)
    o2 = R.call("sgp_R_eval", ctx, 0.0, cf, th, U, delta, 2.0).py()["objective"][0]
    assert abs(o2 - O.elbo_eval(cp, cf, U, X, y2, mu, delta)) <= 1e-6 * abs(o2)
    assert "one value per context row" in _err(R, "sgp_R_set_data", ctx, y2[:5], mu)
    # explicit destroy, then a use is an R error; the finalizer does not run twice
    R.call("sgp_R_ctx_destroy", ctx)
    _GPU_DONE.append("test_full_gp_routine")
    assert "already destroyed" in _err(R, "sgp_R_eval", ctx, 0.0, cf, th, U, delta, 0.0)
    _GPU_DONE.append("test_vi_fitc_routines")


@pytest.mark.gpu
def test_laplace_routines(gR):
    R = gR
    z = np.load(os.path.join(GOLD, "poisson_c5_small.npz"))
    X, U, y, mu, th = z["X"], z["U"], z["y"], z["mu"], z["theta"]
    delta, a, m = float(z["delta"]), float(z["a"]), U.shape[0]
    ctx = R.call("sgp_R_ctx_create", X, y, mu, float(m + 1), None)
    R.call("sgp_R_lap_set_f", ctx, z["f0"])
    out = R.call("sgp_R_eval_laplace", ctx, "sqexp", th, U, delta, a, 1e-5, 1000.0,
                 R.lgl(True)).py()
    tr = z["obj_trace"]
    assert out["nr_iter"][0] == len(tr)
    assert abs(out["objective"][0] - tr[-1]) <= 1e-9 * abs(tr[-1])
    np.testing.assert_allclose(out["gradient"], z["grad"], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(R.call("sgp_R_lap_objective_values", ctx).py(), tr, rtol=1e-9)
    np.testing.assert_allclose(R.call("sgp_R_lap_get_f", ctx).py(), z["ff"], rtol=1e-7, atol=1e-9)
    # NR alone (want_grad = FALSE) from a scalar start value; no grad psi before an NR step
    R.call("sgp_R_lap_set_f", ctx, float(z["f0"][0]))
    assert "no Newton-Raphson step" in _err(R, "sgp_R_lap_get_grad_psi", ctx)
    nr = R.call("sgp_R_eval_laplace", ctx, "sqexp", th, U, delta, a, 1e-5, 1000.0,
                R.lgl(False)).py()
    assert abs(nr["objective"][0] - tr[-1]) <= 1e-8 * abs(tr[-1])
    # newtrap_sparseGP's `gradient`: grad psi of the last NR step, against the oracle's loop
    nr_ref = O.newtrap_sparseGP(z["f0"], dict(zip([str(s) for s in z["names"]], th)), "sqexp",
                                X, U, y, mu, a, delta, tol=1e-5)
    gp = R.call("sgp_R_lap_get_grad_psi", ctx).py()
    assert gp.shape == (X.shape[0],)
    assert np.max(np.abs(gp - nr_ref["gradient"])) < 1e-8
    assert "length 1 or one value" in _err(R, "sgp_R_lap_set_f", ctx, z["f0"][:3])
    # Poisson OAT candidate scoring: newtrap at [U; cand_t] from the resident mode
    cand = np.random.default_rng(4).uniform(0, 10, (2, X.shape[1]))
    sc = R.call("sgp_R_candidates", ctx, 2.0, "sqexp", th, U, delta, cand, a, 1e-5, 1000.0).py()
    cp = dict(zip([str(s) for s in z["names"]], th))
    ff = R.call("sgp_R_lap_get_f", ctx).py()
    for t in range(2):
        ref = O.newtrap_sparseGP(ff, cp, "sqexp", X, np.vstack([U, cand[t]]), y, mu, a,
                                 delta, tol=1e-5)["objective_function_values"][-1]
        assert abs(sc[t] - ref) <= 1e-6 * abs(ref)
    assert R.gc() >= 1                          # the context's finalizer runs at gc
    _GPU_DONE.append("test_laplace_routines")


@pytest.mark.gpu
@pytest.mark.parametrize("full_cov", [False, True])
def test_predict_routine(gR, full_cov):
    R = gR
    rng = np.random.default_rng(12)
    U = rng.uniform(0, 10, (9, 2))
    xp = rng.uniform(0, 10, (6, 2))
    cp = {"sigma": 1.2, "l": 2.0, "tau": 0.3}
    th = np.array([1.2, 2.0, 0.3])
    um, muu = rng.normal(size=9), np.full(9, 0.2)
    A = rng.normal(size=(9, 9))
    uv = A @ A.T / 9 + 0.1 * np.eye(9)
    mp = np.full(6, 0.5)
    out = R.call("sgp_R_predict", 0.0, R.lgl(True), "sqexp", th, 1e-6, U, um, muu, uv, xp, mp,
                 R.lgl(full_cov)).py()
    ref = O.predict_vi(um, uv, U, xp, "sqexp", cp, mp, muu, full_cov)
    np.testing.assert_allclose(out["pred_mean"], ref["pred_mean"], rtol=1e-9, atol=1e-10)
    np.testing.assert_allclose(out["pred_var"], ref["pred_var"], rtol=1e-9, atol=1e-10)
    out = R.call("sgp_R_predict", 1.0, R.lgl(False), "sqexp", th, 1e-6, U, um, muu, uv, xp, mp,
                 R.lgl(full_cov)).py()
    ref = O.predict_laplace(um, uv, U, xp, "sqexp", cp, mp, muu, full_cov, family="poisson")
    np.testing.assert_allclose(out["pred_mean"], ref["pred_mean"], rtol=1e-9, atol=1e-10)
    np.testing.assert_allclose(out["pred_var"], ref["pred_var"], rtol=1e-9, atol=1e-10)
    _GPU_DONE.append("test_predict_routine")


@pytest.mark.gpu
def test_full_gp_routine(gR):
    R = gR
    rng = np.random.default_rng(13)
    X = rng.uniform(0, 10, (120, 3))
    y = np.sin(X).sum(1) + rng.normal(0, 0.3, 120)
    mu = np.full(120, y.mean())
    cp = {"sigma": 1.1, "l": 1.6, "tau": 0.4}
    ctx = R.call("sgp_R_ctx_create", X, y, mu, 120.0, None)
    out = R.call("sgp_R_eval_full", ctx, "sqexp", [1.1, 1.6, 0.4], 1e-6, 0.0).py()
    ro = O.full_obj_eval(cp, "sqexp", X, y, mu)
    rg = O.dlogp_dcov_par_full(cp, "sqexp", X, y, mu)["gradient"]
    assert abs(out["objective"][0] - ro) <= 1e-6 * abs(ro)
    np.testing.assert_allclose(out["gradient"], [rg[k] for k in cp], rtol=1e-6, atol=1e-8)
    R.call("sgp_R_ctx_destroy", ctx)


@pytest.mark.gpu
def test_multi_device_context_routines(gR):
    """An R process on the multi-device path (sgp_hotpath.R's .sgp_devices -> sgp_R_ctx_create
    with one device index per row shard -> sgp_ctx_create_multi, RCCL inside libsgp): three
    shards on device 0 give the one-device answers through the same .Call routines, VI, FITC
    and Poisson Laplace."""
    R = gR
    assert R.call("sgp_R_device_count").py()[0] >= 1
    z = np.load(os.path.join(GOLD, "gauss_c3_small.npz"))
    X, U, y, mu, th = z["X"], z["U"], z["y"], z["mu"], z["theta"]
    cf, delta, m = str(z["cov_fun"]), float(z["delta"]), z["U"].shape[0]
    one = R.call("sgp_R_ctx_create", X, y, mu, float(m + 1), None)
    multi = R.call("sgp_R_ctx_create", X, y, mu, float(m + 1), [0.0, 0.0, 0.0])
    assert list(R.call("sgp_R_ctx_shards", multi).py()) == [3.0, 1.0]
    assert list(R.call("sgp_R_ctx_shards", one).py()) == [1.0, 1.0]
    for meth, key in ((0, "vi"), (1, "fitc")):
        a = R.call("sgp_R_eval", multi, float(meth), cf, th, U, delta, 0.0).py()
        b = R.call("sgp_R_eval", one, float(meth), cf, th, U, delta, 0.0).py()
        assert abs(a["objective"][0] - b["objective"][0]) <= 1e-11 * abs(b["objective"][0])
        np.testing.assert_allclose(a["gradient"], b["gradient"], rtol=1e-10, atol=1e-10)
        assert abs(a["objective"][0] - z[f"{key}_obj"]) <= 1e-9 * abs(z[f"{key}_obj"])
    R.call("sgp_R_ctx_destroy", multi)
    R.call("sgp_R_ctx_destroy", one)
    z = np.load(os.path.join(GOLD, "poisson_c5_small.npz"))
    X, U, y, mu, th = z["X"], z["U"], z["y"], z["mu"], z["theta"]
    delta, a, m = float(z["delta"]), float(z["a"]), U.shape[0]
    multi = R.call("sgp_R_ctx_create", X, y, mu, float(m + 1), [0.0, 0.0])
    R.call("sgp_R_lap_set_f", multi, z["f0"])
    out = R.call("sgp_R_eval_laplace", multi, "sqexp", th, U, delta, a, 1e-5, 1000.0,
                 R.lgl(True)).py()
    tr = z["obj_trace"]
    assert out["nr_iter"][0] == len(tr)
    np.testing.assert_allclose(R.call("sgp_R_lap_objective_values", multi).py(), tr, rtol=1e-9)
    np.testing.assert_allclose(R.call("sgp_R_lap_get_f", multi).py(), z["ff"], rtol=1e-7,
                               atol=1e-9)
    np.testing.assert_allclose(out["gradient"], z["grad"], rtol=1e-7, atol=1e-8)
    R.call("sgp_R_ctx_destroy", multi)
    # a per-row exposure `m` (R/derivative_functions_of_data_likelihoods.R:38, a vector of cell
    # areas) through the same routine: one context and three shards against the frozen oracle
    z = np.load(os.path.join(GOLD, "poisson_c5_expo.npz"))
    X, U, y, mu, th, av = z["X"], z["U"], z["y"], z["mu"], z["theta"], z["a"]
    delta, m = float(z["delta"]), U.shape[0]
    tr = z["obj_trace"]
    for dv in (None, [0.0, 0.0, 0.0]):
        c = R.call("sgp_R_ctx_create", X, y, mu, float(m + 1), dv)
        R.call("sgp_R_lap_set_f", c, z["f0"])
        out = R.call("sgp_R_eval_laplace", c, "sqexp", th, U, delta, av, 1e-5, 1000.0,
                     R.lgl(True)).py()
        assert out["nr_iter"][0] == len(tr), dv
        np.testing.assert_allclose(R.call("sgp_R_lap_objective_values", c).py(), tr, rtol=1e-9)
        np.testing.assert_allclose(out["gradient"], z["grad"], rtol=1e-7, atol=1e-8)
        assert "length 1 or one value per row" in _err(R, "sgp_R_eval_laplace", c, "sqexp", th,
                                                      U, delta, av[:7], 1e-5, 1000.0,
                                                      R.lgl(True))
        bad = av.copy()
        bad[3] = -1.0
        assert "a[3]" in _err(R, "sgp_R_eval_laplace", c, "sqexp", th, U, delta, bad, 1e-5,
                              1000.0, R.lgl(True))
        R.call("sgp_R_ctx_destroy", c)
    _GPU_DONE.append("test_multi_device_context_routines")


@pytest.mark.gpu
def test_every_device_routine_ran(gR):
    """Runs last in this module (pytest keeps file order): after the GPU tests above every
    registered routine that needs the device -- the four matrix fillers and the 15 fused
    routines -- has been called through mock_call (the 16 host-only per-pair / transform
    routines are covered by test_every_host_routine_ran on the CPU)."""
    if len(_GPU_DONE) < 5:
        pytest.skip("only a subset of this module's GPU tests ran")
    dev = [n for n, _ in gR.routines if n.startswith("sgp_R_") or "cov_mat" in n or "dsig_" in n]
    assert len(dev) == 21
    missing = [n for n in dev if n not in gR.called]
    assert not missing, missing
