"""Pin the CPU oracle (oracle/sgp_oracle.py) before trusting it as the parity checker.

The reference has no tests, golden vectors or runnable build here, so the
restatement is pinned independently:
  * closed forms of the per-pair kernels/derivatives (covariance_functionsC.cpp:5-52,
    covariance_function_derivativesC.cpp:35-171);
  * dense n x n formulations of the objectives (slogdet of Sigma_y) vs the Woodbury forms;
  * central finite differences of the objectives in log(theta) vs the analytic gradients
    (the reference's own commented FD checks, covariance_function_derivatives.R:156-173);
  * the committed golden fixtures (tests/golden/make_golden.py) for regression;
  * the adjoint (S, t, G) protocol of libsgp (oracle/adjoint_ref.py) against the literal path.
"""
import math
import os
from collections import OrderedDict

import numpy as np
import pytest

from oracle import sgp_oracle as O
from oracle import adjoint_ref as A

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def fd_grad(fun, cp, h=1e-5):
    g = OrderedDict()
    for k in cp:
        a, b = OrderedDict(cp), OrderedDict(cp)
        a[k] = cp[k] * math.exp(h)
        b[k] = cp[k] * math.exp(-h)
        g[k] = (fun(a) - fun(b)) / (2 * h)
    return g


# ----------------------------------------------------------------------- closed forms
def test_pair_closed_forms():
    x1, x2 = np.array([[0.0, 1.0]]), np.array([[2.0, -1.0]])
    cp = {"sigma": 2.0, "l": 0.5, "tau": 0.3}
    d2 = 8.0
    assert np.isclose(O.make_cov_matC(x1, x2, cp, "sqexp", 0)[0, 0], 4 * math.exp(-d2 / (2 * 0.25)))
    assert np.isclose(O.make_cov_matC(x1, x2, cp, "exp", 0)[0, 0], 4 * math.exp(-4.0 / 0.5))   # L1 (Q12)
    assert np.isclose(O.dsig_dthetaC(x1, x2, cp, "sqexp", "sigma")[0, 0], 2 * 4 * math.exp(-16))
    assert np.isclose(O.dsig_dthetaC(x1, x2, cp, "sqexp", "l")[0, 0], 4 * math.exp(-16) * d2 / 0.25)
    assert np.isclose(O.dsig_dthetaC(x1, x2, cp, "exp", "sigma")[0, 0],
                      2 * 4 * math.exp(-math.sqrt(d2) / 0.5))                                     # L2 (Q12)
    sym = O.make_cov_matC(np.vstack([x1, x2]), None, cp, "sqexp", 1e-6)
    assert np.isclose(sym[0, 0], 4 + 0.09 + 1e-6) and np.isclose(sym[1, 0], sym[0, 1])


def test_tau_coincidence_rule():
    x = np.array([[1.0, 2.0], [3.0, 4.0]])
    xp = np.array([[3.0, 4.0], [1.0, 2.5]])
    cp = {"sigma": 1.0, "l": 1.0, "tau": 0.5}
    d = O.dsig_dthetaC(x, xp, cp, "sqexp", "tau")
    assert np.array_equal(d, np.array([[0.0, 0.0], [0.5, 0.0]]))
    assert not O.dsig_dthetaC(x, xp, cp, "exp", "tau").any()                 # Q13
    assert np.array_equal(np.diag(O.dsig_dthetaC(x, None, cp, "exp", "tau")), [0.5, 0.5])
    assert O.dsig_dthetaC(x, None, cp, "sqexp", "bogus").shape == (0, 0)
    assert O.make_cov_matC(x, None, cp, "bogus", 1e-6).shape == (0, 0)


# ----------------------------------------------------------------------- dense formulations
def _dense_logpdf(r, Sig):
    sgn, ld = np.linalg.slogdet(Sig)
    assert sgn > 0
    return -0.5 * (r @ np.linalg.solve(Sig, r)) - 0.5 * ld - len(r) / 2 * math.log(2 * math.pi)


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_vi_objective_dense(cfg):
    P = O.make_gaussian_problem(cfg, n=160, m=14)
    cp = P["cov_par"]
    K12, K22, Z = O.vi_mats(cp, P["cov_fun"], P["U"], P["X"], P["delta"])
    Q = K12 @ np.linalg.solve(K22, K12.T)
    r = P["y"] - P["mu"]
    tau2, sig2 = cp["tau"] ** 2, cp["sigma"] ** 2
    dense = _dense_logpdf(r, Q + np.diag(Z)) - np.sum(sig2 + P["delta"] - np.diag(Q)) / (2 * tau2)
    got = O.elbo_eval(cp, P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])
    assert abs(got - dense) / abs(dense) < 1e-10


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_fitc_objective_dense(cfg):
    P = O.make_gaussian_problem(cfg, n=160, m=14)
    cp = P["cov_par"]
    K12, K22, Z = O.fitc_mats(cp, P["cov_fun"], P["U"], P["X"], P["delta"])
    Q = K12 @ np.linalg.solve(K22, K12.T)
    dense = _dense_logpdf(P["y"] - P["mu"], Q + np.diag(Z))
    got = O.fitc_obj_eval(cp, P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])
    assert abs(got - dense) / abs(dense) < 1e-10


def test_poisson_objective_dense():
    """log q = log p(y|f) - 1/2 (f-mu)^T Sig^-1 (f-mu) - 1/2 log|I + Sig (-W)|  (R&W 3.32)."""
    P = O.make_poisson_problem(n=90, m=9)
    cp = P["cov_par"]
    K12, K22, Z = O.laplace_mats(cp, "sqexp", P["U"], P["X"], P["delta"])
    Sig = K12 @ np.linalg.solve(K22, K12.T) + np.diag(Z)
    f = P["f0"] + 0.1 * np.sin(np.arange(90))
    W = -P["a"] * np.exp(f)
    logpy = np.sum(P["y"] * math.log(P["a"]) - O.lfactorial(P["y"]) - P["a"] * np.exp(f) + P["y"] * f)
    d = f - P["mu"]
    _, ld = np.linalg.slogdet(np.eye(90) + Sig @ np.diag(-W))
    dense = logpy - 0.5 * d @ np.linalg.solve(Sig, d) - 0.5 * ld
    got = O.obj_fun_pois(f, P["mu"], Z, K12, K22, P["y"], P["a"])
    assert abs(got - dense) / abs(dense) < 1e-10


# ----------------------------------------------------------------------- finite differences
@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_vi_gradient_fd(cfg):
    P = O.make_gaussian_problem(cfg, n=200, m=15)
    cp = P["cov_par"]
    f = lambda c: O.elbo_eval(c, P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])
    g = O.delbo_dcov_par(cp, P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    gf = fd_grad(f, cp)
    for k in cp:
        assert abs(g[k] - gf[k]) / max(1.0, abs(g[k])) < 1e-7, k


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_fitc_gradient_fd(cfg):
    P = O.make_gaussian_problem(cfg, n=200, m=15)
    cp = P["cov_par"]
    f = lambda c: O.fitc_obj_eval(c, P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])
    g = O.dlogp_dcov_par(cp, P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    gf = fd_grad(f, cp)
    for k in cp:
        assert abs(g[k] - gf[k]) / max(1.0, abs(g[k])) < 1e-7, k


def test_laplace_gradient_fd_sigma_tau():
    """The reference's Laplace gradient matches FD of log q(f_hat) for sigma and tau; for the
    length scale it does not -- the author notes a suspected discrepancy
    (laplace_approx_gradient.R:5-23).  Parity is with the reference formula, so the oracle
    reproduces it as written; this test records both facts."""
    P = O.make_poisson_problem(n=160, m=12)
    cp = P["cov_par"]

    def obj(c):
        r = O.newtrap_sparseGP(P["f0"], c, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"], tol=1e-11)
        return r["objective_function_values"][-1]

    nr = O.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"], tol=1e-11)
    g = O.dlogq_dcov_par(cp, "sqexp", P["U"], P["X"], P["y"], nr["gp"], P["mu"], P["a"])["gradient"]
    gf = fd_grad(obj, cp)
    assert abs(g["sigma"] - gf["sigma"]) / abs(g["sigma"]) < 1e-6
    assert abs(g["tau"] - gf["tau"]) / max(1.0, abs(g["tau"])) < 1e-6
    assert abs(g["l"] - gf["l"]) / abs(gf["l"]) > 1e-3    # reference formula, not the FD value


def test_newton_raphson_converges():
    P = O.make_poisson_problem(n=120, m=10)
    r = O.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"], tol=1e-8)
    v = r["objective_function_values"]
    assert len(v) < 30 and abs(v[-1] - v[-2]) < 1e-8 and np.all(np.abs(r["gradient"]) < 1e-6)


def test_r_det_overflow_quirk():
    """log(det(Sigma22)) via R's det() underflows to -Inf once log det < -745."""
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 1, size=(50, 1))
    U = np.linspace(0, 1, 80).reshape(-1, 1)           # dense knots -> tiny eigenvalues
    cp = OrderedDict([("sigma", 1.0), ("l", 0.5), ("tau", 0.5)])
    y = np.sin(X[:, 0])
    K12, K22, Z = O.vi_mats(cp, "sqexp", U, X, 1e-6)
    assert np.linalg.slogdet(K22)[1] < -745
    # det() -> 0, log(0) = -Inf, det_part = -1/2 (... - (-Inf) ...) = -Inf
    assert O.elbo_eval(cp, "sqexp", U, X, y, np.full(50, y.mean()), 1e-6) == -math.inf


# ----------------------------------------------------------------------- adjoint protocol model
@pytest.mark.parametrize("cfg,coinc", [("C2", False), ("C3", False), ("C2", True), ("C3", True)])
def test_adjoint_model_matches_literal(cfg, coinc):
    P = O.make_gaussian_problem(cfg, n=180, m=13)
    U = P["U"].copy()
    if coinc:
        U[:4] = P["X"][:4]
    cp = P["cov_par"]
    o = O.elbo_eval(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])
    g = O.delbo_dcov_par(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    obj, grad = A.eval_vi(P["cov_fun"], np.array(list(cp.values())), P["X"], P["y"], P["mu"], U, P["delta"])
    assert abs(obj - o) / abs(o) < 1e-12
    assert np.max(np.abs(grad - np.array(list(g.values()))) / np.maximum(1, np.abs(list(g.values())))) < 1e-11


@pytest.mark.parametrize("cfg,coinc", [("C2", False), ("C3", True), ("C2", True)])
def test_chunked_adjoint_model_matches_literal(cfg, coinc):
    """oracle/adjoint_chunked.py (the C4-shard / full-n checker and CPU bar) equals the literal
    restatement; chunk < n so the row-chunk loop and the coincidence matching are exercised,
    and a row split with n_global sums to the whole."""
    from oracle import adjoint_chunked as AC
    P = O.make_gaussian_problem(cfg, n=301, m=17)
    U = P["U"].copy()
    if coinc:
        U[:3] = P["X"][[0, 150, 300]]
        U[5] = -0.0 + P["X"][7]
    cp = P["cov_par"]
    th = np.array(list(cp.values()))
    o = O.elbo_eval(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])
    g = np.array(list(O.delbo_dcov_par(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"],
                                       P["delta"])["gradient"].values()))
    obj, grad = AC.eval_vi(P["cov_fun"], th, P["X"], P["y"], P["mu"], U, P["delta"], chunk=64)
    assert abs(obj - o) / abs(o) < 1e-11
    assert np.max(np.abs(grad - g) / np.maximum(1, np.abs(g))) < 1e-10


# ----------------------------------------------------------------------- golden fixtures
@pytest.mark.parametrize("name", ["gauss_c2_small.npz", "gauss_c3_small.npz", "gauss_c2_coincident.npz",
                                  "gauss_c2_m256.npz"])
def test_golden_gaussian(name):
    z = np.load(os.path.join(GOLD, name))
    cp = OrderedDict(zip([str(s) for s in z["names"]], z["theta"]))
    cf = str(z["cov_fun"])
    args = (cp, cf, z["U"], z["X"], z["y"], z["mu"], float(z["delta"]))
    assert np.isclose(O.elbo_eval(*args), z["vi_obj"], rtol=1e-13, atol=0)
    assert np.allclose(list(O.delbo_dcov_par(*args)["gradient"].values()), z["vi_grad"], rtol=1e-11, atol=1e-11)
    assert np.isclose(O.fitc_obj_eval(*args), z["fitc_obj"], rtol=1e-13, atol=0)
    assert np.allclose(list(O.dlogp_dcov_par(*args)["gradient"].values()), z["fitc_grad"], rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("name", ["poisson_c5_small.npz", "poisson_c5_m512.npz",
                                  "poisson_c5_expo.npz"])
def test_golden_poisson(name):
    z = np.load(os.path.join(GOLD, name))
    cp = OrderedDict(zip([str(s) for s in z["names"]], z["theta"]))
    a = z["a"] if z["a"].ndim else float(z["a"])    # per-row exposure in poisson_c5_expo
    nr = O.newtrap_sparseGP(z["f0"], cp, "sqexp", z["X"], z["U"], z["y"], z["mu"], a, tol=1e-5)
    assert np.allclose(nr["gp"], z["ff"], rtol=1e-12, atol=1e-12)
    g = O.dlogq_dcov_par(cp, "sqexp", z["U"], z["X"], z["y"], nr["gp"], z["mu"], a)["gradient"]
    assert np.allclose(list(g.values()), z["grad"], rtol=1e-10, atol=1e-10)


def test_golden_fills():
    z = np.load(os.path.join(GOLD, "fills.npz"))
    cp = {"sigma": 1.3, "l": 1.7, "tau": 0.4}
    assert np.allclose(O.make_cov_matC(z["x"], z["xp"], cp, "sqexp", 1e-6), z["cov_sqexp_cross"], rtol=1e-14)
    assert np.allclose(O.dsig_dthetaC(z["x"], None, cp, "exp", "l"), z["d_exp_l_sym"], rtol=1e-14)


@pytest.mark.parametrize("cov_fun,coinc", [("sqexp", False), ("ard", True)])
def test_laplace_adjoint_model_matches_oracle(cov_fun, coinc):
    """The adjoint-form Laplace algebra the GPU implements (oracle/adjoint_ref.py) reproduces the
    literal newtrap_sparseGP + dlogq_dcov_par, including the reference's comp3 form."""
    from oracle import adjoint_ref as A
    P = O.make_poisson_problem(n=260, m=18)
    U = P["U"].copy()
    if coinc:
        U[:2] = P["X"][[4, 9]]
    cp = P["cov_par"]
    if cov_fun == "ard":
        cp = OrderedDict([("sigma", 1.1)] + [(f"l{c + 1}", 1.5 + 0.3 * c) for c in range(5)]
                         + [("tau", 0.2)])
    th = np.array(list(cp.values()))
    nr = O.newtrap_sparseGP(P["f0"], cp, cov_fun, P["X"], U, P["y"], P["mu"], P["a"], P["delta"],
                            tol=1e-5)
    g = np.array(list(O.dlogq_dcov_par(cp, cov_fun, U, P["X"], P["y"], nr["gp"], P["mu"], P["a"],
                                       P["delta"])["gradient"].values()))
    o, grad, f, it = A.eval_laplace(cov_fun, th, P["X"], P["y"], P["mu"], U, P["f0"], P["a"],
                                    P["delta"], tol=1e-5)
    assert it == len(nr["objective_function_values"])
    assert abs(o - nr["objective_function_values"][-1]) < 1e-10 * abs(o)
    assert np.max(np.abs(grad - g) / np.maximum(1, np.abs(g))) < 1e-10


@pytest.mark.parametrize("cov_fun,coinc,n,m", [("sqexp", False, 2000, 40), ("sqexp", True, 1500, 33),
                                               ("ard", True, 900, 25)])
def test_chunked_laplace_model_matches_literal(cov_fun, coinc, n, m):
    """oracle/adjoint_chunked.eval_laplace (the full-size C5 checker: K12 rebuilt per row chunk)
    equals the literal newtrap_sparseGP + dlogq_dcov_par: same NR iteration count, every NR
    objective to 1e-12, the mode and the gradient; chunk < n exercises the chunk loop and the
    coincidence matching."""
    from oracle import adjoint_chunked as AC
    P = O.make_poisson_problem(n=n, m=m)
    U = P["U"].copy()
    if coinc:
        U[:2] = P["X"][[4, n - 1]]
        U[3] = -0.0 + P["X"][11]
    cp = P["cov_par"]
    if cov_fun == "ard":
        cp = OrderedDict([("sigma", 1.1)] + [(f"l{c + 1}", 1.5 + 0.3 * c) for c in range(5)]
                         + [("tau", 0.2)])
    th = np.array(list(cp.values()))
    nr = O.newtrap_sparseGP(P["f0"], cp, cov_fun, P["X"], U, P["y"], P["mu"], P["a"], P["delta"],
                            tol=1e-5)
    g = np.array(list(O.dlogq_dcov_par(cp, cov_fun, U, P["X"], P["y"], nr["gp"], P["mu"], P["a"],
                                       P["delta"])["gradient"].values()))
    o, grad, f, objs = AC.eval_laplace(cov_fun, th, P["X"], P["y"], P["mu"], U, P["f0"], P["a"],
                                       P["delta"], tol=1e-5, chunk=256)
    ov = np.asarray(nr["objective_function_values"])
    assert len(objs) == len(ov)
    np.testing.assert_allclose(objs, ov, rtol=1e-12, atol=0)
    assert o == objs[-1]
    assert np.max(np.abs(f - nr["gp"])) < 1e-10
    assert np.max(np.abs(grad - g) / np.maximum(1, np.abs(g))) < 1e-10


def test_chunked_laplace_model_per_row_exposure():
    """A per-row exposure (the reference's `m` as a vector of cell areas,
    R/derivative_functions_of_data_likelihoods.R:38, used element-wise at l.7-30 and in
    obj_fun_pois, R/laplace_approx_obj_funs.R:125-129): adjoint_chunked.eval_laplace (the GPU's
    full-size checker) equals the literal oracle, and a constant vector equals the scalar."""
    from oracle import adjoint_chunked as AC
    P = O.make_poisson_problem(n=600, m=20, per_row_exposure=True)
    assert np.ndim(P["a"]) == 1 and np.ptp(P["a"]) > 1.0
    cp = P["cov_par"]
    th = np.array(list(cp.values()))
    nr = O.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"],
                            P["delta"], tol=1e-5)
    g = np.array(list(O.dlogq_dcov_par(cp, "sqexp", P["U"], P["X"], P["y"], nr["gp"], P["mu"],
                                       P["a"], P["delta"])["gradient"].values()))
    o, grad, f, objs = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"],
                                       P["a"], P["delta"], tol=1e-5, chunk=128)
    np.testing.assert_allclose(objs, nr["objective_function_values"], rtol=1e-12, atol=0)
    assert np.max(np.abs(f - nr["gp"])) < 1e-10
    assert np.max(np.abs(grad - g) / np.maximum(1, np.abs(g))) < 1e-10
    # the exposure matters (a scalar 1 gives another answer) and a constant vector is the scalar
    o1 = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"], 1.0,
                         P["delta"], tol=1e-5, chunk=128)[0]
    assert abs(o1 - o) > 1.0
    oc = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"],
                         np.full(600, 1.3), P["delta"], tol=1e-5, chunk=128)
    os_ = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"], 1.3,
                          P["delta"], tol=1e-5, chunk=128)
    assert oc[0] == os_[0] and np.array_equal(oc[1], os_[1])


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_vi_candidate_bordering_matches_rebuild(cfg):
    """The bordered-system ELBO (knot proposals) equals rebuilding the whole
    ELBO with the candidate appended, as knot_prop_random_norm_vi does."""
    P = O.make_gaussian_problem(cfg, n=150, m=9)
    cand = P["X"][[3, 50, 99]]
    th = np.array(list(P["cov_par"].values()))
    got = A.vi_candidates(P["cov_fun"], th, P["X"], P["y"], P["mu"], P["U"], cand, P["delta"])
    for k in range(3):
        ref = O.elbo_eval(P["cov_par"], P["cov_fun"], np.vstack([P["U"], cand[k]]), P["X"],
                          P["y"], P["mu"], P["delta"])
        assert abs(got[k] - ref) < 1e-10 * abs(ref)


def test_full_gp_gradient_is_the_objective_derivative_at_zero_mean():
    """dlogp_dcov_par_full uses alpha = Sigma11^-1 y (not y - mu): it is the derivative of
    obj_fun_norm_full exactly when mu = 0 (central differences in log theta)."""
    import math
    from collections import OrderedDict
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 10, (40, 2))
    y = np.sin(X).sum(1) + rng.normal(0, .3, 40)
    z = np.zeros(40)
    for cov_fun, cp in (("sqexp", OrderedDict(sigma=1.2, l=1.5, tau=0.4)),
                        ("ard", OrderedDict(sigma=0.9, l1=1.1, l2=2.0, tau=0.3))):
        g = O.dlogp_dcov_par_full(cp, cov_fun, X, y, z)["gradient"]
        for k in cp:
            a, b = OrderedDict(cp), OrderedDict(cp)
            a[k] *= math.exp(1e-6)
            b[k] *= math.exp(-1e-6)
            fd = (O.full_obj_eval(a, cov_fun, X, y, z) - O.full_obj_eval(b, cov_fun, X, y, z)) / 2e-6
            assert abs(g[k] - fd) < 1e-6 * max(1.0, abs(fd)), (cov_fun, k, g[k], fd)
    # duplicate rows: Sigma11 carries the nugget on its diagonal only, but dsig_dthetaC puts
    # 2 tau^2 on every coincident pair (quirk Q5), so tau's reference gradient gains
    # 2 tau^2 * G_ij * 2 over the off-diagonal coincident pair (i, j), G = (a a^T - S^-1) / 2
    Xd = X.copy()
    Xd[5] = Xd[9]
    cp = OrderedDict(sigma=1.2, l=1.5, tau=0.4)
    g = O.dlogp_dcov_par_full(cp, "sqexp", Xd, y, z)["gradient"]
    a, b = OrderedDict(cp), OrderedDict(cp)
    a["tau"] *= math.exp(1e-6)
    b["tau"] *= math.exp(-1e-6)
    fd = (O.full_obj_eval(a, "sqexp", Xd, y, z) - O.full_obj_eval(b, "sqexp", Xd, y, z)) / 2e-6
    S = O.full_sigma(cp, "sqexp", Xd, 1e-6)
    al = np.linalg.solve(S, y)
    Si = np.linalg.inv(S)
    extra = 2 * 0.4 ** 2 * (al[5] * al[9] - Si[5, 9])      # (1/2) * 2 entries (5,9), (9,5)
    assert abs(g["tau"] - (fd + extra)) < 1e-6 * abs(fd)


@pytest.mark.parametrize("cov_fun,coinc", [("sqexp", False), ("ard", True)])
def test_chunked_fitc_model_matches_literal(cov_fun, coinc):
    """oracle/adjoint_chunked.eval_fitc (the full-size FITC checker) equals the literal
    obj_fun_norm on the FITC Z and dlogp_dcov_par (R/laplace_approx_obj_funs.R:6,
    R/laplace_approx_gradient.R:720-971); chunk < n exercises the row-chunk loop and the
    coincidence matching."""
    from oracle import adjoint_chunked as AC
    P = O.make_gaussian_problem("C3" if cov_fun == "ard" else "C2", n=301, m=17)
    U = P["U"].copy()
    if coinc:
        U[:3] = P["X"][[0, 150, 300]]
    cp = P["cov_par"]
    o = O.fitc_obj_eval(cp, cov_fun, U, P["X"], P["y"], P["mu"], P["delta"])
    g = O.dlogp_dcov_par(cp, cov_fun, U, P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    obj, grad = AC.eval_fitc(cov_fun, np.array(list(cp.values())), P["X"], P["y"], P["mu"], U,
                             P["delta"], chunk=64)
    gv = np.array(list(g.values()))
    assert abs(obj - o) / abs(o) < 1e-11
    assert np.max(np.abs(grad - gv) / np.maximum(1, np.abs(gv))) < 1e-10
