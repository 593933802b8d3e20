"""FITC and Laplace gradients with and without the stored products.

With memory for them, the row-quadratic passes keep T = K M (K K22^-1 and K Bm^-1 / K C) and
the gradient contraction reads both in ONE pass over K (the two G terms of
dlogp_dcov_par / dlogq_dcov_par summed per element: R/laplace_approx_gradient.R:720-1135, 25-553).
SGP_TSTORE=0 forces the path taken when that memory is not there: two contraction passes, each
recomputing its product on MFMA.  Both must agree with the oracle and with each other (the
coincidence sums, knot partials and records included)."""
import numpy as np
import pytest

from oracle import sgp_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-6


@pytest.fixture(scope="module")
def sgp():
    import sparsergps_amd as S
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return S


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))


def _both(monkeypatch, fn):
    monkeypatch.delenv("SGP_TSTORE", raising=False)
    fused = fn()
    monkeypatch.setenv("SGP_TSTORE", "0")
    plain = fn()
    monkeypatch.delenv("SGP_TSTORE")
    return fused, plain


@pytest.mark.parametrize("cfg,n,m,coinc", [("C2", 300, 20, True), ("C3", 700, 200, True),
                                           ("C3", 1500, 300, False)])
def test_fitc_one_pass_and_two(sgp, monkeypatch, cfg, n, m, coinc):
    P = O.make_gaussian_problem(cfg, n=n, m=m)
    U = P["U"].copy()
    if coinc:
        U[:3] = P["X"][:3]
    cp = P["cov_par"]
    (o1, g1), (o2, g2) = _both(monkeypatch, lambda: sgp.fitc_eval(
        cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"]))
    o = O.fitc_obj_eval(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])
    g = O.dlogp_dcov_par(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    gv = [g[k] for k in cp]
    assert abs(o1 - o) / abs(o) < RTOL and abs(o2 - o) / abs(o) < RTOL
    assert _rel([g1[k] for k in cp], gv) < RTOL
    assert _rel([g2[k] for k in cp], gv) < RTOL
    assert o1 == o2   # the objective does not go through the gradient passes
    assert _rel([g1[k] for k in cp], [g2[k] for k in cp]) < 1e-11


@pytest.mark.parametrize("cov_fun", ["sqexp", "ard"])
def test_fitc_knot_gradient_one_pass_and_two(sgp, monkeypatch, cov_fun):
    P = O.make_gaussian_problem("C2", n=85, m=6)
    U = P["U"].copy()
    U[:2] = P["X"][[4, 40]]
    cp = P["cov_par"] if cov_fun == "sqexp" else {"sigma": 1.2, "l1": 0.8, "l2": 1.1, "l3": 1.4,
                                                    "tau": 0.3}
    ref = O.dlogp_dcov_par(cp, cov_fun, U, P["X"], P["y"], P["mu"], P["delta"],
                           dcov_fun_dknot=cov_fun)
    a, b = _both(monkeypatch, lambda: sgp.dlogp_dcov_par(
        cp, cov_fun, True, cov_fun, None, U, P["X"], P["y"], None, P["mu"], True, P["delta"]))
    for got in (a, b):
        assert _rel(got["knot_gradient"], ref["knot_gradient"]) < RTOL
        assert _rel([got["gradient"][k] for k in cp], [ref["gradient"][k] for k in cp]) < RTOL
    assert _rel(a["knot_gradient"], b["knot_gradient"]) < 1e-11


@pytest.mark.parametrize("n,m,coinc", [(400, 30, True), (900, 130, False)])
def test_laplace_one_pass_and_two(sgp, monkeypatch, n, m, coinc):
    P = O.make_poisson_problem(n=n, m=m)
    U = P["U"].copy()
    if coinc:
        U[:2] = P["X"][[3, n - 1]]
    cp = P["cov_par"]
    nr = O.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], U, P["y"], P["mu"], P["a"], P["delta"],
                            tol=1e-5)
    g = O.dlogq_dcov_par(cp, "sqexp", U, P["X"], P["y"], nr["gp"], P["mu"], P["a"],
                         P["delta"])["gradient"]
    r1, r2 = _both(monkeypatch, lambda: sgp.laplace_eval(
        cp, "sqexp", U, P["X"], P["y"], P["mu"], P["f0"], P["a"], P["delta"], tol=1e-5))
    for r in (r1, r2):
        assert r["nr_iter"] == len(nr["objective_function_values"])
        assert _rel([r["gradient"][k] for k in cp], [g[k] for k in cp]) < RTOL
    assert r1["objective"] == r2["objective"]
    assert _rel([r1["gradient"][k] for k in cp], [r2["gradient"][k] for k in cp]) < 1e-11
