"""GPU parity for the knot posterior (end of the drivers) and sparse prediction
(predict_vi / predict_laplace / predict_gp) vs the CPU oracle."""
from collections import OrderedDict

import numpy as np
import pytest

from oracle import sgp_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-8


@pytest.fixture(scope="module")
def sgp():
    import sparsergps_amd as S
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return S


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


def _theta(P):
    return np.array(list(P["cov_par"].values()))


@pytest.mark.parametrize("cfg,n,m", [("C2", 300, 20), ("C3", 400, 24), ("C2", 500, 130)])
def test_posterior_u_vi(sgp, cfg, n, m):
    P = O.make_gaussian_problem(cfg, n=n, m=m)
    muu = np.full(m, P["y"].mean())
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m) as ctx:
        ctx.eval_vi(_theta(P), P["cov_fun"], P["U"], P["delta"])
        um, uv = ctx.posterior_u(muu)
    rm, rv = O.vi_posterior_u(P["cov_par"], P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], muu,
                              P["delta"])
    assert _rel(um, rm) < RTOL and _rel(uv, rv) < 1e-7


def test_posterior_u_fitc(sgp):
    P = O.make_gaussian_problem("C3", n=350, m=30)
    muu = np.full(30, P["y"].mean())
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=30) as ctx:
        ctx.eval_fitc(_theta(P), "ard", P["U"], P["delta"])
        um, uv = ctx.posterior_u(muu)
    rm, rv = O.fitc_posterior_u(P["cov_par"], "ard", P["U"], P["X"], P["y"], P["mu"], muu,
                                P["delta"])
    assert _rel(um, rm) < RTOL and _rel(uv, rv) < 1e-7


def test_posterior_u_laplace(sgp):
    P = O.make_poisson_problem(n=400, m=25)
    muu = np.full(25, P["mu"][0])
    nr = O.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], P["U"], P["y"], P["mu"],
                            P["a"], P["delta"], tol=1e-5, muu=muu)
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=25) as ctx:
        ctx.lap_set_f(P["f0"])
        ctx.eval_laplace(_theta(P), "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        um, uv = ctx.posterior_u(muu)
    assert _rel(um, nr["u_posterior_mean"]) < RTOL
    assert _rel(uv, nr["u_posterior_variance"]) < 1e-7


def _pred_inputs(cfg, n, m, npred, seed=21):
    P = O.make_gaussian_problem(cfg, n=n, m=m)
    muu = np.full(m, P["y"].mean())
    um, uv = O.vi_posterior_u(P["cov_par"], P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], muu,
                              P["delta"])
    d = P["X"].shape[1]
    xp = np.random.default_rng(seed).uniform(0, 10, size=(npred, d))
    xp[:2] = P["U"][:2]                               # prediction at knots (exact coincidence)
    return P, muu, um, uv, xp, np.full(npred, P["y"].mean())


@pytest.mark.parametrize("cfg,full", [("C2", False), ("C2", True), ("C3", False), ("C3", True)])
def test_predict_vi(sgp, cfg, full):
    P, muu, um, uv, xp, mup = _pred_inputs(cfg, 300, 20, 150)
    got = sgp.predict_vi(um, uv, P["U"], xp, P["cov_fun"], P["cov_par"], mup, muu, full,
                         delta=P["delta"])
    ref = O.predict_vi(um, uv, P["U"], xp, P["cov_fun"], P["cov_par"], mup, muu, full, P["delta"])
    assert _rel(got["pred_mean"].ravel(), ref["pred_mean"]) < RTOL
    assert got["pred_var"].shape == ref["pred_var"].shape
    assert _rel(got["pred_var"], ref["pred_var"]) < RTOL


@pytest.mark.parametrize("family,full", [("gaussian", False), ("gaussian", True),
                                         ("poisson", False), ("poisson", True)])
def test_predict_laplace(sgp, family, full):
    if family == "gaussian":
        P, muu, um, uv, xp, mup = _pred_inputs("C2", 300, 20, 140)
    else:
        P = O.make_poisson_problem(n=300, m=20)
        muu = np.full(20, P["mu"][0])
        nr = O.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], P["U"], P["y"], P["mu"],
                                P["a"], P["delta"], tol=1e-5, muu=muu)
        um, uv = nr["u_posterior_mean"], nr["u_posterior_variance"]
        xp = np.random.default_rng(5).uniform(0, 10, size=(140, 5))
        mup = np.full(140, P["mu"][0])
    got = sgp.predict_laplace(um, uv, P["U"], xp, P["cov_fun"], P["cov_par"], mup, muu, full,
                              family, P["delta"])
    ref = O.predict_laplace(um, uv, P["U"], xp, P["cov_fun"], P["cov_par"], mup, muu, full,
                            family, P["delta"])
    assert _rel(got["pred_mean"].ravel(), ref["pred_mean"]) < RTOL
    assert _rel(got["pred_var"], ref["pred_var"]) < RTOL


def test_predict_gp_dispatch(sgp):
    P, muu, um, uv, xp, mup = _pred_inputs("C2", 250, 16, 70)
    mod = {"family": "gaussian", "sparse": True, "delta": P["delta"],
           "results": {"u_mean": um, "u_var": uv, "xu": P["U"], "cov_fun": "sqexp",
                       "cov_par": P["cov_par"], "muu": muu}}
    r_vi = sgp.predict_gp(mod, xp, mup, full_cov=False, vi=True)
    r_lp = sgp.predict_gp(mod, xp, mup, full_cov=False, vi=False)
    ref_vi = O.predict_vi(um, uv, P["U"], xp, "sqexp", P["cov_par"], mup, muu, False, P["delta"])
    ref_lp = O.predict_laplace(um, uv, P["U"], xp, "sqexp", P["cov_par"], mup, muu, False,
                               "gaussian", P["delta"])
    assert _rel(r_vi["pred"]["pred_var"], ref_vi["pred_var"]) < RTOL
    assert _rel(r_lp["pred"]["pred_var"], ref_lp["pred_var"]) < RTOL
    assert sgp.predict_gp(dict(mod, family="poisson"), xp, mup, vi=True).startswith("Error")
