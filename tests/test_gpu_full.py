"""GPU parity for the full (non-sparse) Gaussian GP, config 1:
sgp_eval_full vs obj_fun_norm_full / dlogp_dcov_par_full, predict_gp_full, and the
norm_grad_ascent_full trajectory, against the oracle.  The boston.R data file is absent
(SURVEY F-notes); two shapes with synthetic values: boston.R's real selection (n = 392 rows,
d = 3, exec/boston.R:80) and the shape BASELINE.json configs[0] states (n = 506, d = 13)."""
from collections import OrderedDict

import numpy as np
import pytest

from oracle import drivers as OD
from oracle import sgp_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-6


@pytest.fixture(scope="module")
def sgp():
    import sparsergps_amd as S
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return S


def _data(n=392, d=3, seed=31, dup=True):
    rng = np.random.default_rng(seed)
    X = rng.uniform(0, 10, (n, d))
    if dup:
        X[7] = X[100]                             # coincident rows (tau's dSigma/dtau term)
    y = np.sin(X).sum(1) + rng.normal(0, 0.4, n)
    return X, y, np.full(n, y.mean())


def _cov_par(cov_fun, d):
    if d == 3:
        return (OrderedDict(sigma=1.3, l=1.7, tau=0.45) if cov_fun == "sqexp" else
                OrderedDict(sigma=1.1, l1=1.2, l2=2.2, l3=0.9, tau=0.35))
    # d = 13: length scales wide enough that K is far from its diagonal in 13 dimensions
    if cov_fun == "sqexp":
        return OrderedDict(sigma=1.3, l=5.5, tau=0.45)
    cp = OrderedDict(sigma=1.1)
    for c in range(d):
        cp[f"l{c + 1}"] = 4.0 + 0.4 * c
    cp["tau"] = 0.35
    return cp


@pytest.mark.parametrize("n,d", [(392, 3), (506, 13)])
@pytest.mark.parametrize("cov_fun", ["sqexp", "ard"])
def test_full_eval_matches_oracle(sgp, cov_fun, n, d):
    X, y, mu = _data(n=n, d=d)
    cp = _cov_par(cov_fun, d)
    obj, g = sgp.full_eval(cp, cov_fun, X, y, mu)
    ro = O.full_obj_eval(cp, cov_fun, X, y, mu)
    rg = O.dlogp_dcov_par_full(cp, cov_fun, X, y, mu)["gradient"]
    assert abs(obj - ro) / abs(ro) < RTOL
    for k in cp:
        assert abs(g[k] - rg[k]) / max(1.0, abs(rg[k])) < RTOL, (k, g[k], rg[k])
    assert abs(sgp.obj_fun_norm_full(cp, cov_fun, X, y, mu) - ro) / abs(ro) < RTOL


@pytest.mark.parametrize("full_cov", [False, True])
def test_predict_gp_full_matches_oracle(sgp, full_cov):
    X, y, mu = _data(n=200, dup=False)
    rng = np.random.default_rng(8)
    xp = rng.uniform(0, 10, (57, 3))
    cp = OrderedDict(sigma=1.3, l=1.7, tau=0.45)
    mup = np.full(57, 0.25)
    got = sgp.predict_gp_full(X, y, xp, "sqexp", cp, mu, mup, full_cov)
    ref = O.predict_gp_full(X, y, xp, "sqexp", cp, mu, mup, full_cov)
    np.testing.assert_allclose(got["pred_mean"], ref["pred_mean"], rtol=1e-8, atol=1e-9)
    np.testing.assert_allclose(got["pred_var"], ref["pred_var"], rtol=1e-8, atol=1e-9)
    mod = {"family": "gaussian", "sparse": False, "delta": 1e-6,
           "results": {"xy": X, "y": y, "mu": mu, "cov_fun": "sqexp", "cov_par": cp}}
    pg = sgp.predict_gp(mod, xp, mup, full_cov)
    np.testing.assert_allclose(pg["pred"]["pred_mean"], ref["pred_mean"], rtol=1e-8, atol=1e-9)


def test_norm_grad_ascent_full_matches_oracle(sgp):
    X, y, mu = _data(n=150, dup=False)
    cp = OrderedDict(sigma=1.0, l=1.0, tau=0.5)
    opt = {"maxit": 5, "obj_tol": 0.0}
    ref = OD.norm_grad_ascent_full(cp, "sqexp", X, y, mu, opt)
    got = sgp.norm_grad_ascent_full(cp, "sqexp", True, X, y, mu, opt)
    assert got["iter"] == ref["iter"] == 5
    np.testing.assert_allclose(got["obj_fun"], ref["obj_fun"], rtol=RTOL)
    np.testing.assert_allclose(got["cov_par_history"], ref["cov_par_history"], rtol=RTOL)
    np.testing.assert_allclose(got["grad"], ref["grad"], rtol=RTOL, atol=1e-7)
