"""GPU parity for knot gradients (xu_opt = "simultaneous"): the knot branches of
delbo_dcov_par / dlogp_dcov_par / dlogq_dcov_par with dsqexp_dx2(_ard) vs the literal oracle
(which loops over all m*d knot coordinates with dense derivative matrices)."""
from collections import OrderedDict

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


def _close(a, b, tol=RTOL):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) < tol


def _ard_par(d):
    return OrderedDict([("sigma", 1.2)] + [(f"l{c + 1}", 1.3 + 0.4 * c) for c in range(d)] +
                       [("tau", 0.45)])


@pytest.mark.parametrize("cov_fun,coinc", [("sqexp", False), ("ard", False), ("sqexp", True)])
def test_vi_knot_gradient(sgp, cov_fun, coinc):
    P = O.make_gaussian_problem("C2", n=90, m=7)
    cp = P["cov_par"] if cov_fun == "sqexp" else _ard_par(3)
    U = P["U"].copy()
    if coinc:
        U[1] = P["X"][4]
    ref = O.delbo_dcov_par(cp, cov_fun, U, P["X"], P["y"], P["mu"], P["delta"],
                           dcov_fun_dknot=cov_fun)
    got = sgp.delbo_dcov_par(cp, cov_fun, True, "dsqexp_dx2" if cov_fun == "sqexp" else
                             "dsqexp_dx2_ard", None, U, P["X"], P["y"], None, P["mu"], True,
                             P["delta"])
    assert _close(got["knot_gradient"], ref["knot_gradient"])
    assert _close(got["trans_knot"], ref["trans_knot"], 1e-12)
    for k in cp:
        assert abs(got["gradient"][k] - ref["gradient"][k]) / max(1, abs(ref["gradient"][k])) < RTOL


@pytest.mark.parametrize("cov_fun", ["sqexp", "ard"])
def test_vi_knot_gradient_mp256(sgp, cov_fun):
    # 129 <= m <= 256 (m_p = 256, C2's knot count): the fragment-balanced k_syrk_s256 path
    P = O.make_gaussian_problem("C2", n=230, m=140)
    cp = P["cov_par"] if cov_fun == "sqexp" else _ard_par(3)
    U = P["U"].copy()
    U[3] = P["X"][17]
    ref = O.delbo_dcov_par(cp, cov_fun, U, P["X"], P["y"], P["mu"], P["delta"],
                           dcov_fun_dknot=cov_fun)
    got = sgp.delbo_dcov_par(cp, cov_fun, True, "dsqexp_dx2" if cov_fun == "sqexp" else
                             "dsqexp_dx2_ard", None, U, P["X"], P["y"], None, P["mu"], True,
                             P["delta"])
    assert _close(got["knot_gradient"], ref["knot_gradient"])
    for k in cp:
        assert abs(got["gradient"][k] - ref["gradient"][k]) / max(1, abs(ref["gradient"][k])) < RTOL


def test_vi_knot_opt_subset(sgp):
    P = O.make_gaussian_problem("C2", n=80, m=6)
    ref = O.delbo_dcov_par(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], P["mu"], P["delta"],
                           dcov_fun_dknot="sqexp", knot_opt=[2, 5])
    got = sgp.delbo_dcov_par(P["cov_par"], "sqexp", True, "sqexp", [2, 5], P["U"], P["X"],
                             P["y"], None, P["mu"], True, P["delta"])
    assert _close(got["knot_gradient"], ref["knot_gradient"])
    assert np.count_nonzero(got["knot_gradient"]) == 2 * 3


@pytest.mark.parametrize("cov_fun", ["sqexp", "ard"])
def test_fitc_knot_gradient(sgp, cov_fun):
    P = O.make_gaussian_problem("C2", n=85, m=6)
    cp = P["cov_par"] if cov_fun == "sqexp" else _ard_par(3)
    ref = O.dlogp_dcov_par(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"],
                           dcov_fun_dknot=cov_fun)
    got = sgp.dlogp_dcov_par(cp, cov_fun, True, cov_fun, None, P["U"], P["X"], P["y"], None,
                             P["mu"], True, P["delta"])
    assert _close(got["knot_gradient"], ref["knot_gradient"])


@pytest.mark.parametrize("cov_fun", ["sqexp", "ard"])
def test_laplace_knot_gradient(sgp, cov_fun):
    P = O.make_poisson_problem(n=90, m=6)
    cp = P["cov_par"] if cov_fun == "sqexp" else _ard_par(5)
    ff = P["f0"] + 0.05 * np.cos(np.arange(90))
    ref = O.dlogq_dcov_par(cp, cov_fun, P["U"], P["X"], P["y"], ff, P["mu"], P["a"], P["delta"],
                           dcov_fun_dknot=cov_fun)
    got = sgp.dlogq_dcov_par(cp, cov_fun, True, cov_fun, None, P["U"], P["X"], P["y"], ff,
                             P["mu"], P["a"], P["delta"])
    assert _close(got["knot_gradient"], ref["knot_gradient"])
    for k in cp:
        assert abs(got["gradient"][k] - ref["gradient"][k]) / max(1, abs(ref["gradient"][k])) < RTOL


def test_knot_gradient_larger_m(sgp):
    """m = 200 knots (two 128-column tiles, padded) against the adjoint identity: the GPU knot
    gradient equals central differences of the GPU ELBO in u times the reference factor."""
    P = O.make_gaussian_problem("C2", n=3000, m=200)
    th = np.array(list(P["cov_par"].values()))
    b = O.knot_bounds_of(P["X"])
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=200) as ctx:
        ctx.enable_knot_grad(True)
        ctx.eval_vi(th, "sqexp", P["U"], P["delta"])
        g = ctx.knot_gradient(b)
        ctx.enable_knot_grad(False)
        h = 1e-5
        for k, c in [(0, 0), (77, 2), (199, 1)]:
            Up, Um = P["U"].copy(), P["U"].copy()
            Up[k, c] += h
            Um[k, c] -= h
            fd = (ctx.eval_vi(th, "sqexp", Up, P["delta"])[0] -
                  ctx.eval_vi(th, "sqexp", Um, P["delta"])[0]) / (2 * h)
            u = P["U"][k, c]
            chain = (b[c, 1] - b[c, 0]) / ((u - b[c, 0]) * (b[c, 1] - u) + 1e-4)
            assert abs(fd * chain - g[k * 3 + c]) / max(1.0, abs(g[k * 3 + c])) < 1e-5


def _hd_problem(n, m, d, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    X = g.uniform(0.0, 10.0, size=(n, d))
    U = g.uniform(0.0, 10.0, size=(m, d))
    y = np.sin(X).sum(axis=1) / np.sqrt(d) + g.normal(0.0, 0.5, size=n)
    cp = OrderedDict([("sigma", 1.2)] + [(f"l{c + 1}", np.sqrt(d) + 0.2 * c)
                                          for c in range(d)] + [("tau", 0.45)])
    return X, U, y, np.full(n, y.mean()), cp


@pytest.mark.parametrize("mode,d", [("vi", 12), ("fitc", 12), ("vi", 20)])
def test_knot_gradient_high_dim(sgp, mode, d):
    """d > 8: the knot partials leave the contraction epilogue one chunk of 8 coordinates at a
    time (k_contract<32, ..., KNOT>)."""
    X, U, y, mu, cp = _hd_problem(200, 7, d, seed=600 + d)
    delta = 1e-6
    if mode == "vi":
        ref = O.delbo_dcov_par(cp, "ard", U, X, y, mu, delta, dcov_fun_dknot="ard")
        got = sgp.delbo_dcov_par(cp, "ard", True, "dsqexp_dx2_ard", None, U, X, y, None, mu, True,
                                 delta)
    else:
        ref = O.dlogp_dcov_par(cp, "ard", U, X, y, mu, delta, dcov_fun_dknot="ard")
        got = sgp.dlogp_dcov_par(cp, "ard", True, "ard", None, U, X, y, None, mu, True, delta)
    kg, kr = np.asarray(got["knot_gradient"]), np.asarray(ref["knot_gradient"])
    assert np.max(np.abs(kg - kr)) < RTOL * np.max(np.abs(kr))   # relative to the largest
    for k in cp:
        assert abs(got["gradient"][k] - ref["gradient"][k]) / max(1, abs(ref["gradient"][k])) < RTOL


def test_laplace_knot_gradient_high_dim(sgp):
    g = np.random.Generator(np.random.PCG64(707))
    n, m, d = 150, 6, 10
    X = g.uniform(0.0, 10.0, size=(n, d))
    U = g.uniform(0.0, 10.0, size=(m, d))
    f = 0.5 * np.sin(X).sum(axis=1) / np.sqrt(d) + np.log(2.0)
    y = g.poisson(np.exp(f)).astype(np.float64)
    mu = np.full(n, np.log(y.mean()))
    ff = mu + 0.05 * np.cos(np.arange(n))
    cp = OrderedDict([("sigma", 1.0)] + [(f"l{c + 1}", np.sqrt(d) + 0.2 * c) for c in range(d)]
                     + [("tau", 0.1)])
    ref = O.dlogq_dcov_par(cp, "ard", U, X, y, ff, mu, 1.0, 1e-6, dcov_fun_dknot="ard")
    got = sgp.dlogq_dcov_par(cp, "ard", True, "ard", None, U, X, y, ff, mu, 1.0, 1e-6)
    kg, kr = np.asarray(got["knot_gradient"]), np.asarray(ref["knot_gradient"])
    assert np.max(np.abs(kg - kr)) < RTOL * np.max(np.abs(kr))
    for k in cp:
        assert abs(got["gradient"][k] - ref["gradient"][k]) / max(1, abs(ref["gradient"][k])) < RTOL
