"""GPU parity at the shape edges the fused kernels' tiling must get right: fewer rows than
knots, row / knot counts exactly on the 128-tile grid and one past it, one input dimension,
and a single data row.  Checker: the CPU oracle (literal restatement of the reference), held
to the north-star 1e-6 relative bar like the other parity tests.

The reference has no tests of its own; these shapes are the ones its callers
reach: optimize_gp() with few observations per knot, and predict_* with one-row inputs.
"""
import math
from collections import OrderedDict

import numpy as np
import pytest

from oracle import sgp_oracle as O

pytestmark = pytest.mark.gpu
EVAL_RTOL = 1e-6


@pytest.fixture(scope="module")
def sgp():
    import sparsergps_amd as S
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return S


def _gauss(n, m, d, cov_fun, seed):
    """Synthetic Gaussian regression of any shape (same recipe as SURVEY 8(d)'s generators)."""
    g = np.random.Generator(np.random.PCG64(seed))
    X = g.uniform(0.0, 10.0, size=(n, d))
    U = g.uniform(0.0, 10.0, size=(m, d))
    y = np.sin(X).sum(axis=1) / math.sqrt(d) + g.normal(0.0, 0.5, size=n)
    l0 = 1.7
    if d == 1:
        # random knots on a line nearly coincide (cond(K22) ~ 1e7 at m = 40, where two fp64
        # algorithms -- the oracle's LU solves vs a Cholesky/inverse model -- already differ by
        # 1e-4 in the gradient); a knot grid with l ~ its spacing is how 1-D fits are set up
        U = np.linspace(0.1, 9.9, m)[:, None]
        l0 = 0.5
    if cov_fun == "ard":
        cp = OrderedDict([("sigma", 1.2)] + [(f"l{c + 1}", l0 + 0.25 * c) for c in range(d)]
                         + [("tau", 0.5)])
    else:
        cp = OrderedDict([("sigma", 1.2), ("l", l0), ("tau", 0.5)])
    return dict(X=X, U=U, y=y, mu=np.full(n, y.mean()), cov_par=cp, cov_fun=cov_fun, delta=1e-6)


def _close(obj, grad, o_ref, g_ref, cp):
    assert abs(obj - o_ref) / abs(o_ref) < EVAL_RTOL, (obj, o_ref)
    for k in cp:
        assert abs(grad[k] - g_ref[k]) / max(1.0, abs(g_ref[k])) < EVAL_RTOL, (k, grad[k], g_ref[k])


SHAPES = [
    # n, m, d, cov_fun
    (60, 200, 3, "sqexp"),     # fewer rows than knots
    (1024, 128, 8, "ard"),     # both exactly on the 128-tile grid
    (1025, 129, 8, "ard"),     # one past it on both axes
    (500, 20, 1, "sqexp"),     # one input dimension (knot grid, cond(K22) ~ 50)
    (700, 20, 1, "ard"),
    (1, 7, 3, "sqexp"),        # a single data row
]


@pytest.mark.parametrize("n,m,d,cov_fun", SHAPES)
def test_vi_edge_shapes(sgp, n, m, d, cov_fun):
    P = _gauss(n, m, d, cov_fun, seed=100 + n + m + d)
    cp = P["cov_par"]
    obj, grad = sgp.vi_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    o = O.elbo_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    g = O.delbo_dcov_par(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    _close(obj, grad, o, g, cp)


@pytest.mark.parametrize("n,m,d,cov_fun", SHAPES)
def test_fitc_edge_shapes(sgp, n, m, d, cov_fun):
    P = _gauss(n, m, d, cov_fun, seed=200 + n + m + d)
    cp = P["cov_par"]
    obj, grad = sgp.fitc_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    o = O.fitc_obj_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    g = O.dlogp_dcov_par(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    _close(obj, grad, o, g, cp)


# (777, 300) and (500, 1100): knot tiles (mp = 384, 1152) that do not divide the fused Newton
# pass's 8192-double row image (k_lap_nr_a_fused: 21- and 7-row blocks, short last blocks)
@pytest.mark.parametrize("n,m", [(60, 150), (1024, 128), (1025, 129), (777, 300), (500, 1100)])
def test_laplace_edge_shapes(sgp, n, m):
    P = O.make_poisson_problem(n=n, m=m)
    cp = P["cov_par"]
    nr = O.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"],
                            P["delta"], tol=1e-5)
    g = O.dlogq_dcov_par(cp, "sqexp", P["U"], P["X"], P["y"], nr["gp"], P["mu"], P["a"],
                         P["delta"])["gradient"]
    r = sgp.laplace_eval(cp, "sqexp", P["U"], P["X"], P["y"], P["mu"], P["f0"], P["a"],
                         P["delta"], tol=1e-5)
    ov = nr["objective_function_values"]
    assert r["nr_iter"] == len(ov)
    _close(r["objective"], r["gradient"], ov[-1], g, cp)


@pytest.mark.parametrize("mode", ["vi", "fitc"])
def test_more_knots_than_c3(sgp, mode):
    """m = 1536 (12 knot tiles: the packed SYRK's nb = 12 grouping, 24 Gauss-Jordan pivots).
    |K22| underflows here, so the literal oracle's objective is R's det() quirk -inf (Q4): the
    objective is checked against the adjoint model (log-determinants from the factorisation),
    the gradient -- which the reference computes without det() -- against the oracle."""
    from oracle import adjoint_ref as A
    P = O.make_gaussian_problem("C3", n=2000, m=1536)
    cp = P["cov_par"]
    theta = np.array(list(cp.values()))
    if mode == "vi":
        obj, grad = sgp.vi_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o_lit = O.elbo_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o, _ = A.eval_vi("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"])
        g = O.delbo_dcov_par(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    else:
        obj, grad = sgp.fitc_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o_lit = O.fitc_obj_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o, _ = A.eval_fitc("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"])
        g = O.dlogp_dcov_par(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    assert o_lit == -np.inf                  # the quirk this case exercises
    _close(obj, grad, o, g, cp)


@pytest.mark.parametrize("dup_at,order", [(150, 151), (40, 41)])
def test_not_positive_definite_order(sgp, dup_at, order):
    """A duplicated knot with a negative jitter makes K22 = Kuu + delta I indefinite from the
    leading minor of order dup_at + 1 on (the earlier minors are PD: min eigenvalue 0.14);
    the reference's chol() fails there (an R error, caught by try() in the knot proposals).
    The GPU inverse must report the same order (SGP_ENOTPD, include/sgp.h)."""
    from sparsergps_amd._lib import NotPositiveDefinite
    g = np.random.Generator(np.random.PCG64(77))
    n, m, d = 500, 200, 3
    U = g.uniform(0.0, 10.0, size=(m, d))
    U[dup_at] = U[3]
    X = g.uniform(0.0, 10.0, size=(n, d))
    y = np.sin(X).sum(axis=1) + g.normal(0.0, 0.5, size=n)
    cp = OrderedDict([("sigma", 1.0), ("l", 0.3), ("tau", 0.5)])
    with pytest.raises(NotPositiveDefinite, match=f"order {order} of Sigma22"):
        sgp.vi_eval(cp, "sqexp", U, X, y, np.full(n, y.mean()), -1e-3)
    # the context recovers: a valid evaluation right after succeeds
    P = _gauss(300, 40, 3, "sqexp", seed=5)
    obj, _ = sgp.vi_eval(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], P["mu"], P["delta"])
    assert np.isfinite(obj)


@pytest.mark.parametrize("mode", ["vi", "fitc"])
def test_coincidence_flags_follow_knot_changes(sgp, mode):
    """One context, knot sets alternating between data rows (x_i == u_j exactly: the tau
    coincidence rule, quirk Q5) and random knots.  The rows that equal a knot are found once
    per knot set and cached; every evaluation must still match the oracle."""
    P = _gauss(400, 30, 3, "sqexp", seed=31)
    X, y, mu, cp = P["X"], P["y"], P["mu"], P["cov_par"]
    U_on = X[[5, 17, 40, 99, 123] + list(range(200, 225))].copy()
    U_off = P["U"]
    for U in (U_on, U_off, U_on, U_on, U_off):
        if mode == "vi":
            obj, grad = sgp.vi_eval(cp, "sqexp", U, X, y, mu, P["delta"])
            o = O.elbo_eval(cp, "sqexp", U, X, y, mu, P["delta"])
            g = O.delbo_dcov_par(cp, "sqexp", U, X, y, mu, P["delta"])["gradient"]
        else:
            obj, grad = sgp.fitc_eval(cp, "sqexp", U, X, y, mu, P["delta"])
            o = O.fitc_obj_eval(cp, "sqexp", U, X, y, mu, P["delta"])
            g = O.dlogp_dcov_par(cp, "sqexp", U, X, y, mu, P["delta"])["gradient"]
        _close(obj, grad, o, g, cp)


def _gauss_hd(n, m, d, cov_fun, seed):
    """Higher-dimensional inputs (d > 8: the contraction processes coordinates in chunks of 8);
    length scales ~ sqrt(d) keep K12 away from underflow."""
    P = _gauss(n, m, d, cov_fun, seed)
    s = math.sqrt(d)
    if cov_fun == "ard":
        P["cov_par"] = OrderedDict([("sigma", 1.2)] + [(f"l{c + 1}", 1.2 * s + 0.2 * c)
                                                        for c in range(d)] + [("tau", 0.5)])
    else:
        P["cov_par"] = OrderedDict([("sigma", 1.2), ("l", 1.4 * s), ("tau", 0.5)])
    return P


HD_SHAPES = [(600, 40, 12, "ard"), (600, 40, 12, "sqexp"), (500, 33, 20, "ard"),
             (300, 20, 32, "ard")]


@pytest.mark.parametrize("n,m,d,cov_fun", HD_SHAPES)
def test_vi_high_dim(sgp, n, m, d, cov_fun):
    P = _gauss_hd(n, m, d, cov_fun, seed=400 + d)
    cp = P["cov_par"]
    obj, grad = sgp.vi_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    o = O.elbo_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    g = O.delbo_dcov_par(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    assert max(abs(v) for v in g.values()) > 1.0    # a non-trivial gradient
    _close(obj, grad, o, g, cp)


@pytest.mark.parametrize("n,m,d,cov_fun", HD_SHAPES)
def test_fitc_high_dim(sgp, n, m, d, cov_fun):
    P = _gauss_hd(n, m, d, cov_fun, seed=500 + d)
    cp = P["cov_par"]
    obj, grad = sgp.fitc_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    o = O.fitc_obj_eval(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    g = O.dlogp_dcov_par(cp, cov_fun, P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    _close(obj, grad, o, g, cp)


def test_laplace_high_dim(sgp):
    g0 = np.random.Generator(np.random.PCG64(77))
    n, m, d = 400, 30, 10
    X = g0.uniform(0.0, 10.0, size=(n, d))
    U = g0.uniform(0.0, 10.0, size=(m, d))
    f = 0.5 * np.sin(X).sum(axis=1) / math.sqrt(d) + math.log(2.0)
    y = g0.poisson(np.exp(f)).astype(np.float64)
    mu = np.full(n, math.log(y.mean()))
    f0 = mu.copy()
    cp = OrderedDict([("sigma", 1.0), ("l", 1.4 * math.sqrt(d)), ("tau", 0.1)])
    nr = O.newtrap_sparseGP(f0, cp, "sqexp", X, U, y, mu, 1.0, 1e-6, tol=1e-5)
    g = O.dlogq_dcov_par(cp, "sqexp", U, X, y, nr["gp"], mu, 1.0, 1e-6)["gradient"]
    r = sgp.laplace_eval(cp, "sqexp", U, X, y, mu, f0, 1.0, 1e-6, tol=1e-5)
    ov = nr["objective_function_values"]
    assert r["nr_iter"] == len(ov)
    _close(r["objective"], r["gradient"], ov[-1], g, cp)


@pytest.mark.parametrize("mode", ["vi", "fitc", "laplace"])
def test_knots_past_the_syrk_table(sgp, mode):
    """m = 2048 (nb = 16: 136 packed SYRK groups per row chunk, more than the balanced t-slice
    table holds, so the weighted SYRK with t -- FITC phase 1, the Laplace objective pass --
    takes the one-slice-per-panel placement).  Gaussian objectives against the adjoint model
    (R's det() underflows here, quirk Q4), gradients against the literal oracle."""
    from oracle import adjoint_ref as A
    if mode == "laplace":
        P = O.make_poisson_problem(n=700, m=2048)
        cp = P["cov_par"]
        nr = O.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"],
                                P["delta"], tol=1e-5)
        g = O.dlogq_dcov_par(cp, "sqexp", P["U"], P["X"], P["y"], nr["gp"], P["mu"], P["a"],
                             P["delta"])["gradient"]
        r = sgp.laplace_eval(cp, "sqexp", P["U"], P["X"], P["y"], P["mu"], P["f0"], P["a"],
                             P["delta"], tol=1e-5)
        ov = nr["objective_function_values"]
        assert r["nr_iter"] == len(ov)
        _close(r["objective"], r["gradient"], ov[-1], g, cp)
        return
    P = O.make_gaussian_problem("C3", n=700, m=2048)
    cp = P["cov_par"]
    theta = np.array(list(cp.values()))
    if mode == "vi":
        obj, grad = sgp.vi_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o, _ = A.eval_vi("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"])
        g = O.delbo_dcov_par(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    else:
        obj, grad = sgp.fitc_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o, _ = A.eval_fitc("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"])
        g = O.dlogp_dcov_par(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    _close(obj, grad, o, g, cp)


@pytest.mark.parametrize("maxit", [0, 1, 2, 3])
def test_newtrap_small_maxit(sgp, maxit):
    """newtrap_sparseGP.R:79-96 performs the first update before its while loop whatever maxit
    is: maxit <= 2 returns two objective values, maxit = 3 at most three."""
    P = O.make_poisson_problem(n=400, m=30)
    cp = P["cov_par"]
    nr = O.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"],
                            P["delta"], maxit=maxit, tol=1e-6)
    r = sgp.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"],
                             P["delta"], maxit=maxit, tol=1e-6)
    ov, rv = nr["objective_function_values"], np.asarray(r["objective_function_values"])
    assert len(rv) == len(ov) == (2 if maxit <= 2 else 3)
    assert np.max(np.abs(rv - ov) / np.abs(ov)) < 1e-9
    assert np.max(np.abs(r["gp"] - nr["gp"])) < 1e-8


@pytest.mark.parametrize("mode", ["vi", "fitc"])
@pytest.mark.parametrize("layout", ["offset", "wide"])
def test_data_far_from_origin_or_widely_spread(sgp, mode, layout):
    """The matrix-core K12 builder forms the exponent as x~.u~ - |x~|^2/2 - |u~|^2/2 around
    the knots' mean, whose rounding grows with |x~|^2 (k_cov.hip).  "offset": data 5e3 away
    from the origin (centring keeps the matrix-core form exact to ~1e-14); "wide": data spread
    over ~300 length scales (|x~|^2 ~ 1e5, past SGP_MFMA_SPAN2_MAX: the direct-difference
    builder runs instead).  Knots are data rows plus a small jitter so K12 is not all zeros."""
    g = np.random.Generator(np.random.PCG64(91 if layout == "offset" else 92))
    n, m, d = 1500, 40, 3 if layout == "offset" else 2
    if layout == "offset":
        X = 5.0e3 + g.uniform(0.0, 10.0, size=(n, d))
        cp = OrderedDict([("sigma", 1.2), ("l", 1.7), ("tau", 0.5)])
    else:
        X = g.uniform(0.0, 400.0, size=(n, d))
        cp = OrderedDict([("sigma", 1.2), ("l", 0.7), ("tau", 0.5)])
    U = X[g.choice(n, m, replace=False)] + g.normal(0.0, 0.3, size=(m, d))
    y = np.sin(X / 7.0).sum(axis=1) + g.normal(0.0, 0.5, size=n)
    mu = np.full(n, y.mean())
    if mode == "vi":
        obj, grad = sgp.vi_eval(cp, "sqexp", U, X, y, mu, 1e-6)
        o = O.elbo_eval(cp, "sqexp", U, X, y, mu, 1e-6)
        gr = O.delbo_dcov_par(cp, "sqexp", U, X, y, mu, 1e-6)["gradient"]
    else:
        obj, grad = sgp.fitc_eval(cp, "sqexp", U, X, y, mu, 1e-6)
        o = O.fitc_obj_eval(cp, "sqexp", U, X, y, mu, 1e-6)
        gr = O.dlogp_dcov_par(cp, "sqexp", U, X, y, mu, 1e-6)["gradient"]
    _close(obj, grad, o, gr, cp)


@pytest.mark.parametrize("mode", ["vi", "fitc"])
def test_knots_past_the_persistent_chain(sgp, mode):
    """m = 4160 (m_p = 4224, nb = 66 > 64): the m x m inverses fall back from the persistent
    Gauss-Jordan kernel to one launch per pivot step, and the SYRKs from the balanced plan to the
    packed one (m > 3968).  Objective and gradient against the adjoint model (R's det()
    underflows here, quirk Q4; the literal oracle's n x m algebra is too slow at this m)."""
    from oracle import adjoint_ref as A
    P = O.make_gaussian_problem("C3", n=300, m=4160)
    cp = P["cov_par"]
    theta = np.array(list(cp.values()))
    if mode == "vi":
        obj, grad = sgp.vi_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o, g = A.eval_vi("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"])
    else:
        obj, grad = sgp.fitc_eval(cp, "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        o, g = A.eval_fitc("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"])
    _close(obj, grad, o, dict(zip(cp, np.asarray(g))), cp)
