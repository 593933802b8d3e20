"""GPU parity for the Poisson sparse-Laplace path (newtrap_sparseGP + dlogq_dcov_par) vs the
CPU oracle.  The NR iteration count must match exactly (same stop rule on the same values);
objective and gradient are held to the north-star 1e-6 relative bar."""
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


def _problem(n, m, cov_fun="sqexp", coinc=False):
    P = O.make_poisson_problem(n=n, m=m)
    U = P["U"].copy()
    if coinc:
        U[:2] = P["X"][[3, n - 1]]
    P["U"] = U
    if cov_fun == "ard":
        P["cov_par"] = OrderedDict([("sigma", 1.1)] + [(f"l{c + 1}", 1.5 + 0.3 * c) for c in range(5)]
                                   + [("tau", 0.2)])
    P["cov_fun"] = cov_fun
    return P


def _oracle(P, ff, tol):
    nr = O.newtrap_sparseGP(ff, P["cov_par"], P["cov_fun"], P["X"], P["U"], P["y"], P["mu"],
                            P["a"], P["delta"], tol=tol)
    g = O.dlogq_dcov_par(P["cov_par"], P["cov_fun"], P["U"], P["X"], P["y"], nr["gp"], P["mu"],
                         P["a"], P["delta"])["gradient"]
    return nr, g


@pytest.mark.parametrize("n,m,cov_fun,coinc", [(300, 20, "sqexp", False), (400, 30, "sqexp", True),
                                               (350, 25, "ard", True), (257, 1, "sqexp", False),
                                               (900, 130, "sqexp", False)])
def test_laplace_matches_oracle(sgp, n, m, cov_fun, coinc):
    P = _problem(n, m, cov_fun, coinc)
    nr, g = _oracle(P, P["f0"], 1e-5)
    r = sgp.laplace_eval(P["cov_par"], cov_fun, P["U"], P["X"], P["y"], P["mu"], P["f0"], P["a"],
                         P["delta"], tol=1e-5)
    ov = nr["objective_function_values"]
    assert r["nr_iter"] == len(ov)
    np.testing.assert_allclose(r["objective_function_values"], ov, rtol=1e-9)
    assert np.max(np.abs(r["gp"] - nr["gp"])) < 1e-8
    assert abs(r["objective"] - ov[-1]) / abs(ov[-1]) < EVAL_RTOL
    for k in P["cov_par"]:
        assert abs(r["gradient"][k] - g[k]) / max(1.0, abs(g[k])) < EVAL_RTOL, (k, r["gradient"][k], g[k])


@pytest.mark.parametrize("maxit", [2, 1000])
def test_newtrap_returns_grad_psi(sgp, maxit):
    """newtrap_sparseGP's `gradient` element: grad psi of the last NR step, i.e. at the f that
    step started from (R/newtrap_sparseGP.R:97-104, 183-184).  maxit = 2 stops after the first
    update (grad psi at f0, O(1) values); maxit = 1000 runs to the stop rule."""
    P = _problem(300, 20)
    nr = O.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], P["U"], P["y"], P["mu"],
                            P["a"], P["delta"], maxit=maxit, tol=1e-5)
    got = sgp.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], P["U"], P["y"], P["mu"],
                               P["a"], P["delta"], maxit=maxit, tol=1e-5)
    assert len(got["objective_function_values"]) == len(nr["objective_function_values"])
    g_ref = nr["gradient"]
    if maxit == 2:
        assert np.max(np.abs(g_ref)) > 0.1
        np.testing.assert_allclose(got["gradient"], g_ref, rtol=1e-9, atol=1e-12)
    else:
        # at the mode: |grad psi| <= tol, compared absolutely (f agrees to ~1e-9)
        assert np.max(np.abs(got["gradient"] - g_ref)) < 1e-8


def test_dlogq_and_obj_at_given_ff(sgp):
    """maxit = 0: no NR step, the gradient and objective at the supplied f (not a mode)."""
    P = _problem(320, 24)
    ff = P["f0"] + 0.1 * np.sin(np.arange(320))
    res = sgp.dlogq_dcov_par(P["cov_par"], "sqexp", True, None, None, P["U"], P["X"], P["y"], ff,
                             P["mu"], P["a"], P["delta"])
    g = O.dlogq_dcov_par(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], ff, P["mu"], P["a"],
                         P["delta"])["gradient"]
    for k in P["cov_par"]:
        assert abs(res["gradient"][k] - g[k]) / max(1.0, abs(g[k])) < EVAL_RTOL
    s12, s22, Z = O.laplace_mats(P["cov_par"], "sqexp", P["U"], P["X"], P["delta"])
    o = O.obj_fun_pois(ff, P["mu"], Z, s12, s22, P["y"], P["a"])
    got = sgp.obj_fun_pois(ff, P["cov_par"], "sqexp", P["U"], P["X"], P["y"], P["mu"], P["a"],
                           P["delta"])
    assert abs(got - o) / abs(o) < 1e-10


def test_warm_start_sequence(sgp):
    """Two driver iterations at different theta: the second NR starts from the resident mode
    (laplace_gradient_ascent.R:510-519)."""
    P = _problem(500, 40)
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=40) as ctx:
        ctx.lap_set_f(P["f0"])
        o1, g1, it1 = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        f1 = ctx.lap_get_f()
        th2 = th * np.array([1.05, 0.97, 1.1])
        o2, g2, it2 = ctx.eval_laplace(th2, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
    cp2 = OrderedDict(zip(P["cov_par"].keys(), th2))
    P2 = dict(P, cov_par=cp2)
    nr, g = _oracle(P2, f1, 1e-5)
    assert it2 == len(nr["objective_function_values"]) and it2 <= it1
    assert abs(o2 - nr["objective_function_values"][-1]) / abs(o2) < EVAL_RTOL
    gv = np.array(list(g.values()))
    assert np.max(np.abs(g2 - gv) / np.maximum(1, np.abs(gv))) < EVAL_RTOL


def test_laplace_larger_against_adjoint_model(sgp):
    from oracle import adjoint_ref as A
    P = _problem(6000, 256)
    th = np.array(list(P["cov_par"].values()))
    o, g, f, it = A.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"], P["a"],
                                 P["delta"], tol=1e-5)
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=256) as ctx:
        ctx.lap_set_f(P["f0"])
        obj, grad, nit = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        fg = ctx.lap_get_f()
    assert nit == it
    assert abs(obj - o) / abs(o) < 1e-10
    assert np.max(np.abs(fg - f)) < 1e-9
    assert np.max(np.abs(grad - g) / np.maximum(1, np.abs(g))) < 1e-8


def test_dlogq_mu_omitted_defaults_to_log_mean(sgp):
    """mu=None (no ctx): the Laplace entry points fall back to log(mean(y))
    (poisson-regression-vignette.Rmd:92), cached under their own context key."""
    P = _problem(310, 22)
    ff = P["f0"] + 0.05 * np.cos(np.arange(310))
    res = sgp.dlogq_dcov_par(P["cov_par"], "sqexp", True, None, None, P["U"], P["X"], P["y"], ff,
                             None, P["a"], P["delta"])
    g = O.dlogq_dcov_par(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], ff,
                         np.full(310, np.log(P["y"].mean())), P["a"], P["delta"])["gradient"]
    for k in P["cov_par"]:
        assert abs(res["gradient"][k] - g[k]) / max(1.0, abs(g[k])) < EVAL_RTOL
    o = sgp.obj_fun_pois(ff, P["cov_par"], "sqexp", P["U"], P["X"], P["y"], None, P["a"], P["delta"])
    s12, s22, Z = O.laplace_mats(P["cov_par"], "sqexp", P["U"], P["X"], P["delta"])
    o_ref = O.obj_fun_pois(ff, np.full(310, np.log(P["y"].mean())), Z, s12, s22, P["y"], P["a"])
    assert abs(o - o_ref) / abs(o_ref) < 1e-10


def test_mu_none_defaults_do_not_share_a_context(sgp):
    """A Laplace call with mu=None (log mean(y)) followed by VI / FITC calls with mu=None
    (mean(y), quirk Q14) on the same arrays: each path uses its own default mean."""
    P = _problem(300, 20)
    X, y = P["X"], P["y"].astype(np.float64)
    sgp.obj_fun_pois(P["f0"], P["cov_par"], "sqexp", P["U"], X, y, None, P["a"], P["delta"])
    mu_vi = np.full(len(y), y.mean())
    o_vi, g_vi = sgp.vi_eval(P["cov_par"], "sqexp", P["U"], X, y, None, P["delta"])
    o_ref = O.elbo_eval(P["cov_par"], "sqexp", P["U"], X, y, mu_vi, P["delta"])
    assert abs(o_vi - o_ref) / abs(o_ref) < EVAL_RTOL
    o_fitc, _ = sgp.fitc_eval(P["cov_par"], "sqexp", P["U"], X, y, None, P["delta"])
    o_fitc_ref, _ = sgp.fitc_eval(P["cov_par"], "sqexp", P["U"], X, y, y.mean(), P["delta"])
    assert abs(o_fitc - o_fitc_ref) / abs(o_fitc_ref) < 1e-12
    # and back: the Laplace default is still log mean(y)
    o = sgp.obj_fun_pois(P["f0"], P["cov_par"], "sqexp", P["U"], X, y, None, P["a"], P["delta"])
    s12, s22, Z = O.laplace_mats(P["cov_par"], "sqexp", P["U"], X, P["delta"])
    o_ref = O.obj_fun_pois(P["f0"], np.full(len(y), np.log(y.mean())), Z, s12, s22, y, P["a"])
    assert abs(o - o_ref) / abs(o_ref) < 1e-10


def test_grad_psi_invalid_after_maxit0_eval(sgp):
    """sgp_lap_get_grad_psi refers to the last NR run: after an NR run followed by a maxit = 0
    evaluation (no NR step) it reports SGP_EINVAL instead of the earlier run's values."""
    from sparsergps_amd import _lib
    P = _problem(300, 20)
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=20) as ctx:
        ctx.lap_set_f(P["f0"])
        ctx.lap_nr(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        ctx.lap_get_grad_psi()
        ctx.eval_laplace(th * 1.1, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 0)
        with pytest.raises(_lib.SGPError):
            ctx.lap_get_grad_psi()


@pytest.mark.parametrize("first", ["vi", "fitc"])
def test_abandoned_phase1_then_laplace(sgp, first):
    """A VI / FITC evaluation begun (phase 1, other knots) and never finished, then a Laplace
    evaluation on the same context: the abandoned evaluation's queued K22 chain must not race
    the new one's knot upload and resets (sgp_lap_begin drains it first)."""
    import torch
    P = _problem(400, 30)
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=64) as ctx:
        if first == "vi":
            red1 = torch.zeros(ctx.vi_red1_count(30), dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            ctx.vi_phase1(th, "sqexp", P["U"] + 0.3, P["delta"], red1.data_ptr())
        else:
            red1 = torch.zeros(ctx.fitc_red1_count(30), dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            ctx.fitc_phase1(th, "sqexp", P["U"] + 0.3, P["delta"], red1.data_ptr())
        ctx.lap_set_f(P["f0"])
        obj, grad, it = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        torch.cuda.synchronize()
    nr, g = _oracle(P, P["f0"], 1e-5)
    assert it == len(nr["objective_function_values"])
    assert abs(obj - nr["objective_function_values"][-1]) / abs(obj) < EVAL_RTOL
    gv = np.array(list(g.values()))
    assert np.max(np.abs(grad - gv) / np.maximum(1, np.abs(gv))) < EVAL_RTOL
