"""GPU parity for the objective-only evaluations (SGP_FLAG_OBJ_ONLY: elbo_fun, obj_fun_norm,
newtrap_sparseGP without the gradient) and for the FITC / Laplace OAT candidate scoring
(knot_prop_random_norm / knot_prop_random, R/knot_proposal_functions.R:1176-1363, 1001-1173)
against the literal oracle at the augmented knot sets [U; x*]."""
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


@pytest.mark.parametrize("cfg,n,m", [("C2", 300, 20), ("C3", 400, 24), ("C2", 500, 130)])
def test_obj_only_equals_full_objective(sgp, cfg, n, m):
    P = O.make_gaussian_problem(cfg, n=n, m=m)
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m) as ctx:
        ctx.enable_knot_grad(True)
        for ev in (ctx.eval_vi, ctx.eval_fitc):
            full, g = ev(th, P["cov_fun"], P["U"], P["delta"])
            assert g is not None and np.all(np.isfinite(g))
            ctx.knot_gradient()                        # available after a full evaluation
            o, g2 = ev(th, P["cov_fun"], P["U"], P["delta"], obj_only=True)
            assert g2 is None
            assert abs(o - full) <= 1e-13 * abs(full), (ev.__name__, o, full)
            with pytest.raises(sgp.SGPError):          # no stale knot gradient after obj-only
                ctx.knot_gradient()
    ref_vi = O.elbo_eval(P["cov_par"], P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])
    got = sgp.elbo_fun(P["cov_par"], P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])
    assert abs(got - ref_vi) / abs(ref_vi) < EVAL_RTOL


@pytest.mark.parametrize("cfg,n,m,T", [("C2", 300, 20, 5), ("C3", 350, 16, 4), ("C2", 260, 127, 3)])
def test_fitc_candidates_match_oracle(sgp, cfg, n, m, T):
    P = O.make_gaussian_problem(cfg, n=n, m=m)
    rng = np.random.default_rng(11)
    cand = P["X"][rng.choice(n, size=T, replace=False)]
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m + 1) as ctx:
        got = ctx.fitc_candidates(th, P["cov_fun"], P["U"], cand, P["delta"])
        # the candidate loop leaves the context usable at the original knots
        base, _ = ctx.eval_fitc(th, P["cov_fun"], P["U"], P["delta"])
    for t in range(T):
        ref = O.fitc_obj_eval(P["cov_par"], P["cov_fun"], np.vstack([P["U"], cand[t]]), P["X"],
                              P["y"], P["mu"], P["delta"])
        assert abs(got[t] - ref) / abs(ref) < EVAL_RTOL, (t, got[t], ref)
    ref0 = O.fitc_obj_eval(P["cov_par"], P["cov_fun"], P["U"], P["X"], P["y"], P["mu"], P["delta"])
    assert abs(base - ref0) / abs(ref0) < EVAL_RTOL


def test_candidates_need_room_for_one_more_knot(sgp):
    P = O.make_gaussian_problem("C2", n=200, m=10)
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=10) as ctx:
        with pytest.raises(sgp.SGPError):
            ctx.fitc_candidates(th, P["cov_fun"], P["U"], P["X"][:2], P["delta"])


def _poisson(n, m):
    return O.make_poisson_problem(n=n, m=m)


@pytest.mark.parametrize("n,m", [(300, 20), (420, 33)])
def test_lap_nr_matches_oracle_newtrap(sgp, n, m):
    P = _poisson(n, m)
    nr = O.newtrap_sparseGP(P["f0"], P["cov_par"], P["cov_fun"], P["X"], P["U"], P["y"], P["mu"],
                            P["a"], P["delta"], tol=1e-5)
    r = sgp.newtrap_sparseGP(P["f0"], P["cov_par"], P["cov_fun"], P["X"], P["U"], P["y"],
                             P["mu"], P["a"], P["delta"], tol=1e-5)
    ov = nr["objective_function_values"]
    np.testing.assert_allclose(r["objective_function_values"], ov, rtol=1e-9)
    assert np.max(np.abs(r["gp"] - nr["gp"])) < 1e-8
    o = sgp.obj_fun_pois(nr["gp"], P["cov_par"], P["cov_fun"], P["U"], P["X"], P["y"], P["mu"],
                         P["a"], P["delta"])
    s12, s22, Z = O.laplace_mats(P["cov_par"], P["cov_fun"], P["U"], P["X"], P["delta"])
    ref = O.obj_fun_pois(nr["gp"], P["mu"], Z, s12, s22, P["y"], P["a"])
    assert abs(o - ref) / abs(ref) < EVAL_RTOL


@pytest.mark.parametrize("n,m,T", [(300, 20, 4), (380, 12, 3)])
def test_lap_candidates_match_oracle(sgp, n, m, T):
    P = _poisson(n, m)
    rng = np.random.default_rng(5)
    cand = P["X"][rng.choice(n, size=T, replace=False)]
    th = np.array(list(P["cov_par"].values()))
    # the fit's mode at the current knots is the warm start of every candidate
    fmax = O.newtrap_sparseGP(P["f0"], P["cov_par"], P["cov_fun"], P["X"], P["U"], P["y"],
                              P["mu"], P["a"], P["delta"], tol=1e-5)["gp"]
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m + 1) as ctx:
        ctx.lap_set_f(fmax)
        got = ctx.lap_candidates(th, P["cov_fun"], P["U"], cand, P["delta"], P["a"], 1e-5, 1000)
        f_after = ctx.lap_get_f()
    assert np.array_equal(f_after, fmax)                # the resident f is restored
    for t in range(T):
        ref = O.newtrap_sparseGP(fmax, P["cov_par"], P["cov_fun"], P["X"],
                                 np.vstack([P["U"], cand[t]]), P["y"], P["mu"], P["a"],
                                 P["delta"], tol=1e-5)["objective_function_values"][-1]
        assert abs(got[t] - ref) / abs(ref) < EVAL_RTOL, (t, got[t], ref)
