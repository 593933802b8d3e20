"""GPU parity on the committed golden fixtures and at BASELINE.json's configs' own shapes.

* Every tests/golden/*.npz fixture (inputs + oracle outputs frozen by
  tests/golden/make_golden.py; checked against the live oracle by test_oracle.py) is
  evaluated through the HIP path here, so the GPU box checks frozen vectors, not only a live
  recomputation: the Layer-1 fills at 1e-12, VI / FITC / Poisson-Laplace objective and
  gradient at the north-star 1e-6 relative bar (NR: iteration count exact, every objective
  value 1e-9).
* C2 (configs[1]: sqexp, d = 3) at its own m = 256 and C5 (configs[4]: Poisson, d = 5) at
  its own m = 512 -- from the fixtures at n = 2000 (literal oracle) and at larger n against
  the adjoint models (C2 at its full n = 1e5 against oracle/adjoint_chunked.py; C5 at
  n = 40 000 against oracle/adjoint_ref.py and at 5e5 against adjoint_chunked; FITC at the
  C3 shape against adjoint_chunked.eval_fitc).
"""
import glob
import os
from collections import OrderedDict

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
EVAL_RTOL = 1e-6
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def sgp():
    import sparsergps_amd as S
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return S


def _cp(z):
    return OrderedDict(zip([str(s) for s in z["names"]], z["theta"]))


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))


GAUSS = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLD, "gauss_*.npz")))
POIS = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLD, "poisson_*.npz")))


def test_fixture_lists_cover_own_knot_counts():
    assert "gauss_c2_m256.npz" in GAUSS and "poisson_c5_m512.npz" in POIS
    assert "poisson_c5_expo.npz" in POIS


@pytest.mark.parametrize("name", GAUSS)
def test_golden_gaussian_vi_fitc(sgp, name):
    z = np.load(os.path.join(GOLD, name))
    cp, cf = _cp(z), str(z["cov_fun"])
    args = (cp, cf, z["U"], z["X"], z["y"], z["mu"], float(z["delta"]))
    obj, grad = sgp.vi_eval(*args)
    assert abs(obj - float(z["vi_obj"])) / abs(float(z["vi_obj"])) < EVAL_RTOL
    assert _rel(list(grad.values()), z["vi_grad"]) < EVAL_RTOL
    obj, grad = sgp.fitc_eval(*args)
    assert abs(obj - float(z["fitc_obj"])) / abs(float(z["fitc_obj"])) < EVAL_RTOL
    assert _rel(list(grad.values()), z["fitc_grad"]) < EVAL_RTOL


@pytest.mark.parametrize("name", POIS)
def test_golden_poisson_laplace(sgp, name):
    z = np.load(os.path.join(GOLD, name))
    cp = _cp(z)
    a = z["a"] if z["a"].ndim else float(z["a"])   # poisson_c5_expo: one exposure per row
    r = sgp.laplace_eval(cp, "sqexp", z["U"], z["X"], z["y"], z["mu"], z["f0"], a,
                         float(z["delta"]), tol=1e-5)
    tr = z["obj_trace"]
    assert r["nr_iter"] == len(tr)
    np.testing.assert_allclose(r["objective_function_values"], tr, rtol=1e-9)
    assert np.max(np.abs(r["gp"] - z["ff"])) < 1e-8
    assert _rel(list(r["gradient"].values()), z["grad"]) < EVAL_RTOL


def test_golden_fills(sgp):
    z = np.load(os.path.join(GOLD, "fills.npz"))
    x, xp = z["x"], z["xp"]
    cp = {"sigma": 1.3, "l": 1.7, "tau": 0.4}
    cpa = {"sigma": 0.9, "l1": 0.8, "l2": 1.5, "l3": 2.2, "tau": 0.3}
    ln = ["l1", "l2", "l3"]
    for f in ("sqexp", "exp"):
        np.testing.assert_allclose(sgp.make_cov_matC(x, None, cp, f, 1e-6), z[f"cov_{f}_sym"], rtol=1e-12)
        np.testing.assert_allclose(sgp.make_cov_matC(x, xp, cp, f, 1e-6), z[f"cov_{f}_cross"], rtol=1e-12)
        for p in ("sigma", "l", "tau"):
            np.testing.assert_allclose(sgp.dsig_dthetaC(x, None, cp, f, p), z[f"d_{f}_{p}_sym"],
                                       rtol=1e-12, atol=1e-300)
            np.testing.assert_allclose(sgp.dsig_dthetaC(x, xp, cp, f, p), z[f"d_{f}_{p}_cross"],
                                       rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(sgp.make_cov_mat_ardC(x, None, cpa, "ard", 1e-6, ln), z["cov_ard_sym"], rtol=1e-12)
    np.testing.assert_allclose(sgp.make_cov_mat_ardC(x, xp, cpa, "ard", 1e-6, ln), z["cov_ard_cross"], rtol=1e-12)
    for p in ("sigma", "l1", "l2", "l3", "tau"):
        np.testing.assert_allclose(sgp.dsig_dtheta_ardC(x, None, cpa, "ard", p, ln), z[f"d_ard_{p}_sym"],
                                   rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose(sgp.dsig_dtheta_ardC(x, xp, cpa, "ard", p, ln), z[f"d_ard_{p}_cross"],
                                   rtol=1e-12, atol=1e-300)


def test_c2_full_n_against_chunked_adjoint_model(sgp):
    """configs[1] exactly: n = 1e5, m = 256, d = 3, sqexp (VI)."""
    from oracle import adjoint_chunked as AC
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C2")
    assert P["X"].shape == (100_000, 3) and P["U"].shape == (256, 3)
    th = np.array(list(P["cov_par"].values()))
    o, g = AC.eval_vi("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["delta"])
    obj, grad = sgp.vi_eval(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], P["mu"], P["delta"])
    assert abs(obj - o) / abs(o) < 1e-9
    assert _rel(list(grad.values()), g) < 1e-7


def test_c5_own_knot_count_against_adjoint_model(sgp):
    """configs[4]'s m = 512, d = 5 Poisson Laplace at n = 40 000 (warm NR from f0)."""
    from oracle import adjoint_ref as A
    from sparsergps_amd.workloads import make_poisson_problem
    P = make_poisson_problem(n=40_000)
    assert P["U"].shape == (512, 5)
    th = np.array(list(P["cov_par"].values()))
    o, g, f, it = A.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"], P["a"],
                                 P["delta"], tol=1e-5)
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=512) as ctx:
        ctx.lap_set_f(P["f0"])
        obj, grad, nit = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        fg = ctx.lap_get_f()
    assert nit == it
    assert abs(obj - o) / abs(o) < 1e-9
    assert np.max(np.abs(fg - f)) < 1e-8
    assert _rel(grad, g) < 1e-7


def test_c5_full_size_against_chunked_laplace_model(sgp):
    """configs[4] exactly (the Laplace bench workload): n = 5e5, m = 512, d = 5, sqexp Poisson,
    NR from f0 = log mean(y) to the stop rule, then dlogq_dcov_par at the mode -- against the
    row-chunked CPU model of the same algebra (oracle/adjoint_chunked.eval_laplace, pinned to
    the literal newtrap_sparseGP + dlogq_dcov_par in tests/test_oracle.py; ~15-30 s of host
    BLAS).  NR count exact, every NR objective to 1e-9, the mode to 1e-8, the gradient to 1e-7.
    Reference: R/newtrap_sparseGP.R:6-186, R/laplace_approx_gradient.R:25-553."""
    from oracle import adjoint_chunked as AC
    from sparsergps_amd.workloads import make_poisson_problem
    P = make_poisson_problem()
    assert P["X"].shape == (500_000, 5) and P["U"].shape == (512, 5)
    th = np.array(list(P["cov_par"].values()))
    o, g, f, objs = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"], P["a"],
                                    P["delta"], tol=1e-5)
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=512) as ctx:
        ctx.lap_set_f(P["f0"])
        obj, grad, nit = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        fg = ctx.lap_get_f()
        ov = ctx.lap_objective_values()
    assert nit == len(objs) == len(ov)
    np.testing.assert_allclose(ov, objs, rtol=1e-9, atol=0)
    assert abs(obj - o) / abs(o) < 1e-9
    assert np.max(np.abs(fg - f)) < 1e-8
    assert _rel(grad, g) < 1e-7


def test_c5_full_size_per_row_exposure_against_chunked_laplace_model(sgp):
    """configs[4]'s shape with the exposure `m` as one value per row (a vector of cell areas,
    R/derivative_functions_of_data_likelihoods.R:7-61; optimize_gp.R:461-468 passes `a` through
    unchanged): the resident exposure (sgp_lap_set_expo, expo = SGP_EXPO_ROWS) against
    adjoint_chunked.eval_laplace with the same vector (pinned to the literal oracle with per-row
    exposure in tests/test_oracle.py).  NR count exact, NR objectives 1e-9, mode 1e-8, gradient
    1e-7; then a scalar evaluation on the same context ignores the resident vector."""
    from oracle import adjoint_chunked as AC
    from sparsergps_amd.workloads import make_poisson_problem
    P = make_poisson_problem(per_row_exposure=True)
    assert P["X"].shape == (500_000, 5) and np.ndim(P["a"]) == 1
    th = np.array(list(P["cov_par"].values()))
    o, g, f, objs = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"], P["a"],
                                    P["delta"], tol=1e-5)
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=512) as ctx:
        ctx.lap_set_f(P["f0"])
        obj, grad, nit = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        fg = ctx.lap_get_f()
        ov = ctx.lap_objective_values()
        assert nit == len(objs) == len(ov)
        np.testing.assert_allclose(ov, objs, rtol=1e-9, atol=0)
        assert abs(obj - o) / abs(o) < 1e-9
        assert np.max(np.abs(fg - f)) < 1e-8
        assert _rel(grad, g) < 1e-7
        # a positive scalar still means that exposure on every row (resident vector unused)
        ctx.lap_set_f(P["f0"][:1].repeat(P["X"].shape[0]))
        o1, _, _ = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], 1.0, 1e-5, 1000)
        o1c, _, _, _ = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"],
                                       P["f0"][:1].repeat(P["X"].shape[0]), 1.0, P["delta"],
                                       tol=1e-5)
        assert abs(o1 - o1c) / abs(o1c) < 1e-9


def test_c3_headline_shape_against_chunked_adjoint_model(sgp):
    """configs[2] exactly (the bench workload): n = 1e6, m = 1024, d = 8, ARD -- the product
    path against the row-chunked CPU model of the same adjoint algebra (~15-40 s of host
    BLAS), i.e. parity at the headline size, not only at reduced n."""
    from oracle import adjoint_chunked as AC
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C3")
    assert P["X"].shape == (1_000_000, 8) and P["U"].shape == (1024, 8)
    th = np.array(list(P["cov_par"].values()))
    obj, grad = sgp.vi_eval(P["cov_par"], "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
    o, g = AC.eval_vi("ard", th, P["X"], P["y"], P["mu"], P["U"], P["delta"])
    assert abs(obj - o) / abs(o) < 1e-9
    assert _rel(list(grad.values()), g) < 1e-7


def test_fitc_headline_shape_against_chunked_fitc_model(sgp):
    """The FITC bench workload (--mode fitc: configs[2]'s n = 1e6, m = 1024, d = 8, ARD) against
    the row-chunked CPU model (oracle/adjoint_chunked.eval_fitc, pinned to the literal
    obj_fun_norm + dlogp_dcov_par in tests/test_oracle.py; ~30 s of host BLAS).  Exercises the
    t-carrying and signed-weight SYRKs on the balanced plan at their production split counts.
    Reference: R/laplace_approx_obj_funs.R:6, R/laplace_approx_gradient.R:720-971."""
    from oracle import adjoint_chunked as AC
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C3")
    assert P["X"].shape == (1_000_000, 8) and P["U"].shape == (1024, 8)
    th = np.array(list(P["cov_par"].values()))
    obj, grad = sgp.fitc_eval(P["cov_par"], "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
    o, g = AC.eval_fitc("ard", th, P["X"], P["y"], P["mu"], P["U"], P["delta"])
    assert abs(obj - o) / abs(o) < 1e-9
    assert _rel(list(grad.values()), g) < 1e-7


@pytest.mark.parametrize("m,n,cov", [(600, 60_000, "ard"), (384, 40_000, "sqexp"), (1100, 30_000, "ard")])
def test_fitc_balanced_plans_against_chunked_fitc_model(sgp, m, n, cov):
    """FITC's t-carrying and signed-weight SYRKs at other balanced-plan shapes (nb = 5, 3 and 9
    128-tiles; the nb = 4 / 8 shapes are the C5 / C3 tests above) against the row-chunked
    FITC model.  Reference: R/laplace_approx_obj_funs.R:6, R/laplace_approx_gradient.R:720-971."""
    from oracle import adjoint_chunked as AC
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C3" if cov == "ard" else "C2", n=n, m=m)
    th = np.array(list(P["cov_par"].values()))
    obj, grad = sgp.fitc_eval(P["cov_par"], cov, P["U"], P["X"], P["y"], P["mu"], P["delta"])
    o, g = AC.eval_fitc(cov, th, P["X"], P["y"], P["mu"], P["U"], P["delta"])
    assert abs(obj - o) / abs(o) < 1e-9
    assert _rel(list(grad.values()), g) < 1e-7


@pytest.mark.parametrize("m,n", [(384, 30_000), (640, 20_000)])
def test_laplace_balanced_plans_against_chunked_laplace_model(sgp, m, n):
    """The Laplace NR objectives (sqrt(w) SYRK with t on the balanced plan), S_a (signed) and the
    streamed Newton passes at nb = 3 and 5 against the row-chunked Laplace model."""
    from oracle import adjoint_chunked as AC
    from sparsergps_amd.workloads import make_poisson_problem
    P = make_poisson_problem(n=n, m=m)
    th = np.array(list(P["cov_par"].values()))
    o, g, f, objs = AC.eval_laplace("sqexp", th, P["X"], P["y"], P["mu"], P["U"], P["f0"], P["a"],
                                    P["delta"], tol=1e-5)
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m) as ctx:
        ctx.lap_set_f(P["f0"])
        obj, grad, nit = ctx.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
        ov = ctx.lap_objective_values()
    assert nit == len(objs) == len(ov)
    np.testing.assert_allclose(ov, objs, rtol=1e-9, atol=0)
    assert abs(obj - o) / abs(o) < 1e-9
    assert _rel(grad, g) < 1e-7
