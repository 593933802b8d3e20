"""GPU parity of the optimizer drivers: sparsergps_amd.norm_grad_ascent_vi / norm_grad_ascent /
laplace_grad_ascent (one fused HIP evaluation per iteration) vs the oracle's literal
restatement of the R drivers (oracle/drivers.py) over a few iterations: objective trajectory,
parameter path, gradients, knot path and the final knot posterior."""
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


def _close(a, b, rtol=RTOL, atol=1e-9):
    np.testing.assert_allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64),
                               rtol=rtol, atol=atol)


@pytest.mark.parametrize("mode,cov_fun,knots", [("vi", "sqexp", None), ("vi", "sqexp", "sqexp"),
                                                ("fitc", "ard", None), ("fitc", "sqexp", "sqexp")])
def test_gaussian_drivers_match_oracle(sgp, mode, cov_fun, knots):
    P = O.make_gaussian_problem("C2", n=240, m=12)
    cp = P["cov_par"]
    if cov_fun == "ard":
        cp = OrderedDict([("sigma", 1.0), ("l1", 1.0), ("l2", 1.3), ("l3", 0.8), ("tau", 0.5)])
    opt = {"maxit": 5, "obj_tol": 0.0}
    mu = np.full(P["y"].size, P["y"].mean())
    muu = np.full(P["U"].shape[0], P["y"].mean())
    ref_fn = OD.norm_grad_ascent_vi if mode == "vi" else OD.norm_grad_ascent
    fn = sgp.norm_grad_ascent_vi if mode == "vi" else sgp.norm_grad_ascent
    ref = ref_fn(cp, cov_fun, P["U"], P["X"], P["y"], mu, muu, dcov_fun_dknot=knots, opt=opt)
    got = fn(cp, cov_fun, True, knots, None, P["U"], P["X"], P["y"], mu, muu, opt)
    assert got["iter"] == ref["iter"] == 5
    _close(got["obj_fun"], ref["obj_fun"])
    _close(got["cov_par_history"], ref["cov_par_history"])
    _close(got["grad"], ref["grad"], atol=1e-7)
    _close(got["u_mean"], ref["u_mean"], atol=1e-7)
    _close(got["u_var"], ref["u_var"], atol=1e-7)
    if knots:
        _close(got["knot_history"], ref["knot_history"])
        _close(got["knot_grad"], ref["knot_grad"], atol=1e-6)


def test_laplace_driver_matches_oracle(sgp):
    P = O.make_poisson_problem(n=300, m=10)
    opt = {"maxit": 4, "obj_tol": 0.0, "tol_nr": 1e-5}
    muu = np.full(P["U"].shape[0], P["mu"][0])
    ref = OD.laplace_grad_ascent(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], P["f0"],
                                 P["mu"], muu, P["a"], opt=opt)
    got = sgp.laplace_grad_ascent(P["cov_par"], "sqexp", True, None, None, P["U"], P["X"],
                                  P["y"], P["f0"], P["mu"], muu, P["a"], opt)
    assert got["iter"] == ref["iter"] == 4
    assert list(got["nr_iter"]) == list(ref["nr_iter"])
    _close(got["obj_fun"], ref["obj_fun"])
    _close(got["cov_par_history"], ref["cov_par_history"])
    _close(got["grad"], ref["grad"], atol=1e-7)
    _close(got["fmax"], ref["fmax"], atol=1e-7)
    _close(got["u_mean"], ref["u_mean"], atol=1e-7)
    _close(got["u_var"], ref["u_var"], atol=1e-7)
