"""Optimizer-driver logic (norm_grad_ascent_vi, norm_grad_ascent, laplace_grad_ascent) on CPU:
the product loop sparsergps_amd.drivers._ascent, fed the oracle's objective/gradient, must
retrace the oracle's literal restatement of the R drivers (oracle/drivers.py) step for step:
Adadelta with sign-change damping, "ga", the knot transform and the stop rule."""
from collections import OrderedDict

import numpy as np
import pytest

from oracle import drivers as OD
from oracle import sgp_oracle as O
from sparsergps_amd import drivers as D


def _oracle_eval(mode, cov_fun, xy, y, mu, dl, knot_kind):
    def ev(cp, U):
        if mode == "vi":
            obj = O.elbo_eval(cp, cov_fun, U, xy, y, mu, dl)
            r = O.delbo_dcov_par(cp, cov_fun, U, xy, y, mu, dl, knot_kind)
        else:
            obj = O.fitc_obj_eval(cp, cov_fun, U, xy, y, mu, dl)
            r = O.dlogp_dcov_par(cp, cov_fun, U, xy, y, mu, dl, knot_kind)
        return obj, [r["gradient"][k] for k in cp], r.get("knot_gradient")
    return ev


@pytest.mark.parametrize("mode,cov_fun,knots,method", [
    ("vi", "sqexp", None, "adadelta"), ("vi", "ard", None, "ga"),
    ("fitc", "sqexp", None, "adadelta"), ("vi", "sqexp", "sqexp", "adadelta"),
    ("fitc", "sqexp", "sqexp", "ga")])
def test_ascent_loop_matches_oracle_driver(mode, cov_fun, knots, method):
    P = O.make_gaussian_problem("C2", n=60, m=5)
    cp = P["cov_par"]
    if cov_fun == "ard":
        cp = OrderedDict([("sigma", 1.0), ("l1", 1.0), ("l2", 1.3), ("l3", 0.8), ("tau", 0.5)])
    opt = {"maxit": 6, "optim_method": method, "learn_rate": 1e-3, "obj_tol": 0.0}
    mu = np.full(P["y"].size, P["y"].mean())
    fn = OD.norm_grad_ascent_vi if mode == "vi" else OD.norm_grad_ascent
    ref = fn(cp, cov_fun, P["U"], P["X"], P["y"], mu, dcov_fun_dknot=knots, opt=opt)
    got = D._ascent(_oracle_eval(mode, cov_fun, P["X"], P["y"], mu, 1e-6, knots), cp, P["U"],
                    P["X"], True, knots is not None, D._opts(opt))
    assert got["iter"] == ref["iter"] == 6
    np.testing.assert_allclose(got["obj_fun"], ref["obj_fun"], rtol=1e-12)
    np.testing.assert_allclose(got["cov_par_history"], ref["cov_par_history"], rtol=1e-12)
    np.testing.assert_allclose(got["grad"], ref["grad"], rtol=1e-10, atol=1e-12)
    if knots:
        np.testing.assert_allclose(got["knot_history"], ref["knot_history"], rtol=1e-12)
        np.testing.assert_allclose(got["knot_grad"], ref["knot_grad"], rtol=1e-10, atol=1e-12)


def test_stop_rule_and_opt_defaults():
    o = D._opts({"maxit": 3, "not_an_option": 1})
    assert o["maxit"] == 3 and "not_an_option" not in o and o["grad_tol"] == np.inf
    with pytest.raises(ValueError):
        D._opts({"optim_method": "newton"})
    calls = []

    def ev(cp, U):                      # a flat objective stops after the first update
        calls.append(1)
        return 1.0, [0.1, 0.1, 0.1], None
    cp = OrderedDict([("sigma", 1.0), ("l", 1.0), ("tau", 0.5)])
    out = D._ascent(ev, cp, np.zeros((2, 1)), np.zeros((3, 1)), True, False, D._opts({}))
    assert out["iter"] == 2 and len(calls) == 2
