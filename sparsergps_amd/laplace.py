"""Poisson sparse-Laplace evaluation on the MI355X (config 5 of SURVEY.md sec. 8).

Host-side mirror of the reference's Laplace hot path (luisdamiano/sparseRGPs):
  newtrap_sparseGP        R/newtrap_sparseGP.R:6-186 (+ _update 234-325)
  obj_fun_pois            R/laplace_approx_obj_funs.R:108-174
  dlogq_dcov_par          R/laplace_approx_gradient.R:25-553   (knots fixed)
  d{1,2,3}log_py_dff_pois R/derivative_functions_of_data_likelihoods.R:7-61
with K22 = k(xu, xu) + (tau^2 + delta) I (quirk Q1) and Z the FITC diagonal.  One call of
``laplace_eval`` is one iteration body of laplace_grad_ascent
(R/laplace_gradient_ascent.R:510-541): NR warm-started from the previous mode, then the
gradient at the new mode.  All work runs in libsgp.so (no CPU fallback); the mode f stays
resident on the device between calls.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .covariance import theta_vector
from .vi import _context_for, _knot_outputs, knot_fun_kind, param_names


def _prep(cov_par, cov_fun, xu, xy):
    xy_m = np.asarray(xy, dtype=np.float64)
    d = 1 if xy_m.ndim == 1 else xy_m.shape[1]
    lnames = [f"l{c + 1}" for c in range(d)] if cov_fun == "ard" else None
    theta = theta_vector(cov_par, cov_fun, d, lnames)
    names = param_names(cov_fun, d, lnames)
    xu_m = np.asarray(xu, dtype=np.float64).reshape(-1, d)
    return theta, names, xu_m


def _mu_vec(mu, y):
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if mu is None:
        mu = np.log(np.mean(y))          # poisson-regression-vignette.Rmd:92
    return np.ascontiguousarray(np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape))


def laplace_eval(cov_par, cov_fun, xu, xy, y, mu, ff=None, m=1.0, delta=1e-6, tol=1e-5,
                 maxit=1000, ctx=None):
    """NR to the Laplace mode from `ff` (or the context's resident mode when ff is None), then
    dlogq_dcov_par there.  Returns dict(objective, gradient (names(cov_par) order), gp,
    objective_function_values, nr_iter)."""
    # newtrap_sparseGP.R:79-96 runs the first update whatever maxit is
    return _eval(cov_par, cov_fun, xu, xy, y, mu, ff, m, delta, tol, max(int(maxit), 1), ctx)


def _eval(cov_par, cov_fun, xu, xy, y, mu, ff, m, delta, tol, maxit, ctx):
    """laplace_eval with the C ABI's maxit as given (0 = objective and gradient at f, no NR)."""
    theta, names, xu_m = _prep(cov_par, cov_fun, xu, xy)
    muv = _mu_vec(mu, y)
    if ctx is None:
        ctx = _context_for(xy, y, mu, xu_m.shape[0], muv)
        ctx.set_data(y, muv)
    if ff is not None:
        ctx.lap_set_f(ff)
    obj, g, it = ctx.eval_laplace(theta, cov_fun, xu_m, delta, m, tol, maxit)
    byname = dict(zip(names, g))
    return {"objective": obj,
            "gradient": OrderedDict((k, float(byname[k])) for k in cov_par.keys()),
            "gp": ctx.lap_get_f(),
            "objective_function_values": ctx.lap_objective_values(),
            "nr_iter": it}


def _lap_ctx(cov_par, cov_fun, xu, xy, y, mu, ctx):
    theta, names, xu_m = _prep(cov_par, cov_fun, xu, xy)
    if ctx is None:
        muv = _mu_vec(mu, y)
        ctx = _context_for(xy, y, mu, xu_m.shape[0], muv)
        ctx.set_data(y, muv)
    return ctx, theta, xu_m


def newtrap_sparseGP(start_vals, cov_par, cov_fun, xy, xu, y, mu, m=1.0, delta=1e-6,
                     maxit=1000, tol=1e-6, ctx=None):
    """R/newtrap_sparseGP.R:6-186 for the Poisson likelihood: {"gp",
    "objective_function_values", "gradient"} (sgp_lap_nr: the NR loop alone, no gradient work;
    "gradient" is grad psi of the last NR step, as the reference returns it, l.183-184)."""
    ctx, theta, xu_m = _lap_ctx(cov_par, cov_fun, xu, xy, y, mu, ctx)
    if start_vals is not None:
        ctx.lap_set_f(start_vals)
    ctx.lap_nr(theta, cov_fun, xu_m, delta, m, tol, max(int(maxit), 1))   # first update always
    return {"gp": ctx.lap_get_f(), "objective_function_values": ctx.lap_objective_values(),
            "gradient": ctx.lap_get_grad_psi()}


def dlogq_dcov_par(cov_par, cov_fun, dcov_fun_dtheta=True, dcov_fun_dknot=None, knot_opt=None,
                   xu=None, xy=None, y=None, ff=None, mu=None, m=1.0, delta=1e-6,
                   transform=True, ctx=None):
    """R/laplace_approx_gradient.R:25-553 at the given ff (no NR step): {"gradient",
    "trans_par"}."""
    kind = knot_fun_kind(dcov_fun_dknot)
    theta, names, xu_m = _prep(cov_par, cov_fun, xu, xy)
    if ctx is None:
        muv = _mu_vec(mu, y)
        ctx = _context_for(xy, y, mu, xu_m.shape[0], muv)
        ctx.set_data(y, muv)
    ctx.enable_knot_grad(kind is not None)
    r = _eval(cov_par, cov_fun, xu, xy, y, mu, ff, m, delta, 0.0, 0, ctx)   # no NR step
    grad = r["gradient"] if dcov_fun_dtheta else 0
    trans_par = OrderedDict((k, float(np.log(v))) for k, v in cov_par.items())
    if kind is not None:
        gk, tk = _knot_outputs(ctx, xu_m, xy, knot_opt)
        return {"gradient": grad, "knot_gradient": gk, "trans_par": trans_par, "trans_knot": tk}
    return {"gradient": grad, "trans_par": trans_par}


def obj_fun_pois(ff, cov_par, cov_fun, xu, xy, y, mu, m=1.0, delta=1e-6, ctx=None):
    """R/laplace_approx_obj_funs.R:108-174 at ff (log q(y | theta, xu, ff))."""
    ctx, theta, xu_m = _lap_ctx(cov_par, cov_fun, xu, xy, y, mu, ctx)
    if ff is not None:
        ctx.lap_set_f(ff)
    return ctx.lap_nr(theta, cov_fun, xu_m, delta, m, 0.0, 0)[0]
