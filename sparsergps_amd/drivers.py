"""The reference's gradient-ascent drivers over the fused MI355X evaluation.

  norm_grad_ascent_vi  R/vi_functions.R:606-1218             (Titsias VI)
  norm_grad_ascent     R/laplace_gradient_ascent.R:1111-1693  (FITC)
  laplace_grad_ascent  R/laplace_gradient_ascent.R:10-623     (Poisson sparse Laplace)

The loop itself is host logic (a few vector operations per iteration); every iteration body --
the two K builds, the objective and the gradient the reference computes separately
(quirk Q17) -- is ONE fused device evaluation through a resident SparseGPContext (or, for
multi-GPU, a row-sharded runner from sparsergps_amd.dist).  Semantics follow the reference:
opt() defaults and unknown-name skipping, "adadelta" (with the sign-change damping
(1/eta)^s, s halved for theta but not for the knots) or "ga" updates in log-parameter space,
the bounded knot transform accumulated in transformed space, the stop rule
`iter < maxit && (any(|grad| > grad_tol) || |obj_k - obj_{k-1}| > obj_tol)`, and the knot
posterior of the final iterate.  Return values are dicts with the reference's list names.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .covariance import theta_vector
from .vi import SparseGPContext, knot_bounds, knot_fun_kind, param_names

OPT_DEFAULTS = {"optim_method": "adadelta", "decay": 0.95, "epsilon": 1e-6, "learn_rate": 1e-2,
                "eta": 1e3, "maxit": 1000, "obj_tol": 1e-3, "grad_tol": np.inf, "delta": 1e-6}


def _opts(opt, extra=None):
    o = dict(OPT_DEFAULTS)
    o.update(extra or {})
    for k, v in (opt or {}).items():
        if k in o:                       # misspelled / unused names are skipped, not errors
            o[k] = v
    if o["optim_method"] not in ("adadelta", "ga"):
        raise ValueError(f"optim_method must be 'adadelta' or 'ga', not {o['optim_method']!r}")
    return o


def _bounded(t, bounds):
    """real -> bounded knot transform (covariance_function_derivatives.R:191-197), row-wise."""
    return bounds[:, 1] / (1.0 + np.exp(-t)) + bounds[:, 0] / (1.0 + np.exp(t))


def _unbounded(xu, bounds):
    return np.log((xu - bounds[:, 0]) + 1e-4) - np.log((bounds[:, 1] - xu) + 1e-4)


class _Trace:
    def __init__(self):
        self.obj, self.grad, self.cov, self.knot_grad, self.xu = [], [], [], [], []


def _ascent(evaluate, cov_par_start, xu, xy, dtheta, dknot, o, verbose=False):
    """evaluate(cov_par OrderedDict, xu) -> (obj, grad in names order, knot_grad or None)."""
    names = list(cov_par_start.keys())
    cur = np.array([float(cov_par_start[k]) for k in names])
    xu = np.array(xu, dtype=np.float64, copy=True)
    m, d = xu.shape
    tr = _Trace()
    obj, g, gk = evaluate(OrderedDict(zip(names, cur)), xu)
    tr.obj.append(obj)
    tr.cov.append(cur.copy())
    gt = np.asarray(g, dtype=np.float64) if dtheta else np.zeros(0)
    tr.grad.append(gt if dtheta else np.full(len(names), np.nan))
    gkn = np.asarray(gk, dtype=np.float64) if dknot else np.zeros(0)
    if dknot:
        tr.knot_grad.append(gkn)
        bounds = knot_bounds(xy)
        xu_t = _unbounded(xu, bounds)
        tr.xu.append(xu.copy())
    log_t = np.log(cur)
    sg2_t, sd2_t, sc_t = (np.zeros(len(names)) for _ in range(3))
    sg2_k, sd2_k, sc_k = (np.zeros(m * d) for _ in range(3))
    it = 1
    adadelta = o["optim_method"] == "adadelta"
    while it < o["maxit"] and (
            bool(np.any(np.abs(np.concatenate([gt, gkn])) > o["grad_tol"])) or
            (abs(obj - tr.obj[it - 2]) > o["obj_tol"] if it > 1 else True)):
        it += 1
        if verbose:
            print(f"iteration {it}")
            print(np.concatenate([gt, gkn]))
        if dtheta:
            if adadelta:
                sg2_t = o["decay"] * sg2_t + (1 - o["decay"]) * gt ** 2
                step = ((1 / o["eta"]) ** sc_t) * (np.sqrt(sd2_t + o["epsilon"]) /
                                                   np.sqrt(sg2_t + o["epsilon"])) * gt
                sd2_t = o["decay"] * sd2_t + (1 - o["decay"]) * step ** 2
            else:
                step = o["learn_rate"] * gt
            log_t = log_t + step
        if dknot:
            if adadelta:
                sg2_k = o["decay"] * sg2_k + (1 - o["decay"]) * gkn ** 2
                step_k = ((1 / o["eta"]) ** sc_k) * (np.sqrt(sd2_k + o["epsilon"]) /
                                                     np.sqrt(sg2_k + o["epsilon"])) * gkn
                sd2_k = o["decay"] * sd2_k + (1 - o["decay"]) * step_k ** 2
            else:
                step_k = o["learn_rate"] * gkn
            xu_t = xu_t + step_k.reshape(m, d)          # gradient vector is row-major (Q16)
            xu = np.vstack([_bounded(xu_t[k], bounds) for k in range(m)])
            tr.xu.append(xu.copy())
        if dtheta:
            cur = np.exp(log_t)
        obj, g, gk = evaluate(OrderedDict(zip(names, cur)), xu)
        tr.obj.append(obj)
        tr.cov.append(cur.copy())
        if dtheta:
            gnew = np.asarray(g, dtype=np.float64)
            if adadelta:
                sc_t = o["decay"] * sc_t + (1 - o["decay"]) * np.abs(np.sign(gnew) - np.sign(gt)) / 2
            gt = gnew
            log_t = np.log(cur)
            tr.grad.append(gt)
        if dknot:
            gknew = np.asarray(gk, dtype=np.float64)
            if adadelta:
                sc_k = o["decay"] * sc_k + (1 - o["decay"]) * np.abs(np.sign(gknew) - np.sign(gkn))
            gkn = gknew
            tr.knot_grad.append(gkn)
    out = {"cov_par": OrderedDict(zip(names, cur)), "xu": xu, "iter": it,
           "obj_fun": np.array(tr.obj), "grad": np.array(tr.grad),
           "cov_par_history": np.array(tr.cov),
           "knot_grad": np.array(tr.knot_grad) if dknot else 0,
           "knot_history": np.stack(tr.xu, axis=2) if dknot else xu}
    return out


def _names_and_theta(cov_par, cov_fun, d):
    lnames = [f"l{c + 1}" for c in range(d)] if cov_fun == "ard" else None
    return param_names(cov_fun, d, lnames), theta_vector(cov_par, cov_fun, d, lnames)


class _Gaussian:
    """One fused VI / FITC evaluation per call on a resident context (or a row-sharded
    runner: runner.eval(theta, U, delta) -> (obj, grad in theta layout))."""

    def __init__(self, mode, cov_fun, xy, y, mu, m_max, knot_kind, knot_opt, ctx, runner,
                 delta):
        self.mode, self.cov_fun, self.delta = mode, cov_fun, delta
        self.xy = np.asarray(xy, dtype=np.float64).reshape(len(y), -1)
        self.d = self.xy.shape[1]
        self.knot_kind, self.knot_opt = knot_kind, knot_opt
        self.runner = runner
        if runner is not None:
            self.ctx = runner.backend.ctx
        else:
            self.ctx = ctx if ctx is not None else SparseGPContext(self.xy, y, mu, m_max=m_max)
            self.ctx.enable_knot_grad(knot_kind is not None)
        self.bounds = knot_bounds(self.xy)

    def __call__(self, cov_par, xu):
        names, theta = _names_and_theta(cov_par, self.cov_fun, self.d)
        if self.runner is not None:
            obj, g = self.runner.eval(theta, xu, self.delta)
        elif self.mode == "vi":
            obj, g = self.ctx.eval_vi(theta, self.cov_fun, xu, self.delta)
        else:
            obj, g = self.ctx.eval_fitc(theta, self.cov_fun, xu, self.delta)
        byname = dict(zip(names, g))
        grad = [byname[k] for k in cov_par.keys()]
        gk = None
        if self.knot_kind is not None:
            gk = self.ctx.knot_gradient(self.bounds)
            if self.knot_opt is not None:
                keep = np.zeros(xu.shape[0], dtype=bool)
                keep[np.asarray(list(self.knot_opt), dtype=int) - 1] = True
                gk = gk * np.repeat(keep, self.d)
        return obj, grad, gk


def _gaussian_driver(mode, cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot, knot_opt,
                     xu, xy, y, mu, muu, opt, verbose, ctx, runner):
    o = _opts(opt)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    xu = np.asarray(xu, dtype=np.float64).reshape(-1, np.asarray(xy).reshape(len(y), -1).shape[1])
    if mu is None or (np.ndim(mu) == 0 and not np.isfinite(mu)):
        mu = np.full(y.size, y.mean())                                  # quirk Q14
    if muu is None or (np.ndim(muu) == 0 and not np.isfinite(muu)):
        muu = np.full(xu.shape[0], y.mean())
    mu = np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape)
    kind = knot_fun_kind(dcov_fun_dknot)
    ev = _Gaussian(mode, cov_fun, xy, y, mu, xu.shape[0], kind,
                   knot_opt, ctx, runner, o["delta"])
    out = _ascent(ev, cov_par_start, xu, ev.xy, bool(dcov_fun_dtheta), kind is not None, o,
                  verbose)
    u_mean, u_var = ev.ctx.posterior_u(np.broadcast_to(np.asarray(muu, dtype=np.float64),
                                                       (xu.shape[0],)))
    out.update({"cov_fun": cov_fun, "xy": ev.xy, "mu": mu, "muu": muu, "u_mean": u_mean,
                "u_var": u_var})
    return out


def norm_grad_ascent_vi(cov_par_start, cov_fun, dcov_fun_dtheta=True, dcov_fun_dknot=None,
                        knot_opt=None, xu=None, xy=None, y=None, mu=None, muu=None, opt=None,
                        verbose=False, ctx=None, runner=None):
    """R/vi_functions.R:606-1218: Titsias-ELBO gradient ascent (obj_fun = elbo_fun)."""
    return _gaussian_driver("vi", cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot,
                            knot_opt, xu, xy, y, mu, muu, opt, verbose, ctx, runner)


def norm_grad_ascent(cov_par_start, cov_fun, dcov_fun_dtheta=True, dcov_fun_dknot=None,
                     knot_opt=None, xu=None, xy=None, y=None, mu=None, muu=None, opt=None,
                     verbose=False, ctx=None, runner=None):
    """R/laplace_gradient_ascent.R:1111-1693: FITC gradient ascent (obj_fun_norm)."""
    return _gaussian_driver("fitc", cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot,
                            knot_opt, xu, xy, y, mu, muu, opt, verbose, ctx, runner)


def laplace_grad_ascent(cov_par_start, cov_fun, dcov_fun_dtheta=True, dcov_fun_dknot=None,
                        knot_opt=None, xu=None, xy=None, y=None, ff=None, mu=None, muu=None,
                        m=1.0, opt=None, verbose=False, ctx=None):
    """R/laplace_gradient_ascent.R:10-623 for the Poisson likelihood: every iteration is
    newtrap_sparseGP warm-started from the previous mode (resident on the device) followed by
    dlogq_dcov_par at the new mode, as one fused evaluation (sgp_eval_laplace)."""
    o = _opts(opt, {"maxit_nr": 1000, "tol_nr": 1e-6})
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    xy_m = np.asarray(xy, dtype=np.float64).reshape(len(y), -1)
    d = xy_m.shape[1]
    xu = np.asarray(xu, dtype=np.float64).reshape(-1, d)
    mu = np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape)
    muu = np.broadcast_to(np.asarray(muu, dtype=np.float64), (xu.shape[0],))
    kind = knot_fun_kind(dcov_fun_dknot)
    if ctx is None:
        ctx = SparseGPContext(xy_m, y, mu, m_max=xu.shape[0])
    ctx.enable_knot_grad(kind is not None)
    ctx.lap_set_f(ff)
    bounds = knot_bounds(xy_m)
    nr_iter = []

    def evaluate(cov_par, U):
        names, theta = _names_and_theta(cov_par, cov_fun, d)
        obj, g, it = ctx.eval_laplace(theta, cov_fun, U, o["delta"], m, o["tol_nr"],
                                      o["maxit_nr"])
        nr_iter.append(it)
        byname = dict(zip(names, g))
        gk = None
        if kind is not None:
            gk = ctx.knot_gradient(bounds)
            if knot_opt is not None:
                keep = np.zeros(U.shape[0], dtype=bool)
                keep[np.asarray(list(knot_opt), dtype=int) - 1] = True
                gk = gk * np.repeat(keep, d)
        return obj, [byname[k] for k in cov_par.keys()], gk

    out = _ascent(evaluate, cov_par_start, xu, xy_m, bool(dcov_fun_dtheta), kind is not None, o,
                  verbose)
    u_mean, u_var = ctx.posterior_u(muu)
    out.update({"cov_fun": cov_fun, "xy": xy_m, "mu": mu, "muu": muu, "fmax": ctx.lap_get_f(),
                "u_mean": u_mean, "u_var": u_var, "nr_iter": np.array(nr_iter)})
    return out
