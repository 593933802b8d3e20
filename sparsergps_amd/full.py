"""Full (non-sparse) Gaussian GP on the MI355X -- config 1 of SURVEY.md sec. 8, rank 4 of 8(f).

Host-side mirror of the reference's full-GP Gaussian path:
  obj_fun_norm_full      R/laplace_approx_obj_funs.R:56-61   (mvtnorm::dmvnorm, log = TRUE)
  dlogp_dcov_par_full    R/laplace_approx_gradient.R:1140-1269
  norm_grad_ascent_full  R/laplace_gradient_ascent.R:1700-2011
  predict_gp_full        R/laplace_approx_prediction.R:281-405
Sigma11 = k(xy, xy) + (tau^2 + delta) I is built, inverted (Gauss-Jordan, MFMA) and contracted
against dSigma11/dlog(theta) on the device (sgp_eval_full); the n x n system lives in a
SparseGPContext whose "knots" are its own rows.  Quirk kept: the gradient's alpha is
Sigma11^-1 y, not Sigma11^-1 (y - mu) (laplace_approx_gradient.R:1186).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from . import _lib
from .covariance import theta_vector
from .drivers import _ascent, _opts
from .predict import _predict
from .vi import SparseGPContext, param_names

_CTX = {}


def _ctx_for(xy, y, mu):
    xy = np.asarray(xy, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    xy = xy.reshape(y.size, -1)
    mu = np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape)
    key = (xy.shape, xy.tobytes(), y.tobytes(), mu.tobytes())
    ctx = _CTX.get(key)
    if ctx is None:
        _CTX.clear()
        ctx = SparseGPContext(xy, y, mu, m_max=y.size)
        _CTX[key] = ctx
    return ctx, xy.shape[1]


def full_eval(cov_par, cov_fun, xy, y, mu, delta=1e-6, ctx=None, obj_only=False):
    """(log dmvnorm(y; mu, Sigma11), OrderedDict d/dlog(theta) in names(cov_par) order)."""
    if ctx is None:
        ctx, d = _ctx_for(xy, y, mu)
    else:
        d = ctx.d
    lnames = [f"l{c + 1}" for c in range(d)] if cov_fun == "ard" else None
    theta = theta_vector(cov_par, cov_fun, d, lnames)
    obj, g = ctx.eval_full(theta, cov_fun, delta, obj_only)
    if obj_only:
        return obj, None
    byname = dict(zip(param_names(cov_fun, d, lnames), g))
    return obj, OrderedDict((k, float(byname[k])) for k in cov_par.keys())


def obj_fun_norm_full(cov_par, cov_fun, xy, y, mu, delta=1e-6, ctx=None):
    """R/laplace_approx_obj_funs.R:56-61 at Sigma11(cov_par)."""
    return full_eval(cov_par, cov_fun, xy, y, mu, delta, ctx, obj_only=True)[0]


def dlogp_dcov_par_full(cov_par, cov_fun, dcov_fun_dtheta=True, xy=None, y=None, mu=None,
                        transform=True, delta=1e-6, ctx=None):
    """R/laplace_approx_gradient.R:1140-1269: {"gradient", "trans_par"}."""
    if mu is None:
        mu = np.mean(np.asarray(y, dtype=np.float64))
    _, grad = full_eval(cov_par, cov_fun, xy, y, mu, delta, ctx)
    trans_par = OrderedDict((k, float(np.log(v))) for k, v in cov_par.items())
    return {"gradient": grad if dcov_fun_dtheta else 0, "trans_par": trans_par}


def norm_grad_ascent_full(cov_par_start, cov_fun, dcov_fun_dtheta=True, xy=None, y=None,
                          mu=None, opt=None, verbose=False, ctx=None):
    """R/laplace_gradient_ascent.R:1700-2011 (obj_fun = obj_fun_norm_full): the drivers'
    Adadelta / "ga" loop with one fused device evaluation per iteration."""
    o = _opts(opt)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if mu is None or (np.ndim(mu) == 0 and not np.isfinite(mu)):
        mu = np.full(y.size, y.mean())
    mu = np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape)
    if ctx is None:
        ctx, _ = _ctx_for(xy, y, mu)

    def evaluate(cov_par, _xu):
        obj, g = full_eval(cov_par, cov_fun, xy, y, mu, o["delta"], ctx)
        return obj, [g[k] for k in cov_par.keys()], None

    out = _ascent(evaluate, cov_par_start, np.zeros((1, 1)), None, bool(dcov_fun_dtheta), False,
                  o, verbose)
    return {"cov_par": out["cov_par"], "cov_fun": cov_fun, "xy": np.asarray(xy), "y": y,
            "mu": mu, "iter": out["iter"], "obj_fun": out["obj_fun"], "grad": out["grad"],
            "cov_par_history": out["cov_par_history"]}


def predict_gp_full(xy, y, x_pred, cov_fun, cov_par, mu, mu_pred, full_cov=False, delta=1e-6):
    """R/laplace_approx_prediction.R:281-405: mean mu_pred + Sigma12 Sigma22^-1 (y - mu),
    variance Sigma11 - Sigma12 Sigma22^-1 Sigma21 (diagonal unless full_cov)."""
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    xy = np.asarray(xy, dtype=np.float64).reshape(y.size, -1)
    mu = np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape)
    return _predict(_lib.SGP_PRED_FULL, True, y, None, xy, x_pred, cov_fun, cov_par, mu_pred, mu,
                    full_cov, delta)
