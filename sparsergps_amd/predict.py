"""Sparse prediction on the MI355X.

Host-side mirror of the reference's prediction functions:
  predict_vi       R/vi_functions.R:1222-1333
  predict_laplace  R/laplace_approx_prediction.R:3-123   (FITC and Poisson-Laplace fits)
  predict_gp       R/laplace_approx_prediction.R:408-542 (dispatcher; sparse fits and the
                   full Gaussian GP via sparsergps_amd.full.predict_gp_full)
The knot posterior (u_mean, u_var) that these consume comes from
``SparseGPContext.posterior_u`` (the drivers' end-of-fit computation).  K(x_pred, xu), the
m x m solves and the per-row variance quadratic forms run in libsgp.so (sgp_predict).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .covariance import theta_vector
from .vi import _device


def _predict(method, gaussian, u_mean, u_var, xu, x_pred, cov_fun, cov_par, mu, muu, full_cov,
             delta):
    lib = _lib.lib()
    _lib.require_gpu()
    x_pred = np.asarray(x_pred, dtype=np.float64)
    if x_pred.ndim == 1:
        x_pred = x_pred.reshape(-1, 1)
    xp = np.asfortranarray(x_pred)
    npred, d = xp.shape
    U = np.asfortranarray(np.asarray(xu, dtype=np.float64).reshape(-1, d))
    m = U.shape[0]
    lnames = [f"l{c + 1}" for c in range(d)] if cov_fun == "ard" else None
    theta = np.ascontiguousarray(theta_vector(cov_par, cov_fun, d, lnames))
    um = np.ascontiguousarray(np.asarray(u_mean, dtype=np.float64).reshape(-1))
    mu_u = np.ascontiguousarray(np.broadcast_to(np.asarray(muu, dtype=np.float64), (m,)))
    uv = (None if u_var is None
          else np.asfortranarray(np.asarray(u_var, dtype=np.float64).reshape(m, m)))
    mu_p = np.ascontiguousarray(np.broadcast_to(np.asarray(mu, dtype=np.float64), (npred,)))
    pm = np.zeros(npred, dtype=np.float64)
    pv = np.zeros((npred, npred) if full_cov else npred, dtype=np.float64, order="F")
    _lib.check(lib.sgp_predict(_device(), _lib.KERNELS[cov_fun], _lib.dptr(theta), float(delta),
                               method, 1 if gaussian else 0, _lib.dptr(U), m, m, _lib.dptr(um),
                               _lib.dptr(mu_u), None if uv is None else _lib.dptr(uv), m,
                               _lib.dptr(xp), npred, npred, d,
                               _lib.dptr(mu_p), 1 if full_cov else 0, _lib.dptr(pm),
                               _lib.dptr(pv), npred))
    return {"pred_mean": pm.reshape(-1, 1), "pred_var": pv}


def predict_vi(u_mean, u_var, xu, x_pred, cov_fun, cov_par, mu, muu, full_cov=False,
               family="gaussian", delta=1e-6):
    """R/vi_functions.R:1222-1333; only the gaussian family (the reference returns an error
    string otherwise, l.1263-1267 -- here: SGPError)."""
    return _predict(_lib.SGP_PRED_VI, family == "gaussian", u_mean, u_var, xu, x_pred, cov_fun,
                    cov_par, mu, muu, full_cov, delta)


def predict_laplace(u_mean, u_var, xu, x_pred, cov_fun, cov_par, mu, muu, full_cov=False,
                    family="gaussian", delta=1e-6):
    """R/laplace_approx_prediction.R:3-123."""
    return _predict(_lib.SGP_PRED_LAPLACE, family == "gaussian", u_mean, u_var, xu, x_pred,
                    cov_fun, cov_par, mu, muu, full_cov, delta)


def predict_gp(mod, x_pred, mu_pred=None, full_cov=False, vi=False):
    """R/laplace_approx_prediction.R:408-542 for sparse fits.  `mod` mirrors the reference's
    fit object: {"family", "sparse", "delta", "results": {"u_mean", "u_var", "xu", "cov_fun",
    "cov_par", "muu"}}."""
    family = mod["family"]
    res = mod["results"]
    delta = mod.get("delta", 1e-6)
    if vi and family != "gaussian":
        return "Error: VI not supported for non-gaussian data."
    inv_link = {"poisson": np.exp, "bernoulli": lambda x: 1 / (1 + np.exp(-x))}.get(family)
    x_pred = np.asarray(x_pred, dtype=np.float64)
    if x_pred.ndim == 1:
        print("Warning: x_pred must be a matrix. I'll try to make the conversion.")
        x_pred = x_pred.reshape(-1, 1)
    if mu_pred is None or np.any(np.isnan(np.asarray(mu_pred, dtype=np.float64))):
        print("Warnings: you did not define the mean of the GP at locations at which you wish "
              "to make predictions. Setting the mean to be zero.")
        mu_pred = np.zeros(x_pred.shape[0])
    if not mod.get("sparse", True):
        if family != "gaussian":
            raise NotImplementedError("predict_laplace_full (full-GP Poisson / Bernoulli fits) "
                                      "is outside this build's scope (DESIGN.md sec. 8)")
        from .full import predict_gp_full
        pred = predict_gp_full(res["xy"], res["y"], x_pred, res["cov_fun"], res["cov_par"],
                               res["mu"], mu_pred, full_cov, delta)
        return {"pred": pred, "sparse": False, "family": family, "x_pred": x_pred,
                "inverse_link": inv_link}
    m = np.asarray(res["xu"]).shape[0]
    if vi:
        pred = predict_vi(res["u_mean"], res["u_var"], res["xu"], x_pred, res["cov_fun"],
                          res["cov_par"], mu_pred, res["muu"], full_cov, family, delta)
    else:
        pred = predict_laplace(np.asarray(res["u_mean"])[:m], res["u_var"], res["xu"], x_pred,
                               res["cov_fun"], res["cov_par"], mu_pred,
                               np.asarray(res["muu"])[:m], full_cov, family, delta)
    return {"pred": pred, "sparse": True, "family": family, "x_pred": x_pred,
            "inverse_link": inv_link}
