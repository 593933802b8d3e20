"""Reference-named covariance fillers on the MI355X (Layer 1 of include/sgp.h).

Mirrors the Rcpp exports of luisdamiano/sparseRGPs:
  make_cov_matC     src/covariance_functionsC.cpp:72-169
  make_cov_mat_ardC src/covariance_functionsC.cpp:191-252
  dsig_dthetaC      src/covariance_function_derivativesC.cpp:307-552
  dsig_dtheta_ardC  src/covariance_function_derivativesC.cpp:555-722
  cov_fun_sqrd_expC / cov_fun_sqrd_exp_ardC / cov_fun_expC (covariance_functionsC.cpp:5-52)
Same argument meaning and error behaviour: ``x_pred=None`` (or a 1x1 NaN matrix, R's
``matrix()``) selects the symmetric mode, an invalid covariance function or parameter name
returns a 0x0 matrix after printing the reference's message to stderr.  Computation runs in
HIP kernels; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

from . import _lib

_THETA_SCALARS = ("sigma", "tau")


def _device():
    return int(os.environ.get("SGP_DEVICE", "0"))


def _is_sym(x_pred):
    if x_pred is None:
        return True
    xp = np.asarray(x_pred, dtype=np.float64)
    return xp.size >= 1 and bool(np.isnan(xp.reshape(-1)[0]))


def _mat(x):
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        x = x.reshape(-1, 1)
    return np.asfortranarray(x)


def theta_vector(cov_par, kernel, d, lnames=None, need_tau=True):
    """[sigma, l (or l_1..l_d read by lnames), tau] in the layout of include/sgp.h."""
    if kernel == "ard":
        lnames = list(lnames) if lnames is not None else [f"l{c + 1}" for c in range(d)]
        ls = [float(cov_par[nm]) for nm in lnames[:d]]
    else:
        ls = [float(cov_par["l"])]
    tau = float(cov_par["tau"]) if (need_tau or "tau" in cov_par) else 0.0
    return np.array([float(cov_par["sigma"])] + ls + [tau], dtype=np.float64)


def _rcerr(msg):
    print(msg, file=sys.stderr, end="")


def _fill(kind, x, x_pred, cov_par, kernel, delta, param, d, lnames):
    lib = _lib.lib()
    _lib.require_gpu()
    x = _mat(x)
    sym = _is_sym(x_pred)
    theta = theta_vector(cov_par, kernel, d, lnames, need_tau=sym or param == "tau")
    n = x.shape[0]
    if sym:
        xp, npr, pxp, ldxp = None, n, None, n
    else:
        xp = _mat(x_pred)
        npr = xp.shape[0]
        pxp, ldxp = _lib.dptr(xp), npr
    out = np.empty((n, npr), dtype=np.float64, order="F")
    kid = _lib.KERNELS[kernel]
    if kind == "cov":
        st = lib.sgp_make_cov(_device(), kid, _lib.dptr(x), n, n, pxp, npr, ldxp, d,
                              _lib.dptr(theta), float(delta), _lib.dptr(out), n)
    else:
        st = lib.sgp_dsig_dtheta(_device(), kid, _lib.dptr(x), n, n, pxp, npr, ldxp, d,
                                 _lib.dptr(theta), int(param), _lib.dptr(out), n)
    _lib.check(st)
    return out


def make_cov_matC(x, x_pred, cov_par, cov_fun, delta):
    """covariance_functionsC.cpp:72-169 ("sqexp" or "exp")."""
    if cov_fun not in ("sqexp", "exp"):
        _rcerr("Error: invalid covariance function")
        return np.zeros((0, 0))
    x = _mat(x)
    return _fill("cov", x, x_pred, cov_par, cov_fun, delta, None, x.shape[1], None)


def make_cov_mat_ardC(x, x_pred, cov_par, cov_fun, delta, lnames):
    """covariance_functionsC.cpp:191-252 ("ard" only)."""
    if cov_fun != "ard":
        _rcerr("Error: invalid covariance function")
        return np.zeros((0, 0))
    x = _mat(x)
    return _fill("cov", x, x_pred, cov_par, "ard", delta, None, x.shape[1], lnames)


def dsig_dthetaC(x, x_pred, cov_par, cov_fun, par_name):
    """covariance_function_derivativesC.cpp:307-552: d Sigma / d log(par_name)."""
    x = _mat(x)
    sym = _is_sym(x_pred)
    idx = {"sigma": 0, "l": 1, "tau": 2}.get(par_name)
    if cov_fun == "sqexp":
        if idx is None:
            _rcerr("Error: invalid covariance function" if sym else
                   "Error: invalid parameter name for chosen covariance function")
            return np.zeros((0, 0))
    elif cov_fun == "exp":
        if not sym and idx in (None, 2):
            # `return mat;` before the tau branch (l.520): a zero matrix (quirk Q13)
            return np.zeros((x.shape[0], _mat(x_pred).shape[0]), order="F")
        if idx is None:
            _rcerr("Error")
            return np.zeros((0, 0))
    else:
        _rcerr("Error: invalid covariance function")
        return np.zeros((0, 0))
    return _fill("dcov", x, x_pred, cov_par, cov_fun, 0.0, idx, x.shape[1], None)


def dsig_dtheta_ardC(x, x_pred, cov_par, cov_fun, par_name, lnames):
    """covariance_function_derivativesC.cpp:555-722 (ARD)."""
    x = _mat(x)
    sym = _is_sym(x_pred)
    if cov_fun != "ard":
        _rcerr("Error: invalid covariance function")
        return np.zeros((0, 0))
    d = x.shape[1]
    lnames = list(lnames)
    if par_name == "sigma":
        idx = 0
    elif par_name in lnames:
        idx = 1 + lnames.index(par_name)
    elif par_name == "tau":
        idx = d + 1
    else:
        _rcerr("Error" if sym else "Error: invalid parameter name for chosen covariance function")
        return np.zeros((0, 0))
    return _fill("dcov", x, x_pred, cov_par, "ard", 0.0, idx, d, lnames)


def _pair(kernel, x1, x2, theta, param=None):
    lib = _lib.lib()
    a = np.ascontiguousarray(np.asarray(x1, dtype=np.float64).reshape(-1))
    b = np.ascontiguousarray(np.asarray(x2, dtype=np.float64).reshape(-1))
    if param is None:
        return lib.sgp_kernel_pair(_lib.KERNELS[kernel], _lib.dptr(a), _lib.dptr(b), a.size,
                                   _lib.dptr(theta))
    return lib.sgp_dkernel_pair(_lib.KERNELS[kernel], _lib.dptr(a), _lib.dptr(b), a.size,
                                _lib.dptr(theta), int(param))


def cov_fun_sqrd_expC(x1, x2, cov_par):
    """covariance_functionsC.cpp:5-12."""
    return _pair("sqexp", x1, x2, theta_vector(cov_par, "sqexp", 1, need_tau=False))


def cov_fun_sqrd_exp_ardC(x1, x2, cov_par, lnames):
    """covariance_functionsC.cpp:16-42."""
    d = np.asarray(x1).size
    return _pair("ard", x1, x2, theta_vector(cov_par, "ard", d, lnames, need_tau=False))


def cov_fun_expC(x1, x2, cov_par):
    """covariance_functionsC.cpp:45-52 (L1 distance)."""
    return _pair("exp", x1, x2, theta_vector(cov_par, "exp", 1, need_tau=False))
