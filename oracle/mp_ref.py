"""50-digit mpmath restatement of the three objectives -- TEST INFRASTRUCTURE ONLY.

The third independent pin of the oracle that SURVEY.md 4 / 8(c) prescribes ("mpmath 50-digit
evaluation at n <= 16").  It shares no code with ``oracle/sgp_oracle.py``: every objective is
written in its dense n x n form (no Woodbury identity, no Cholesky factor of K22 + K21 Z^-1 K12,
no LU solves with n right-hand sides) and every gradient is mpmath's own numerical derivative
(``mp.diff``) of that objective in log(theta), taken at 50 significant digits.  Only
``tests/`` may import it.

What each dense form restates (reference file:line):
  * VI (Titsias) -- ``elbo_fun`` R/vi_functions.R:64-121 with ``trace_term_fun`` 14-27 as
    driven by ``norm_grad_ascent_vi`` (K22 = Kuu + delta I, Z = tau^2 + delta, l.733-753):
      log N(y - mu; 0, Q + Z I) - (n (sigma^2 + delta) - tr Q) / (2 tau^2),
      Q = K12 K22^-1 K21.
  * FITC -- ``obj_fun_norm`` R/laplace_approx_obj_funs.R:6-52 with Z as in
    ``norm_grad_ascent`` R/laplace_gradient_ascent.R:1238-1263:
      log N(y - mu; 0, Q + diag(Z)),  Z_i = sigma^2 + tau^2 + delta - Q_ii.
  * Poisson sparse Laplace -- ``obj_fun_pois`` R/laplace_approx_obj_funs.R:108-174 at the mode
    of ``newtrap_sparseGP`` R/newtrap_sparseGP.R:6-186 (K22 = Kuu + (tau^2 + delta) I, l.43-60):
      log p(y | f) - 1/2 (f - mu)' S^-1 (f - mu) - 1/2 log det(I + W S),
      S = Q + diag(Z), W = diag(a e^f), f = argmax of the first two terms (Newton to 50 digits).

The reference's tau derivative treats a data row that equals a knot exactly as if K12 carried
the nugget there (dK12/dlog tau = 2 tau^2 on such pairs, Q5:
covariance_function_derivativesC.cpp:157-163) while K12 itself has none (cross mode,
covariance_functionsC.cpp:108-113).  The "reference-implied" objective used for the tau
derivative therefore adds (tau^2 - tau0^2) on coincident pairs of K12, which leaves its value at
tau0 unchanged; VI's trace term keeps K12 at tau0 (its tau derivative is -2 T,
vi_functions.R:38-44, with no coincidence term).
"""
from __future__ import annotations

from collections import OrderedDict

import mpmath as mp

DPS = 50


def _mat(a):
    """numpy 2-D array (or nested list) -> mp.matrix at the current precision."""
    rows = [[mp.mpf(float(v)) for v in row] for row in a]
    return mp.matrix(rows)


def _vec(a):
    return mp.matrix([mp.mpf(float(v)) for v in a])


def _lnames(cov_fun, d):
    return [f"l{c + 1}" for c in range(d)] if cov_fun == "ard" else None


def _kern(x, u, th, cov_fun, d):
    """sqexp: sigma^2 exp(-|x-u|^2 / (2 l^2)) (covariance_functionsC.cpp:10);
    ard: sigma^2 exp(-sum ((x_c - u_c)/l_c)^2 / 2) (l.40)."""
    s = mp.mpf(0)
    for c in range(d):
        l = th["l"] if cov_fun == "sqexp" else th[f"l{c + 1}"]
        s += ((x[c] - u[c]) / l) ** 2
    return th["sigma"] ** 2 * mp.exp(-s / 2)


def _rows(M):
    return [[M[i, j] for j in range(M.cols)] for i in range(M.rows)]


def _cross(X, U, th, cov_fun, coinc=None, tau0=None):
    n, m, d = X.rows, U.rows, X.cols
    K = mp.matrix(n, m)
    for i in range(n):
        xi = [X[i, c] for c in range(d)]
        for j in range(m):
            K[i, j] = _kern(xi, [U[j, c] for c in range(d)], th, cov_fun, d)
            if coinc is not None and coinc[i][j]:
                K[i, j] += th["tau"] ** 2 - tau0 ** 2
    return K


def _coinc(X, U):
    return [[all(X[i, c] == U[j, c] for c in range(X.cols)) for j in range(U.rows)]
            for i in range(X.rows)]


def _logpdf(r, S):
    n = S.rows
    L = mp.cholesky(S)
    logdet = 2 * mp.fsum(mp.log(L[i, i]) for i in range(n))
    w = mp.lu_solve(S, r)
    quad = mp.fsum(r[i] * w[i] for i in range(n))
    return -quad / 2 - logdet / 2 - n * mp.log(2 * mp.pi) / 2


def _q_matrix(K12, K22):
    """Q = K12 K22^-1 K21 (dense)."""
    return K12 * mp.inverse(K22) * K12.T


def _theta(cov_par):
    return OrderedDict((k, mp.mpf(float(v))) for k, v in cov_par.items())


def vi_objective(th, cov_fun, X, U, r, delta, tau0=None, coinc=None):
    n, m = X.rows, U.rows
    d = X.cols
    K12 = _cross(X, U, th, cov_fun, coinc, tau0)
    K12t = K12 if coinc is None else _cross(X, U, dict(th, tau=tau0), cov_fun)
    K22 = _cross(U, U, th, cov_fun) + delta * mp.eye(m)
    z = th["tau"] ** 2 + delta
    S = _q_matrix(K12, K22) + z * mp.eye(n)
    Qt = _q_matrix(K12t, K22)
    trQ = mp.fsum(Qt[i, i] for i in range(n))
    T = -(n * (th["sigma"] ** 2 + delta) - trQ) / (2 * th["tau"] ** 2)
    return _logpdf(r, S) + T


def fitc_objective(th, cov_fun, X, U, r, delta, tau0=None, coinc=None):
    n, m = X.rows, U.rows
    K12 = _cross(X, U, th, cov_fun, coinc, tau0)
    K22 = _cross(U, U, th, cov_fun) + delta * mp.eye(m)
    Q = _q_matrix(K12, K22)
    S = Q.copy()
    for i in range(n):
        S[i, i] = th["sigma"] ** 2 + th["tau"] ** 2 + delta     # Q_ii + Z_i
    return _logpdf(r, S)


def _laplace_sigma(th, cov_fun, X, U, delta, tau0=None, coinc=None):
    n, m = X.rows, U.rows
    K12 = _cross(X, U, th, cov_fun, coinc, tau0)
    K22 = _cross(U, U, th, cov_fun) + (th["tau"] ** 2 + delta) * mp.eye(m)
    S = _q_matrix(K12, K22)
    for i in range(n):
        S[i, i] = th["sigma"] ** 2 + th["tau"] ** 2 + delta
    return S


def laplace_mode(S, y, mu, a, f0=None, tol=None):
    """argmax_f log p(y|f) - 1/2 (f-mu)' S^-1 (f-mu) by Newton at the working precision."""
    n = S.rows
    Si = mp.inverse(S)
    f = mp.matrix([mu[i] for i in range(n)]) if f0 is None else f0.copy()
    tol = tol if tol is not None else mp.mpf(10) ** (-(mp.mp.dps - 5))
    for _ in range(200):
        e = [a * mp.exp(f[i]) for i in range(n)]
        g = mp.matrix([y[i] - e[i] for i in range(n)]) - Si * (f - mu)
        H = Si.copy()
        for i in range(n):
            H[i, i] += e[i]
        step = mp.lu_solve(H, g)
        f = f + step
        if mp.norm(step, mp.inf) < tol:
            break
    else:
        raise RuntimeError("mpmath Newton did not converge")
    return f


def laplace_objective_at(S, f, y, mu, a):
    n = S.rows
    lp = mp.fsum(y[i] * mp.log(a) - mp.loggamma(y[i] + 1) - a * mp.exp(f[i]) + y[i] * f[i]
                 for i in range(n))
    rf = f - mu
    quad = mp.fsum(rf[i] * v for i, v in enumerate(mp.lu_solve(S, rf)))
    Wm = mp.matrix(n, n)
    for i in range(n):
        Wm[i, i] = a * mp.exp(f[i])
    B = mp.eye(n) + Wm * S
    return lp - quad / 2 - mp.log(mp.det(B)) / 2


def laplace_objective(th, cov_fun, X, U, y, mu, a, delta, tau0=None, coinc=None, f0=None):
    S = _laplace_sigma(th, cov_fun, X, U, delta, tau0, coinc)
    f = laplace_mode(S, y, mu, a, f0)
    return laplace_objective_at(S, f, y, mu, a), f


def _dK12(X, U, th, cov_fun, k, coinc):
    """dK12/dlog theta_k (covariance_function_derivativesC.cpp: sigma 2K l.47/78, sqexp l
    K |x-u|^2/l^2 l.98-99, ard l_c K ((x_c-u_c)/l_c)^2 l.133-134, tau 2 tau^2 on coincident
    pairs l.157-163)."""
    n, m, d = X.rows, U.rows, X.cols
    D = mp.matrix(n, m)
    for i in range(n):
        for j in range(m):
            kij = _kern([X[i, c] for c in range(d)], [U[j, c] for c in range(d)], th, cov_fun, d)
            if k == "sigma":
                D[i, j] = 2 * kij
            elif k == "tau":
                D[i, j] = 2 * th["tau"] ** 2 if coinc[i][j] else 0
            elif k == "l":
                D[i, j] = kij * mp.fsum((X[i, c] - U[j, c]) ** 2 for c in range(d)) / th["l"] ** 2
            else:
                c = int(k[1:]) - 1
                D[i, j] = kij * ((X[i, c] - U[j, c]) / th[k]) ** 2
    return D


def laplace_comp3_correction(th, cov_fun, X, U, y, a, delta, f, k, coinc):
    """grad_reference - d/dlog theta_k of the Laplace objective at the mode.

    The reference's comp3_1 (laplace_approx_gradient.R:308-310) takes d(Sigma g) with the
    term K12 K22^-1 dK21 g written as dK12 K22^-1 K21 g (``2 * dSigma12 %*% GG``), so its
    gradient differs from the objective's derivative by
        -1/2 (comp4 * (-W3))' L(dv),  dv = dK12 K22^-1 K21 g - K12 K22^-1 dK21 g,
    L(v) = comp3's operator (l.314-315) = -(1/W) (S - 1/W)^-1 v,
    comp4 = diag((S^-1 - W)^-1) (l.155-178), W = W3 = -a e^f, g = y - a e^f.  Zero for sigma
    (dK12 = 2 K12) and for tau without coincident pairs; the length scales carry it.
    """
    n, m = X.rows, U.rows
    K12 = _cross(X, U, th, cov_fun)
    K22 = _cross(U, U, th, cov_fun) + (th["tau"] ** 2 + delta) * mp.eye(m)
    K22i = mp.inverse(K22)
    S = _laplace_sigma(th, cov_fun, X, U, delta)
    W = [-a * mp.exp(f[i]) for i in range(n)]
    g = mp.matrix([y[i] + W[i] for i in range(n)])
    dK = _dK12(X, U, th, cov_fun, k, coinc)
    dv = dK * (K22i * (K12.T * g)) - K12 * (K22i * (dK.T * g))
    Sw = S.copy()
    for i in range(n):
        Sw[i, i] -= 1 / W[i]
    Lv = mp.lu_solve(Sw, dv)
    Si = mp.inverse(S)
    for i in range(n):
        Si[i, i] -= W[i]
    c4 = mp.inverse(Si)
    return -mp.fsum(c4[i, i] * (-W[i]) * (-Lv[i] / W[i]) for i in range(n)) / 2


def _with(th, k, logv):
    t = OrderedDict(th)
    t[k] = mp.exp(logv)
    return t


def evaluate(kind, cov_par, cov_fun, X, U, y, mu, delta=1e-6, a=1.0, dps=DPS):
    """Objective and d/dlog(theta) (names(cov_par) order) at `dps` digits.

    kind: "vi" | "fitc" | "laplace".  Returns (obj, OrderedDict grad[, mode f]) as mpf; the
    Laplace call also returns the mode so the fp64 oracle can be evaluated at the same f.
    """
    with mp.workdps(dps):
        Xm, Um = _mat(X), _mat(U)
        th0 = _theta(cov_par)
        dl = mp.mpf(float(delta))
        coinc = _coinc(Xm, Um)
        any_c = any(any(row) for row in coinc)
        tau0 = th0["tau"]
        if kind == "laplace":
            yv, muv, am = _vec(y), _vec(mu), mp.mpf(float(a))
            obj, fhat = laplace_objective(th0, cov_fun, Xm, Um, yv, muv, am, dl)

            def F(th, cz):
                return laplace_objective(th, cov_fun, Xm, Um, yv, muv, am, dl, tau0,
                                         cz, fhat)[0]
        else:
            r = _vec(y) - _vec(mu)
            fn = vi_objective if kind == "vi" else fitc_objective

            def F(th, cz):
                return fn(th, cov_fun, Xm, Um, r, dl, tau0, cz)
            obj = F(th0, None)
        grad = OrderedDict()
        for k in th0:
            cz = coinc if (k == "tau" and any_c) else None
            grad[k] = mp.diff(lambda t, k=k, cz=cz: F(_with(th0, k, t), cz), mp.log(th0[k]))
            if kind == "laplace":
                grad[k] += laplace_comp3_correction(th0, cov_fun, Xm, Um, yv, am, dl, fhat, k,
                                                    coinc)
        if kind == "laplace":
            return obj, grad, fhat
        return obj, grad
