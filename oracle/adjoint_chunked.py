"""Row-chunked CPU model of the VI adjoint evaluation -- TEST INFRASTRUCTURE ONLY.

The same algebra as ``adjoint_ref.NumpyVIRank`` (which mirrors sgp_vi_phase1/2/finish,
DESIGN.md sec. 3.1), restated so that its memory is O(chunk * m) instead of O(n * m * d):

  pass 1 over row chunks   K_c = k(X_c, U);  S += K_c^T K_c,  t += K_c^T r_c,  r^T r
  replicated m x m algebra  K22^-1, Bm^-1, u, P, M3, G22, log-dets (adjoint_ref)
  pass 2 over row chunks   alpha_c = (r_c - K_c u)/z,  G_c = alpha_c u^T + K_c P,
                           W = G_c o K_c  contracted with dK/dlog(theta):
                             sigma   sum W
                             l_q     sum_ij W_ij (x_iq - u_jq)^2 / l_q^2
                                     = sum_i x~_iq^2 (W 1)_i - 2 x~_q^T W u~_q + (1^T W)_j u~_jq^2
                           plus the tau coincidence sums over rows equal to a knot (quirk Q5)

Uses:
  * tests: the GPU path at the C4 shard shape (n = 125 000, m = 1024, d = 8) and at full C2 /
    C3-row sizes, where the literal oracle (sgp_oracle.py) cannot run in seconds;
  * bench.py's cpu_baseline: the optimised CPU bar (the GPU's algorithm on the host's BLAS),
    timed directly at n = 1e6 -- the cost is linear in n, nothing is extrapolated.
The exponent is formed as |x~|^2 + |u~|^2 - 2 x~ u~^T (one GEMM per chunk) on coordinates
centred at the knots' mean; the kernel values then carry ~1e-14 relative error, far inside
the 1e-6 parity bar.  Never used by the product path.
"""
from __future__ import annotations

import math

import numpy as np

from .adjoint_ref import _kmat, _params


def _scaled(kernel, A, center, ls):
    """Coordinates centred at `center` and scaled so that the kernel is exp(-|a - b|^2 / 2)."""
    if kernel == "sqexp":
        return (A - center) / ls[0]
    return (A - center) / ls


def _kblock(Xs, x2, Us, u2, sig2, out=None):
    """sig2 * exp(-(|x|^2 + |u|^2 - 2 x u^T) / 2) for one row chunk (scaled coordinates)."""
    E = np.matmul(Xs, Us.T, out=out)
    E *= 2.0
    E -= x2[:, None]
    E -= u2[None, :]
    np.minimum(E, 0.0, out=E)          # the exact exponent is <= 0
    E *= 0.5
    np.exp(E, out=E)
    E *= sig2
    return E


def _row_keys(A):
    """Byte keys of the rows (-0.0 canonicalised to +0.0) for exact-equality matching."""
    A = np.ascontiguousarray(np.asarray(A, dtype=np.float64) + 0.0)
    return A.view(np.dtype((np.void, A.dtype.itemsize * A.shape[1]))).ravel()


def eval_vi(kernel, theta, X, y, mu, U, delta=1e-6, chunk=8192, n_global=None):
    """(ELBO, d ELBO / d log theta) in [sigma, l.., tau] order; X, y, mu may be one rank's rows
    with n_global the total row count (then the value is that rank's partial -- only the
    single-rank call, n_global = None, returns the full objective)."""
    X = np.asarray(X, dtype=np.float64)
    U = np.asarray(U, dtype=np.float64)
    n, d = X.shape
    m = U.shape[0]
    r = np.asarray(y, dtype=np.float64) - np.asarray(mu, dtype=np.float64)
    L, sigma, tau, ls = _params(kernel, theta, d)
    sig2, tau2 = sigma * sigma, tau * tau
    z = tau2 + delta
    center = U.mean(axis=0)
    Us = _scaled(kernel, U, center, ls)
    u2 = np.einsum("ij,ij->i", Us, Us)
    buf = np.empty((min(chunk, n), m))

    # ---- pass 1: S, t, r^T r
    S = np.zeros((m, m))
    t = np.zeros(m)
    for s0 in range(0, n, chunk):
        s1 = min(n, s0 + chunk)
        Xs = _scaled(kernel, X[s0:s1], center, ls)
        K = _kblock(Xs, np.einsum("ij,ij->i", Xs, Xs), Us, u2, sig2, out=buf[:s1 - s0])
        S += K.T @ K
        t += K.T @ r[s0:s1]
    rr = float(r @ r)

    # ---- replicated m x m algebra (as adjoint_ref.NumpyVIRank.phase2)
    Kuu, dU = _kmat(kernel, U, U, sigma, ls)
    K22 = Kuu.copy()
    K22[np.diag_indices(m)] = ((np.diag(Kuu) + tau2) + delta) - tau2
    Bm = K22 + S / z
    ld22 = float(np.sum(np.log(np.diag(np.linalg.cholesky(K22)))))
    ldB = float(np.sum(np.log(np.diag(np.linalg.cholesky(Bm)))))
    K22inv = np.linalg.inv(K22)
    Binv = np.linalg.inv(Bm)
    u = Binv @ t / z
    P = K22inv / tau2 - Binv / z
    M3 = K22inv @ S @ K22inv
    G22 = -0.5 * np.outer(u, u) + 0.5 * (K22inv - Binv) - M3 / (2 * tau2)
    g22 = [float(np.sum(G22 * 2 * Kuu))]
    if kernel == "sqexp":
        g22.append(float(np.sum(G22 * Kuu * np.sum(dU ** 2, axis=2) / ls[0] ** 2)))
    else:
        for c in range(L):
            g22.append(float(np.sum(G22 * Kuu * (dU[:, :, c] / ls[c]) ** 2)))
    tu, trKS, trBS = float(t @ u), float(np.sum(K22inv * S)), float(np.sum(Binv * S))

    # ---- pass 2: contraction of G = alpha u^T + K P with dK/dlog theta
    e_sig = 0.0
    e_l = np.zeros(L)
    aTa = 0.0
    ukeys = _row_keys(U)
    korder = np.argsort(ukeys)
    usorted = ukeys[korder]
    c_sum = c_cnt = c_dg = 0.0
    dg = np.diag(K22inv)
    for s0 in range(0, n, chunk):
        s1 = min(n, s0 + chunk)
        Xs = _scaled(kernel, X[s0:s1], center, ls)
        x2 = np.einsum("ij,ij->i", Xs, Xs)
        K = _kblock(Xs, x2, Us, u2, sig2, out=buf[:s1 - s0])
        alpha = (r[s0:s1] - K @ u) / z
        aTa += float(alpha @ alpha)
        G = K @ P
        G += np.outer(alpha, u)
        # exact coincidences row == knot (dK12/dlog tau = 2 tau^2 there)
        keys = _row_keys(X[s0:s1])
        pos = np.searchsorted(usorted, keys)
        pos[pos >= m] = m - 1
        hit = np.nonzero(usorted[pos] == keys)[0]
        for i in hit:
            for j in np.nonzero(ukeys == keys[i])[0]:
                c_sum += G[i, j]
                c_cnt += 1.0
                c_dg += dg[j]
        G *= K                                         # W = G o K
        rs = G.sum(axis=1)
        cs = G.sum(axis=0)
        e_sig += float(rs.sum())
        XW = Xs.T @ G                                  # d x m
        if kernel == "sqexp":
            e_l[0] += float(x2 @ rs - 2.0 * np.sum(XW * Us.T) + cs @ u2)
        else:
            e_l += (Xs * Xs).T @ rs - 2.0 * np.sum(XW * Us.T, axis=1) + (Us * Us).T @ cs

    nn = float(n if n_global is None else n_global)
    quad = -0.5 * rr / z + 0.5 * tu / z
    det_part = -0.5 * (nn * math.log(z) - 2 * ld22 + 2 * ldB)
    T = -(1.0 / (2 * tau2)) * (nn * (sig2 + delta) - trKS)
    obj = quad + det_part - nn / 2 * math.log(2 * math.pi) + T
    trW = 0.5 * (aTa - (nn / z - trBS / z ** 2))
    grad = np.zeros(L + 2)
    grad[0] = 2 * e_sig + g22[0] - nn * sig2 / tau2
    grad[1:L + 1] = e_l + np.asarray(g22[1:])
    grad[L + 1] = 2 * tau2 * (c_sum - (c_cnt - delta * c_dg) / tau2) + 2 * tau2 * trW - 2 * T
    return obj, grad
