"""numpy model of the libsgp VI reduction protocol -- TEST INFRASTRUCTURE ONLY.

Mirrors, buffer for buffer, what sgp_vi_phase1 / sgp_vi_phase2 / sgp_vi_finish compute on
the GPU (sparsergps_amd/csrc/capi.hip), so that
  * the adjoint algebra is checked against the literal oracle on CPU, and
  * the multi-rank driver (sparsergps_amd/dist.py) can be exercised with the gloo backend
    on hosts without a GPU (tests/test_dist.py).
It is never used by the product path.
"""
from __future__ import annotations

import math

import numpy as np


def _params(kernel, theta, d):
    L = d if kernel == "ard" else 1
    sigma, tau = float(theta[0]), float(theta[L + 1])
    ls = np.asarray(theta[1:L + 1], dtype=np.float64)
    return L, sigma, tau, ls


def _kmat(kernel, A, B, sigma, ls):
    diff = A[:, None, :] - B[None, :, :]
    if kernel == "sqexp":
        s = np.sum(diff ** 2, axis=2)
        return sigma ** 2 * np.exp(-1.0 / (2.0 * ls[0] ** 2) * s), diff
    s = np.sum((diff / ls) ** 2, axis=2)
    return sigma ** 2 * np.exp(-s / 2.0), diff


class NumpyVIRank:
    """One rank's rows (X_loc, r_loc); same phase API as the HIP context."""

    def __init__(self, X, y, mu):
        self.X = np.asarray(X, dtype=np.float64)
        self.r = np.asarray(y, dtype=np.float64) - np.asarray(mu, dtype=np.float64)

    # ---- phase 1: K12 and the first reduction [S, t, rr]
    def phase1(self, kernel, theta, U, delta):
        d = self.X.shape[1]
        self.kernel, self.theta, self.U, self.delta = kernel, np.asarray(theta), np.asarray(U), delta
        L, sigma, tau, ls = _params(kernel, theta, d)
        self.L, self.sigma, self.tau, self.ls = L, sigma, tau, ls
        self.K, self.diff = _kmat(kernel, self.X, self.U, sigma, ls)
        m = self.U.shape[0]
        red1 = np.zeros(m * m + m + 1)
        red1[:m * m] = (self.K.T @ self.K).reshape(-1)
        red1[m * m:m * m + m] = self.K.T @ self.r
        red1[m * m + m] = self.r @ self.r
        return red1

    # ---- phase 2: replicated m x m algebra + local contraction partials
    def phase2(self, red1, n_global):
        m = self.U.shape[0]
        S = red1[:m * m].reshape(m, m)
        t = red1[m * m:m * m + m]
        rr = red1[m * m + m]
        tau2, sig2, delta = self.tau ** 2, self.sigma ** 2, self.delta
        z = tau2 + delta
        Kuu, dU = _kmat(self.kernel, self.U, self.U, self.sigma, self.ls)
        K22 = Kuu.copy()
        K22[np.diag_indices(m)] = ((np.diag(Kuu) + tau2) + delta) - tau2
        Bm = K22 + S / z
        L22 = np.linalg.cholesky(K22)
        LB = np.linalg.cholesky(Bm)
        K22inv = np.linalg.inv(K22)
        Binv = np.linalg.inv(Bm)
        u = Binv @ t / z
        P = K22inv / tau2 - Binv / z
        M3 = K22inv @ S @ K22inv
        G22 = -0.5 * np.outer(u, u) + 0.5 * (K22inv - Binv) - M3 / (2 * tau2)
        # replicated scalars (sc buffer)
        self.sc = dict(ld22=np.sum(np.log(np.diag(L22))), ldB=np.sum(np.log(np.diag(LB))),
                       tu=t @ u, trKS=np.sum(K22inv * S), trBS=np.sum(Binv * S), rr=rr)
        g22 = [np.sum(G22 * 2 * Kuu)]
        if self.kernel == "sqexp":
            g22.append(np.sum(G22 * Kuu * np.sum(dU ** 2, axis=2) / self.ls[0] ** 2))
        else:
            for c in range(self.L):
                g22.append(np.sum(G22 * Kuu * (dU[:, :, c] / self.ls[c]) ** 2))
        self.sc["g22"] = np.array(g22)
        self.n_global = n_global
        # local partials (red2)
        alpha = (self.r - self.K @ u) / z
        G = np.outer(alpha, u) + self.K @ P
        GK = G * self.K
        red2 = [alpha @ alpha, np.sum(GK)]
        if self.kernel == "sqexp":
            red2.append(np.sum(GK * np.sum(self.diff ** 2, axis=2) / self.ls[0] ** 2))
        else:
            for c in range(self.L):
                red2.append(np.sum(GK * (self.diff[:, :, c] / self.ls[c]) ** 2))
        coinc = np.all(self.diff == 0.0, axis=2)
        red2 += [np.sum(G[coinc]), float(np.sum(coinc)),
                 float(np.sum(np.broadcast_to(np.diag(K22inv), coinc.shape)[coinc]))]
        return np.array(red2)

    # ---- finish: objective + gradient from the reduced red2 and the replicated scalars
    def finish(self, red2):
        sc, L = self.sc, self.L
        n = float(self.n_global)
        tau2, sig2, delta = self.tau ** 2, self.sigma ** 2, self.delta
        z = tau2 + delta
        ld22, ldB = 2 * sc["ld22"], 2 * sc["ldB"]
        quad = -0.5 * sc["rr"] / z + 0.5 * sc["tu"] / z
        det_part = -0.5 * (n * math.log(z) - ld22 + ldB)
        T = -(1.0 / (2 * tau2)) * (n * (sig2 + delta) - sc["trKS"])
        obj = quad + det_part - n / 2 * math.log(2 * math.pi) + T
        aTa, e_sig = red2[0], red2[1]
        c_sum, c_cnt, c_dg = red2[2 + L], red2[3 + L], red2[4 + L]
        trW = 0.5 * (aTa - (n / z - sc["trBS"] / z ** 2))
        grad = np.zeros(L + 2)
        grad[0] = 2 * e_sig + sc["g22"][0] - n * sig2 / tau2
        grad[1:L + 1] = red2[2:2 + L] + sc["g22"][1:]
        grad[L + 1] = 2 * tau2 * (c_sum - (c_cnt - delta * c_dg) / tau2) + 2 * tau2 * trW - 2 * T
        return obj, grad


def eval_vi(kernel, theta, X, y, mu, U, delta=1e-6):
    rk = NumpyVIRank(X, y, mu)
    red1 = rk.phase1(kernel, theta, U, delta)
    red2 = rk.phase2(red1, X.shape[0])
    return rk.finish(red2)
