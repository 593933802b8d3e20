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
        red2 = [np.sum(GK)]
        if self.kernel == "sqexp":
            red2.append(np.sum(GK * np.sum(self.diff ** 2, axis=2) / self.ls[0] ** 2))
        else:
            for c in range(self.L):
                red2.append(np.sum(GK * (self.diff[:, :, c] / self.ls[c]) ** 2))
        coinc = np.all(self.diff == 0.0, axis=2)
        red2 += [np.sum(G[coinc]), float(np.sum(coinc)),
                 float(np.sum(np.broadcast_to(np.diag(K22inv), coinc.shape)[coinc])), alpha @ alpha]
        return np.array(red2)      # [e_sig, e_l(L), c_sum, c_cnt, c_dg, alpha^T alpha]

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
        e_sig = red2[0]
        c_sum, c_cnt, c_dg, aTa = red2[1 + L], red2[2 + L], red2[3 + L], red2[4 + L]
        trW = 0.5 * (aTa - (n / z - sc["trBS"] / z ** 2))
        grad = np.zeros(L + 2)
        grad[0] = 2 * e_sig + sc["g22"][0] - n * sig2 / tau2
        grad[1:L + 1] = red2[1:1 + L] + sc["g22"][1:]
        grad[L + 1] = 2 * tau2 * (c_sum - (c_cnt - delta * c_dg) / tau2) + 2 * tau2 * trW - 2 * T
        return obj, grad


def eval_vi(kernel, theta, X, y, mu, U, delta=1e-6):
    rk = NumpyVIRank(X, y, mu)
    red1 = rk.phase1(kernel, theta, U, delta)
    red2 = rk.phase2(red1, X.shape[0])
    return rk.finish(red2)


# ------------------------------------------------------------------------------ FITC model
def eval_fitc(kernel, theta, X, y, mu, U, delta=1e-6):
    """Adjoint-form FITC objective + gradient (mirrors sgp_fitc_* in capi.hip)."""
    X, U = np.asarray(X, dtype=np.float64), np.asarray(U, dtype=np.float64)
    r = np.asarray(y, dtype=np.float64) - np.asarray(mu, dtype=np.float64)
    n, d = X.shape
    m = U.shape[0]
    L, sigma, tau, ls = _params(kernel, theta, d)
    tau2, sig2 = tau ** 2, sigma ** 2
    K, diff = _kmat(kernel, X, U, sigma, ls)
    Kuu, dU = _kmat(kernel, U, U, sigma, ls)
    K22 = Kuu.copy()
    K22[np.diag_indices(m)] = ((np.diag(Kuu) + tau2) + delta) - tau2
    K22inv = np.linalg.inv(K22)
    q = np.sum(K * (K @ K22inv), axis=1)
    Z = sig2 + tau2 + delta - q
    w = 1 / Z
    S = K.T @ (w[:, None] * K)
    t = K.T @ (w * r)
    rr = r @ (w * r)
    Bm = K22 + S
    Binv = np.linalg.inv(Bm)
    u = Binv @ t
    _, ld22 = np.linalg.slogdet(K22)
    _, ldB = np.linalg.slogdet(Bm)
    obj = -0.5 * rr + 0.5 * t @ u - 0.5 * (np.sum(np.log(Z)) - ld22 + ldB) - n / 2 * math.log(2 * math.pi)
    alpha = w * (r - K @ u)
    p = np.sum(K * (K @ Binv), axis=1)
    omega = alpha ** 2 - (w - w * w * p)
    Som = K.T @ (omega[:, None] * K)
    G = np.outer(alpha, u) - w[:, None] * (K @ Binv) - omega[:, None] * (K @ K22inv)
    G22 = -0.5 * np.outer(u, u) + 0.5 * (K22inv - Binv) + 0.5 * K22inv @ Som @ K22inv
    GK = G * K
    grad = np.zeros(L + 2)
    grad[0] = 2 * np.sum(GK) + np.sum(G22 * 2 * Kuu) + sig2 * np.sum(omega)
    if kernel == "sqexp":
        grad[1] = np.sum(GK * np.sum(diff ** 2, axis=2)) / ls[0] ** 2 + \
            np.sum(G22 * Kuu * np.sum(dU ** 2, axis=2)) / ls[0] ** 2
    else:
        for c in range(L):
            grad[1 + c] = np.sum(GK * (diff[:, :, c] / ls[c]) ** 2) + np.sum(G22 * Kuu * (dU[:, :, c] / ls[c]) ** 2)
    coinc = np.all(diff == 0.0, axis=2)
    grad[L + 1] = 2 * tau2 * np.sum(G[coinc]) + tau2 * np.sum(omega)
    return obj, grad


class NumpyFITCRank:
    """One rank of the FITC protocol (mirrors sgp_fitc_phase1/phase2/finish buffer layouts,
    without padding): red1 = [S_D, t, rr, sum log Z], red2 = [S_omega, sum omega, rec1, rec2]."""

    def __init__(self, X, y, mu):
        self.X = np.asarray(X, dtype=np.float64)
        self.r = np.asarray(y, dtype=np.float64) - np.asarray(mu, dtype=np.float64)

    def phase1(self, kernel, theta, U, delta):
        d = self.X.shape[1]
        self.kernel, self.U, self.delta = kernel, np.asarray(U), delta
        L, sigma, tau, ls = _params(kernel, theta, d)
        self.L, self.sigma, self.tau, self.ls = L, sigma, tau, ls
        m = self.U.shape[0]
        self.K, self.diff = _kmat(kernel, self.X, self.U, sigma, ls)
        Kuu, self.dU = _kmat(kernel, self.U, self.U, sigma, ls)
        self.Kuu = Kuu
        K22 = Kuu.copy()
        K22[np.diag_indices(m)] = ((np.diag(Kuu) + tau ** 2) + delta) - tau ** 2
        self.K22, self.K22inv = K22, np.linalg.inv(K22)
        q = np.sum(self.K * (self.K @ self.K22inv), axis=1)
        Z = sigma ** 2 + tau ** 2 + delta - q
        self.w = 1 / Z
        red1 = np.zeros(m * m + m + 2)
        red1[:m * m] = (self.K.T @ (self.w[:, None] * self.K)).reshape(-1)
        red1[m * m:m * m + m] = self.K.T @ (self.w * self.r)
        red1[m * m + m] = self.r @ (self.w * self.r)
        red1[m * m + m + 1] = np.sum(np.log(Z))
        return red1

    def phase2(self, red1, n_global):
        m = self.U.shape[0]
        S, t = red1[:m * m].reshape(m, m), red1[m * m:m * m + m]
        self.rr, self.sumlogz, self.n_global = red1[m * m + m], red1[m * m + m + 1], n_global
        Bm = self.K22 + S
        self.Binv = np.linalg.inv(Bm)
        self.ld22, self.ldB = np.linalg.slogdet(self.K22)[1], np.linalg.slogdet(Bm)[1]
        u = self.Binv @ t
        self.u, self.tu = u, t @ u
        K, w = self.K, self.w
        alpha = w * (self.r - K @ u)
        p = np.sum(K * (K @ self.Binv), axis=1)
        omega = alpha ** 2 - (w - w * w * p)
        G = np.outer(alpha, u) - w[:, None] * (K @ self.Binv) - omega[:, None] * (K @ self.K22inv)
        GK = G * K
        rec = [np.sum(GK)]
        if self.kernel == "sqexp":
            rec.append(np.sum(GK * np.sum(self.diff ** 2, axis=2)) / self.ls[0] ** 2)
        else:
            rec += [np.sum(GK * (self.diff[:, :, c] / self.ls[c]) ** 2) for c in range(self.L)]
        rec.append(np.sum(G[np.all(self.diff == 0.0, axis=2)]))
        red2 = np.concatenate([(K.T @ (omega[:, None] * K)).reshape(-1), [np.sum(omega)], rec])
        return red2

    def finish(self, red2):
        m, L = self.U.shape[0], self.L
        Som, sum_om, rec = red2[:m * m].reshape(m, m), red2[m * m], red2[m * m + 1:]
        n, tau2, sig2 = float(self.n_global), self.tau ** 2, self.sigma ** 2
        obj = -0.5 * self.rr + 0.5 * self.tu - 0.5 * (self.sumlogz - self.ld22 + self.ldB) - \
            n / 2 * math.log(2 * math.pi)
        G22 = -0.5 * np.outer(self.u, self.u) + 0.5 * (self.K22inv - self.Binv) + \
            0.5 * self.K22inv @ Som @ self.K22inv
        grad = np.zeros(L + 2)
        grad[0] = 2 * rec[0] + np.sum(G22 * 2 * self.Kuu) + sig2 * sum_om
        if self.kernel == "sqexp":
            grad[1] = rec[1] + np.sum(G22 * self.Kuu * np.sum(self.dU ** 2, axis=2)) / self.ls[0] ** 2
        else:
            for c in range(L):
                grad[1 + c] = rec[1 + c] + np.sum(G22 * self.Kuu * (self.dU[:, :, c] / self.ls[c]) ** 2)
        grad[L + 1] = 2 * tau2 * rec[1 + L] + tau2 * sum_om
        return obj, grad


# ------------------------------------------------------------------------------ Laplace model
def _lgamma1(y):
    from scipy.special import gammaln
    return gammaln(np.asarray(y, dtype=np.float64) + 1.0)


class NumpyLaplaceRank:
    """Poisson sparse-Laplace evaluation (newtrap_sparseGP + dlogq_dcov_par) in adjoint form,
    as the same reduction state machine as sgp_lap_begin / sgp_lap_step (capi.hip).

    Per-rank partials are summed between steps; everything m x m is replicated.
    Algebra: with Z = s^2+t^2+d-q, W = -a e^f, B = W/(ZW-1),
    S_w = K^T diag(w) K, Bm_Z = K22 + S_{1/Z}, C = (K22 + S_B)^-1:
      obj   = -r'(r/Z)/2 + t_Z' Bm_Z^-1 t_Z/2 + log p(y|f) - (logdet Bm_B - logdet K22)/2
              - sum log(1 - W Z)/2
      NR    f += [Z g - r + K (Bm_Z^-1 t_Z) + K C K^T (gpsi/omzw)] / omzw
      grad  <G, dK12> + <G22, dK22> + A1 sum(a) with
            G = c2 s^T - h GG^T - diag(B) K C - diag(2a) K K22^-1,
            G22 = (K22^-1 - C)/2 - s s^T/2 + sym(Cw GG^T)/2 + K22^-1 S_a K22^-1.
    """

    def __init__(self, X, y, mu):
        self.X = np.asarray(X, dtype=np.float64)
        self.y = np.asarray(y, dtype=np.float64)
        self.mu = np.asarray(mu, dtype=np.float64)
        self.f = None

    def set_f(self, f):
        self.f = np.array(f, dtype=np.float64)

    # -- local row-block partials
    def _obj_partials(self):
        f, Z = self.f, self.Z
        a = self.expo
        W = -a * np.exp(f)
        B = W / (Z * W - 1.0)
        r = f - self.mu
        K = self.K
        # a: the exposure, a scalar or this rank's rows (R/laplace_approx_obj_funs.R:125-129)
        logpy = np.sum(self.y * np.log(a) - _lgamma1(self.y) - a * np.exp(f) + self.y * f)
        return [(K.T @ (B[:, None] * K)).reshape(-1), K.T @ (r / Z),
                np.array([r @ (r / Z), logpy, np.sum(np.log(1.0 - W * Z))])]

    def begin(self, kernel, theta, U, delta, expo, tol=1e-5, maxit=1000):
        d = self.X.shape[1]
        self.kernel, self.U, self.delta, self.expo = kernel, np.asarray(U), delta, expo
        self.tol, self.maxit = tol, maxit
        L, sigma, tau, ls = _params(kernel, theta, d)
        self.L, self.sigma, self.tau, self.ls = L, sigma, tau, ls
        m = self.U.shape[0]
        self.K, self.diff = _kmat(kernel, self.X, self.U, sigma, ls)
        Kuu, self.dU = _kmat(kernel, self.U, self.U, sigma, ls)
        self.Kuu = Kuu
        K22 = Kuu.copy()
        K22[np.diag_indices(m)] = np.diag(Kuu) + tau ** 2 + delta          # quirk Q1
        self.K22, self.K22inv = K22, np.linalg.inv(K22)
        q = np.sum(self.K * (self.K @ self.K22inv), axis=1)
        self.Z = sigma ** 2 + tau ** 2 + delta - q
        self.SZ_local = (self.K.T @ ((1 / self.Z)[:, None] * self.K)).reshape(-1)
        self.objs = []
        self.state = "obj0"
        return np.concatenate([self.SZ_local] + self._obj_partials())

    def _consume_obj(self, red):
        m = self.U.shape[0]
        mm = m * m
        off = 0
        if self.state == "obj0":
            SZ = red[:mm].reshape(m, m)
            self.BmZinv = np.linalg.inv(self.K22 + SZ)
            self.ld22 = np.linalg.slogdet(self.K22)[1]
            off = mm
        SB = red[off:off + mm].reshape(m, m)
        tZ = red[off + mm:off + mm + m]
        rr, logpy, logz2 = red[off + mm + m:off + mm + m + 3]
        BmB = self.K22 + SB
        self.C = np.linalg.inv(BmB)
        self.x1 = self.BmZinv @ tZ
        obj = -0.5 * rr + 0.5 * tZ @ self.x1 + logpy - 0.5 * (-self.ld22 + np.linalg.slogdet(BmB)[1]) \
            - 0.5 * logz2
        self.objs.append(obj)

    def _nr_a(self):
        f, Z = self.f, self.Z
        W = -self.expo * np.exp(f)
        self.omzw = 1.0 - Z * W
        self.g = self.y - self.expo * np.exp(f)
        self.r = f - self.mu
        self.y1 = self.K @ self.x1
        c2 = (self.r - self.y1) / Z
        self.gpsi = self.g - c2
        return np.concatenate([self.K.T @ (self.gpsi / self.omzw),
                               [float(np.sum(np.abs(self.gpsi) > self.tol))]])

    def _grad_a(self):
        f, Z, K = self.f, self.Z, self.K
        W = -self.expo * np.exp(f)
        W3 = W
        B = W / (Z * W - 1.0)
        self.B = B
        self.g = self.y - self.expo * np.exp(f)
        r = f - self.mu
        self.c2 = (r - K @ self.x1) / Z
        p = np.sum(K * (K @ self.C), axis=1)
        self.dMt = B - B * B * p
        D = W - 1.0 / Z
        coef = 1.0 / (Z * D)
        comp4 = -1.0 / D + coef * coef * p
        self.sv = comp4 * W3 / W
        return np.concatenate([K.T @ self.c2, K.T @ self.g, K.T @ (B * self.sv)])

    def _grad_b(self, red):
        m = self.U.shape[0]
        K, B = self.K, self.B
        self.s = self.K22inv @ red[:m]
        self.GG = self.K22inv @ red[m:2 * m]
        self.Cw = self.C @ red[2 * m:3 * m]
        h = B * self.sv - B * (K @ self.Cw)
        a = -0.5 * self.dMt + 0.5 * self.c2 ** 2 - 0.5 * h * self.g
        G = np.outer(self.c2, self.s) - np.outer(h, self.GG) - B[:, None] * (K @ self.C) \
            - (2 * a)[:, None] * (K @ self.K22inv)
        GK = G * K
        rec = [np.sum(GK)]
        if self.kernel == "sqexp":
            rec.append(np.sum(GK * np.sum(self.diff ** 2, axis=2)) / self.ls[0] ** 2)
        else:
            rec += [np.sum(GK * (self.diff[:, :, c] / self.ls[c]) ** 2) for c in range(self.L)]
        rec.append(np.sum(G[np.all(self.diff == 0.0, axis=2)]))
        return np.concatenate([(K.T @ (a[:, None] * K)).reshape(-1), [np.sum(a)], rec])

    def _finish(self, red):
        m, L = self.U.shape[0], self.L
        mm = m * m
        Sa, suma, rec = red[:mm].reshape(m, m), red[mm], red[mm + 1:]
        K22inv = self.K22inv
        X = np.outer(self.Cw, self.GG)
        G22 = 0.5 * (K22inv - self.C) - 0.5 * np.outer(self.s, self.s) + 0.25 * (X + X.T) + \
            K22inv @ Sa @ K22inv
        tau2, sig2 = self.tau ** 2, self.sigma ** 2
        grad = np.zeros(L + 2)
        grad[0] = 2 * rec[0] + np.sum(G22 * 2 * self.Kuu) + 2 * sig2 * suma
        if self.kernel == "sqexp":
            grad[1] = rec[1] + np.sum(G22 * self.Kuu * np.sum(self.dU ** 2, axis=2)) / self.ls[0] ** 2
        else:
            for c in range(L):
                grad[1 + c] = rec[1 + c] + np.sum(G22 * self.Kuu * (self.dU[:, :, c] / self.ls[c]) ** 2)
        coinc22 = np.all(self.dU == 0.0, axis=2)
        grad[L + 1] = 2 * tau2 * rec[1 + L] + 2 * tau2 * np.sum(G22[coinc22]) + 2 * tau2 * suma
        return self.objs[-1], grad

    def step(self, red):
        """Consume the summed partials of the previous step; return (next partials or None,
        done, result)."""
        if self.state in ("obj0", "obj"):
            first = self.state == "obj0"
            self._consume_obj(red)
            it = len(self.objs)
            if first or (it < self.maxit and (abs(self.objs[-1] - self.objs[-2]) > self.tol
                                              or self.cnt > 0)):
                self.state = "nr_b"
                return self._nr_a(), False, None
            self.state = "grad_b"
            return self._grad_a(), False, None
        if self.state == "nr_b":
            m = self.U.shape[0]
            v2, self.cnt = red[:m], red[m]
            x2 = self.C @ v2
            self.f = self.f + (self.Z * self.g - self.r + self.y1 + self.K @ x2) / self.omzw
            self.state = "obj"
            return np.concatenate(self._obj_partials()), False, None
        if self.state == "grad_b":
            self.state = "finish"
            return self._grad_b(red), False, None
        if self.state == "finish":
            self.state = "done"
            return None, True, self._finish(red)
        raise RuntimeError(self.state)


def eval_laplace(kernel, theta, X, y, mu, U, f0, expo=1.0, delta=1e-6, tol=1e-5, maxit=1000):
    rk = NumpyLaplaceRank(X, y, mu)
    rk.set_f(f0)
    red = rk.begin(kernel, theta, U, delta, expo, tol, maxit)
    while True:
        red, done, res = rk.step(red)
        if done:
            return res[0], res[1], rk.f, len(rk.objs)


# ------------------------------------------------------------------------------ OAT candidates
def vi_candidates(kernel, theta, X, y, mu, U, cand, delta=1e-6):
    """ELBO at [U; cand_t] from the base system by bordering (mirrors sgp_vi_candidates)."""
    X, U = np.asarray(X, dtype=np.float64), np.asarray(U, dtype=np.float64)
    n, d = X.shape
    m = U.shape[0]
    L, sigma, tau, ls = _params(kernel, theta, d)
    z = tau ** 2 + delta
    K, _ = _kmat(kernel, X, U, sigma, ls)
    Kuu, _ = _kmat(kernel, U, U, sigma, ls)
    K22 = Kuu.copy()
    K22[np.diag_indices(m)] = ((np.diag(Kuu) + tau ** 2) + delta) - tau ** 2
    r = np.asarray(y) - np.asarray(mu)
    S, t, rr = K.T @ K, K.T @ r, r @ r
    Bm = K22 + S / z
    Binv, K22inv = np.linalg.inv(Bm), np.linalg.inv(K22)
    u = Binv @ t / z
    quad = -0.5 * rr / z + 0.5 * t @ u / z
    ld22, ldB = np.linalg.slogdet(K22)[1], np.linalg.slogdet(Bm)[1]
    trKS = np.sum(K22inv * S)
    kxx = ((sigma ** 2 + tau ** 2) + delta) - tau ** 2
    out = []
    for xs in np.asarray(cand, dtype=np.float64).reshape(-1, d):
        kc = _kmat(kernel, X, xs[None, :], sigma, ls)[0][:, 0]
        k22c = _kmat(kernel, U, xs[None, :], sigma, ls)[0][:, 0]
        p, c, w = K.T @ kc, kc @ kc, K22inv @ k22c
        sK = kxx - k22c @ w
        b = k22c + p / z
        sB = (kxx + c / z) - b @ Binv @ b
        dq = kc @ r - z * (b @ u)
        trinc = w @ S @ w - 2 * w @ p + c
        out.append(quad + 0.5 * dq * dq / (z * z * sB)
                   - 0.5 * (n * math.log(z) - (ld22 + math.log(sK)) + (ldB + math.log(sB)))
                   - n / 2 * math.log(2 * math.pi)
                   - (1 / (2 * tau ** 2)) * (n * (sigma ** 2 + delta) - (trKS + trinc / sK)))
    return np.array(out)
