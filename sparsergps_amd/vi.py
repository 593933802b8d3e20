"""Fused sparse-GP objective + gradient on the MI355X (Layer 2 of include/sgp.h).

Host-side mirror of the reference's hot path (luisdamiano/sparseRGPs):
  elbo_fun        R/vi_functions.R:64-121
  delbo_dcov_par  R/vi_functions.R:126-602   (knots fixed: dcov_fun_dknot = NA)
  trace_term_fun  R/vi_functions.R:14-27     (returned as part of the ELBO)
with the matrices built as norm_grad_ascent_vi builds them (vi_functions.R:1089-1128):
K12 = k(xy, xu), K22 = k(xu, xu) + delta I, Z = tau^2 + delta.

A SparseGPContext keeps X, y - mu and all work buffers resident in HBM; one call of
``eval_vi`` is one optimizer-iteration body (objective and full gradient).  Everything runs in
libsgp.so's HIP kernels; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from collections import OrderedDict

import numpy as np

from . import _lib
from .covariance import theta_vector


def _device():
    return int(os.environ.get("SGP_DEVICE", "0"))


def param_names(cov_fun, d, lnames=None):
    """Parameter names in libsgp's theta layout [sigma, l.., tau]."""
    if cov_fun == "ard":
        ls = list(lnames) if lnames is not None else [f"l{c + 1}" for c in range(d)]
        return ["sigma"] + ls[:d] + ["tau"]
    return ["sigma", "l", "tau"]


class SparseGPContext:
    """Device-resident rows (X, y - mu) plus work space for up to ``m_max`` knots."""

    def __init__(self, xy, y, mu, m_max, device=None, stream=None, devices=None):
        """devices: a list of device indices, one per row shard (repeats allowed) -- a
        row-sharded multi-device context (sgp_ctx_create_multi: the reductions, RCCL over the
        distinct devices included, run inside libsgp); None: one device."""
        if mu is None:
            raise ValueError("SparseGPContext: mu is required (mean(y) for VI / FITC, "
                             "log mean(y) for Poisson Laplace)")
        self._lib = _lib.lib()
        _lib.require_gpu()
        X = np.asfortranarray(np.asarray(xy, dtype=np.float64).reshape(len(y), -1))
        y = np.ascontiguousarray(np.asarray(y, dtype=np.float64).reshape(-1))
        mu = np.ascontiguousarray(np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape))
        self.n, self.d = X.shape
        self.m_max = int(m_max)
        self.device = _device() if device is None else int(device)
        h = C.c_void_p()
        self.devices = None
        if devices is not None:
            self.devices = [int(v) for v in devices]
            dv = (C.c_int * len(self.devices))(*self.devices)
            _lib.check(self._lib.sgp_ctx_create_multi(C.byref(h), dv, len(self.devices),
                                                      _lib.dptr(X), self.n, self.n, self.d,
                                                      _lib.dptr(y), _lib.dptr(mu), self.m_max))
        else:
            _lib.check(self._lib.sgp_ctx_create(C.byref(h), self.device, _lib.dptr(X), self.n,
                                                self.n, self.d, _lib.dptr(y), _lib.dptr(mu),
                                                self.m_max))
        self._h = h
        if stream is not None:
            self.set_stream(stream)

    # ------------------------------------------------------------------ plumbing
    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("SparseGPContext is closed")
        return self._h

    def shards(self):
        """(row shards, distinct devices) of this context"""
        ns, nd = C.c_int(0), C.c_int(0)
        _lib.check(self._lib.sgp_ctx_shards(self.handle, C.byref(ns), C.byref(nd)))
        return ns.value, nd.value

    def set_stream(self, stream):
        """stream: an int hipStream_t handle (e.g. torch.cuda.current_stream().cuda_stream)."""
        _lib.check(self._lib.sgp_ctx_set_stream(self.handle, C.c_void_p(int(stream) if stream else 0)))

    def set_data(self, y, mu):
        if mu is None:
            raise ValueError("set_data: mu is required")
        y = np.ascontiguousarray(np.asarray(y, dtype=np.float64).reshape(-1))
        mu = np.ascontiguousarray(np.broadcast_to(np.asarray(mu, dtype=np.float64), y.shape))
        _lib.check(self._lib.sgp_ctx_set_data(self.handle, _lib.dptr(y), _lib.dptr(mu)))

    def enable_timing(self, on=True):
        _lib.check(self._lib.sgp_ctx_enable_timing(self.handle, 1 if on else 0))

    def timing_filter(self, name=None):
        """Record only the phase `name` (None: all phases) while timing is enabled."""
        _lib.check(self._lib.sgp_ctx_timing_filter(self.handle,
                                                   None if name is None else name.encode()))

    def timing_evals(self):
        """Evaluations recorded since enable_timing(True)."""
        return int(self._lib.sgp_ctx_timing_evals(self.handle))

    def timings(self):
        """[(phase name, total ms)] over the evaluations recorded since enable_timing(True)
        (HIP events on the launch stream, read back only here)."""
        names = C.create_string_buffer(65536)
        ms = (C.c_double * 2048)()
        cnt = C.c_int(0)
        _lib.check(self._lib.sgp_ctx_timings(self.handle, names, 65536, ms, 2048, C.byref(cnt)))
        nm = names.value.decode().split("\n")
        return [(nm[i], ms[i]) for i in range(cnt.value)]

    def close(self):
        if getattr(self, "_h", None) is not None:
            self._lib.sgp_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------------ evaluation
    def _knots(self, xu):
        U = np.asfortranarray(np.asarray(xu, dtype=np.float64).reshape(-1, self.d))
        self._last_m = U.shape[0]
        return U, U.shape[0]

    @staticmethod
    def _flags(r_det, obj_only):
        return (_lib.SGP_FLAG_R_DET if r_det else 0) | (_lib.SGP_FLAG_OBJ_ONLY if obj_only else 0)

    # sgp_eval_vi / sgp_eval_fitc called with raw addresses: an optimizer calls them once per
    # step, and at C2 (~0.6 ms per evaluation) ctypes' pointer objects were ~4 us of it
    _EVAL_PROTO = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64,
                              C.c_int64, C.c_double, C.c_uint, C.c_void_p, C.c_void_p)

    def _fast_buf(self, key, shape, order="C"):
        # a host buffer kept for the context's lifetime with its address: `arr.ctypes.data` costs
        # ~1.5 us per array and call, and the one-call evaluation passes three of them
        bufs = self.__dict__.setdefault("_fast_bufs", {})
        b = bufs.get(key)
        if b is None or b[0].shape != shape:
            arr = np.zeros(shape, dtype=np.float64, order=order)
            b = bufs[key] = (arr, arr.ctypes.data)
        return b

    def _eval_fast(self, name, theta, cov_fun, xu, delta, r_det, obj_only):
        fns = self.__dict__.setdefault("_fast_fns", {})
        fn = fns.get(name)
        if fn is None:
            fn = fns[name] = self._EVAL_PROTO(C.cast(getattr(self._lib, name), C.c_void_p).value)
        theta = np.asarray(theta, dtype=np.float64).reshape(-1)
        th, th_p = self._fast_buf("theta", theta.shape)
        th[...] = theta
        xu = np.asarray(xu, dtype=np.float64)
        m = xu.size // self.d
        U, U_p = self._fast_buf("U", (m, self.d), "F")
        U[...] = xu.reshape(m, self.d)   # (copied every call: the caller may move its knots)
        self._last_m = m
        out, a = self._fast_buf("out", (theta.size + 1,))   # [objective, gradient]
        st = fn(self.handle.value, _lib.KERNELS[cov_fun], th_p, U_p, m, m, float(delta),
                self._flags(r_det, obj_only), a, None if obj_only else a + 8)
        _lib.check(st)
        return float(out[0]), (None if obj_only else out[1:].copy())

    def eval_vi(self, theta, cov_fun, xu, delta=1e-6, r_det=False, obj_only=False):
        """ELBO and d ELBO / d log(theta) with theta in [sigma, l.., tau] layout
        (obj_only: elbo_fun alone, grad None)."""
        return self._eval_fast("sgp_eval_vi", theta, cov_fun, xu, delta, r_det, obj_only)

    def eval_fitc(self, theta, cov_fun, xu, delta=1e-6, r_det=False, obj_only=False):
        """FITC log marginal likelihood and d/d log(theta) (obj_fun_norm + dlogp_dcov_par;
        obj_only: obj_fun_norm alone, grad None)."""
        return self._eval_fast("sgp_eval_fitc", theta, cov_fun, xu, delta, r_det, obj_only)

    def eval_full(self, theta, cov_fun, delta=1e-6, obj_only=False):
        """Full Gaussian GP over this context's rows (m_max >= n): log dmvnorm(y; mu, Sigma11)
        and dlogp_dcov_par_full (grad None with obj_only)."""
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        obj = C.c_double(0.0)
        grad = None if obj_only else np.zeros(theta.size, dtype=np.float64)
        _lib.check(self._lib.sgp_eval_full(self.handle, _lib.KERNELS[cov_fun], _lib.dptr(theta),
                                           float(delta), self._flags(False, obj_only),
                                           C.byref(obj), None if grad is None else _lib.dptr(grad)))
        return obj.value, grad

    def enable_knot_grad(self, on=True):
        """Also contract the adjoint against dK/du (knot gradients)."""
        _lib.check(self._lib.sgp_ctx_enable_knot_grad(self.handle, 1 if on else 0))

    def knot_red_extra(self, m):
        return int(self._lib.sgp_knot_red_extra(self.d, int(m)))

    def row_bounds(self):
        lo = np.zeros(self.d)
        hi = np.zeros(self.d)
        _lib.check(self._lib.sgp_ctx_row_bounds(self.handle, _lib.dptr(lo), _lib.dptr(hi)))
        return lo, hi

    def knot_gradient(self, bounds=None):
        """Row-major (m*d) knot gradient of the last evaluation with the reference's chain
        factor; bounds: d x 2 [lower, upper] (None: knot_bounds of this context's rows)."""
        m = self._last_m
        out = np.zeros(m * self.d, dtype=np.float64)
        b = None if bounds is None else np.asfortranarray(np.asarray(bounds, dtype=np.float64))
        _lib.check(self._lib.sgp_knot_gradient(self.handle, None if b is None else _lib.dptr(b),
                                               _lib.dptr(out)))
        return out

    def posterior_u(self, muu):
        """Knot posterior (u_mean, u_var) of the last completed evaluation, as the drivers
        return it at the end of a fit (vi_functions.R:1161-1180,
        laplace_gradient_ascent.R:1635-1655, newtrap_sparseGP.R:137-176)."""
        mu_u = np.ascontiguousarray(np.asarray(muu, dtype=np.float64).reshape(-1))
        m = mu_u.size
        um = np.zeros(m, dtype=np.float64)
        uv = np.zeros((m, m), dtype=np.float64, order="F")
        _lib.check(self._lib.sgp_posterior_u(self.handle, _lib.dptr(mu_u), _lib.dptr(um),
                                             _lib.dptr(uv)))
        return um, uv

    # ------------------------------------------------------------------ Poisson Laplace
    def lap_set_f(self, f=None, fill=0.0):
        """Set the resident latent vector f (NR warm start); f=None fills with `fill`."""
        if f is None:
            _lib.check(self._lib.sgp_lap_set_f(self.handle, None, float(fill)))
        else:
            f = np.ascontiguousarray(np.broadcast_to(np.asarray(f, dtype=np.float64), (self.n,)))
            _lib.check(self._lib.sgp_lap_set_f(self.handle, _lib.dptr(f), 0.0))

    def lap_set_expo(self, a=None, fill=1.0):
        """Resident per-row Poisson exposure (the reference's `m` as a vector of cell areas,
        R/derivative_functions_of_data_likelihoods.R:38); a=None fills every row with `fill`."""
        if a is None:
            _lib.check(self._lib.sgp_lap_set_expo(self.handle, None, float(fill)))
        else:
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
            if a.size != self.n:
                raise ValueError(f"exposure has {a.size} values for {self.n} rows")
            _lib.check(self._lib.sgp_lap_set_expo(self.handle, _lib.dptr(a), 0.0))

    def _expo(self, expo):
        """The expo argument of the Laplace entry points: a scalar as is; an n-vector is made
        resident (sgp_lap_set_expo) and passed as SGP_EXPO_ROWS.  A length-1 vector is the
        scalar (R recycling)."""
        a = np.asarray(expo, dtype=np.float64)
        if a.size == 1:
            return float(a.reshape(-1)[0])
        self.lap_set_expo(a)
        return _lib.SGP_EXPO_ROWS

    def lap_get_f(self):
        f = np.zeros(self.n, dtype=np.float64)
        _lib.check(self._lib.sgp_lap_get_f(self.handle, _lib.dptr(f)))
        return f

    def lap_get_grad_psi(self):
        """grad psi of the last NR step (newtrap_sparseGP's `gradient`)."""
        g = np.zeros(self.n, dtype=np.float64)
        _lib.check(self._lib.sgp_lap_get_grad_psi(self.handle, _lib.dptr(g)))
        return g

    def lap_objective_values(self):
        cnt = C.c_int(0)
        _lib.check(self._lib.sgp_lap_objective_values(self.handle, None, 0, C.byref(cnt)))
        out = np.zeros(max(cnt.value, 1), dtype=np.float64)
        _lib.check(self._lib.sgp_lap_objective_values(self.handle, _lib.dptr(out), cnt.value,
                                                      C.byref(cnt)))
        return out[:cnt.value]

    def eval_laplace(self, theta, cov_fun, xu, delta=1e-6, expo=1.0, tol=1e-5, maxit=1000):
        """newtrap_sparseGP from the resident f, then dlogq_dcov_par at the mode:
        (log q(y | theta, xu, f_hat), d/d log(theta), NR iteration count)."""
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        obj = C.c_double(0.0)
        it = C.c_int(0)
        grad = np.zeros(theta.size, dtype=np.float64)
        _lib.check(self._lib.sgp_eval_laplace(self.handle, _lib.KERNELS[cov_fun], _lib.dptr(theta),
                                              _lib.dptr(U), m, m, float(delta), self._expo(expo),
                                              float(tol), int(maxit), C.byref(obj),
                                              _lib.dptr(grad), C.byref(it)))
        return obj.value, grad, it.value

    def vi_candidates(self, theta, cov_fun, xu, cand, delta=1e-6, r_det=False):
        """ELBO at knots [xu; cand[t]] for every candidate row t (OAT proposal scoring)."""
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        Cd = np.asfortranarray(np.asarray(cand, dtype=np.float64).reshape(-1, self.d))
        T = Cd.shape[0]
        out = np.zeros(T, dtype=np.float64)
        _lib.check(self._lib.sgp_vi_candidates(self.handle, _lib.KERNELS[cov_fun], _lib.dptr(theta),
                                               _lib.dptr(U), m, m, float(delta),
                                               _lib.SGP_FLAG_R_DET if r_det else 0,
                                               _lib.dptr(Cd), T, T, _lib.dptr(out)))
        return out

    def fitc_candidates(self, theta, cov_fun, xu, cand, delta=1e-6, r_det=False):
        """obj_fun_norm at knots [xu; cand[t]] for every candidate row t (FITC OAT scoring)."""
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        Cd = np.asfortranarray(np.asarray(cand, dtype=np.float64).reshape(-1, self.d))
        T = Cd.shape[0]
        out = np.zeros(T, dtype=np.float64)
        _lib.check(self._lib.sgp_fitc_candidates(self.handle, _lib.KERNELS[cov_fun],
                                                 _lib.dptr(theta), _lib.dptr(U), m, m,
                                                 float(delta), self._flags(r_det, False),
                                                 _lib.dptr(Cd), T, T, _lib.dptr(out)))
        return out

    def lap_candidates(self, theta, cov_fun, xu, cand, delta=1e-6, expo=1.0, tol=1e-5,
                       maxit=1000):
        """Last NR objective of newtrap_sparseGP at knots [xu; cand[t]] from the resident f, for
        every candidate row t (Laplace OAT scoring); the resident f is left unchanged."""
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        Cd = np.asfortranarray(np.asarray(cand, dtype=np.float64).reshape(-1, self.d))
        T = Cd.shape[0]
        out = np.zeros(T, dtype=np.float64)
        _lib.check(self._lib.sgp_lap_candidates(self.handle, _lib.KERNELS[cov_fun],
                                                _lib.dptr(theta), _lib.dptr(U), m, m,
                                                float(delta), self._expo(expo), float(tol),
                                                int(maxit), _lib.dptr(Cd), T, T, _lib.dptr(out)))
        return out

    def lap_nr(self, theta, cov_fun, xu, delta=1e-6, expo=1.0, tol=1e-5, maxit=1000):
        """newtrap_sparseGP alone from the resident f: (last objective value, NR iterations);
        f is left at the mode."""
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        obj = C.c_double(0.0)
        it = C.c_int(0)
        _lib.check(self._lib.sgp_lap_nr(self.handle, _lib.KERNELS[cov_fun], _lib.dptr(theta),
                                        _lib.dptr(U), m, m, float(delta), self._expo(expo), float(tol),
                                        int(maxit), C.byref(obj), C.byref(it)))
        return obj.value, it.value

    def lap_red_count(self, cov_fun, m):
        return int(self._lib.sgp_lap_red_count(_lib.KERNELS[cov_fun], self.d, int(m)))

    def lap_begin(self, theta, cov_fun, xu, delta, expo, tol, maxit, red_ptr, obj_only=False):
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        cnt = C.c_int64(0)
        _lib.check(self._lib.sgp_lap_begin(self.handle, _lib.KERNELS[cov_fun], _lib.dptr(theta),
                                           _lib.dptr(U), m, m, float(delta), self._expo(expo),
                                           float(tol), int(maxit),
                                           self._flags(False, obj_only), C.c_void_p(red_ptr),
                                           C.byref(cnt)))
        return cnt.value

    def lap_step(self, red_in_ptr, red_out_ptr, nparams):
        """-> (count, done, obj, grad, nr_iters)"""
        cnt = C.c_int64(0)
        done = C.c_int(0)
        obj = C.c_double(0.0)
        it = C.c_int(0)
        grad = np.zeros(nparams, dtype=np.float64)
        _lib.check(self._lib.sgp_lap_step(self.handle, C.c_void_p(red_in_ptr),
                                          C.c_void_p(red_out_ptr), C.byref(cnt), C.byref(done),
                                          C.byref(obj), _lib.dptr(grad), C.byref(it)))
        return cnt.value, bool(done.value), obj.value, grad, it.value

    # multi-GPU phases (device buffers passed as integer pointers, e.g. tensor.data_ptr())
    def vi_red1_count(self, m):
        """doubles of VI's first reduction (packed layout when set_packed_reduction is on)"""
        if getattr(self, "_packed", False):
            return int(self._lib.sgp_vi_red1_packed_count(int(m)))
        return int(self._lib.sgp_vi_red1_count(int(m)))

    def set_packed_reduction(self, on=True):
        """VI phase 1 writes S as its packed lower 64-blocks (sgp_ctx_set_packed_reduction):
        the multi-GPU all-reduce #1 moves 53 % of the bytes at m = 1024."""
        _lib.check(self._lib.sgp_ctx_set_packed_reduction(self.handle, 1 if on else 0))
        self._packed = bool(on)

    def vi_red2_count(self, cov_fun):
        return int(self._lib.sgp_vi_red2_count(_lib.KERNELS[cov_fun], self.d))

    def vi_phase1(self, theta, cov_fun, xu, delta, red1_ptr):
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        _lib.check(self._lib.sgp_vi_phase1(self.handle, _lib.KERNELS[cov_fun], _lib.dptr(theta),
                                           _lib.dptr(U), m, m, float(delta), C.c_void_p(red1_ptr)))

    def vi_phase2(self, red1_ptr, n_global, red2_ptr, r_det=False):
        _lib.check(self._lib.sgp_vi_phase2(self.handle, C.c_void_p(red1_ptr), int(n_global),
                                           _lib.SGP_FLAG_R_DET if r_det else 0,
                                           C.c_void_p(red2_ptr)))

    def fitc_red1_count(self, m):
        return int(self._lib.sgp_fitc_red1_count(int(m)))

    def fitc_red2_count(self, cov_fun, m):
        return int(self._lib.sgp_fitc_red2_count(_lib.KERNELS[cov_fun], self.d, int(m)))

    def fitc_phase1(self, theta, cov_fun, xu, delta, red1_ptr):
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        U, m = self._knots(xu)
        _lib.check(self._lib.sgp_fitc_phase1(self.handle, _lib.KERNELS[cov_fun], _lib.dptr(theta),
                                             _lib.dptr(U), m, m, float(delta), C.c_void_p(red1_ptr)))

    def fitc_phase2(self, red1_ptr, n_global, red2_ptr, r_det=False):
        _lib.check(self._lib.sgp_fitc_phase2(self.handle, C.c_void_p(red1_ptr), int(n_global),
                                             _lib.SGP_FLAG_R_DET if r_det else 0,
                                             C.c_void_p(red2_ptr)))

    def fitc_finish(self, red2_ptr, nparams):
        obj = C.c_double(0.0)
        grad = np.zeros(nparams, dtype=np.float64)
        _lib.check(self._lib.sgp_fitc_finish(self.handle, C.c_void_p(red2_ptr), C.byref(obj),
                                             _lib.dptr(grad)))
        return obj.value, grad

    def vi_finish(self, red2_ptr, nparams):
        obj = C.c_double(0.0)
        grad = np.zeros(nparams, dtype=np.float64)
        _lib.check(self._lib.sgp_vi_finish(self.handle, C.c_void_p(red2_ptr), C.byref(obj),
                                           _lib.dptr(grad)))
        return obj.value, grad


# ---------------------------------------------------------------------- reference-named API
_CTX_CACHE = {}


def _fingerprint(a):
    """Shape plus a strided sample of the values: a cheap guard against arrays mutated in
    place between calls (the context holds a device copy taken at creation)."""
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    step = max(1, a.size // 4096)
    return (a.size, float(np.sum(a[::step])), float(a[-1]) if a.size else 0.0)


def _context_for(xy, y, mu, m, mu_vec=None):
    """Reuse one device context per (xy, y, mu), like the reference driver reuses xy across
    iterations.  Arrays are keyed by identity plus a sampled fingerprint; a scalar mu (the
    mean(y) default, quirk Q14) is keyed by value.  mu_vec: the mean actually uploaded; with
    mu=None it is the path's own default (a broadcast scalar: mean(y) for VI / FITC, log mean(y)
    for Laplace) and the key is that value, so paths with different defaults never share a
    context."""
    if mu is None:
        if mu_vec is None:
            raise ValueError("mu=None: the caller must resolve the path's default mean")
        mu_key = ("scalar", float(np.asarray(mu_vec, dtype=np.float64).reshape(-1)[0]))
    elif np.ndim(mu) == 0:
        mu_key = ("scalar", float(mu))
    else:
        mu_key = ("array", id(mu), _fingerprint(mu))
    key = (id(xy), id(y), mu_key, _fingerprint(xy), _fingerprint(y))
    ent = _CTX_CACHE.get(key)
    if ent is not None and ent[0] is xy and ent[1] is y and ent[2].m_max >= m:
        return ent[2]
    ctx = SparseGPContext(xy, y, mu if mu_vec is None else mu_vec, m_max=m)
    _CTX_CACHE.clear()
    _CTX_CACHE[key] = (xy, y, ctx)
    return ctx


def _mu_vec(mu, y):
    return np.broadcast_to(np.asarray(mu, dtype=np.float64), np.asarray(y).reshape(-1).shape)


def knot_fun_kind(dcov_fun_dknot):
    """None (knots fixed), or "sqexp" / "ard" for dsqexp_dx2 / dsqexp_dx2_ard
    (R/covariance_function_derivatives.R:178-302): accepts those names or functions so named."""
    if dcov_fun_dknot is None or dcov_fun_dknot is False:
        return None
    if isinstance(dcov_fun_dknot, float) and np.isnan(dcov_fun_dknot):
        return None
    name = dcov_fun_dknot if isinstance(dcov_fun_dknot, str) else getattr(dcov_fun_dknot,
                                                                          "__name__", "")
    if name in ("sqexp", "dsqexp_dx2"):
        return "sqexp"
    if name in ("ard", "dsqexp_dx2_ard"):
        return "ard"
    raise ValueError(f"unsupported dcov_fun_dknot {dcov_fun_dknot!r}")


def knot_bounds(xy):
    """vi_functions.R:175-178: column range of xy widened by a tenth on each side (d x 2)."""
    xy = np.asarray(xy, dtype=np.float64).reshape(np.shape(xy)[0], -1)
    lo, hi = xy.min(axis=0), xy.max(axis=0)
    diffs = hi - lo
    return np.column_stack([lo - diffs / 10, hi + diffs / 10])


def _knot_outputs(ctx, xu, xy, knot_opt):
    b = knot_bounds(xy)
    g = ctx.knot_gradient(b)
    U = np.asarray(xu, dtype=np.float64).reshape(-1, b.shape[0])
    if knot_opt is not None:
        keep = np.zeros(U.shape[0], dtype=bool)
        keep[np.asarray(list(knot_opt), dtype=int) - 1] = True
        g = g * np.repeat(keep, U.shape[1])
    trans = np.log((U - b[:, 0]) + 1e-4) - np.log((b[:, 1] - U) + 1e-4)
    return g, trans


def vi_eval(cov_par, cov_fun, xu, xy, y, mu, delta=1e-6, ctx=None, r_det=False, obj_only=False):
    """One fused evaluation: (ELBO, OrderedDict gradient in names(cov_par) order; None with
    obj_only)."""
    xy_m = np.asarray(xy, dtype=np.float64)
    d = 1 if xy_m.ndim == 1 else xy_m.shape[1]
    lnames = [f"l{c + 1}" for c in range(d)] if cov_fun == "ard" else None
    theta = theta_vector(cov_par, cov_fun, d, lnames)
    names = param_names(cov_fun, d, lnames)
    xu_m = np.asarray(xu, dtype=np.float64).reshape(-1, d)
    if mu is None:
        mu = np.mean(np.asarray(y, dtype=np.float64))                   # quirk Q14
    if ctx is None:
        ctx = _context_for(xy, y, mu, xu_m.shape[0])
    obj, g = ctx.eval_vi(theta, cov_fun, xu_m, delta, r_det=r_det, obj_only=obj_only)
    if obj_only:
        return obj, None
    byname = dict(zip(names, g))
    grad = OrderedDict((k, float(byname[k])) for k in cov_par.keys())
    return obj, grad


def fitc_eval(cov_par, cov_fun, xu, xy, y, mu, delta=1e-6, ctx=None, r_det=False,
              obj_only=False):
    """One fused FITC evaluation: (log marginal likelihood, OrderedDict gradient) with Z and the
    matrices built as norm_grad_ascent does (laplace_gradient_ascent.R:1238-1263); obj_only:
    obj_fun_norm alone (gradient None)."""
    xy_m = np.asarray(xy, dtype=np.float64)
    d = 1 if xy_m.ndim == 1 else xy_m.shape[1]
    lnames = [f"l{c + 1}" for c in range(d)] if cov_fun == "ard" else None
    theta = theta_vector(cov_par, cov_fun, d, lnames)
    names = param_names(cov_fun, d, lnames)
    xu_m = np.asarray(xu, dtype=np.float64).reshape(-1, d)
    if mu is None:
        mu = np.mean(np.asarray(y, dtype=np.float64))
    if ctx is None:
        ctx = _context_for(xy, y, mu, xu_m.shape[0])
    obj, g = ctx.eval_fitc(theta, cov_fun, xu_m, delta, r_det=r_det, obj_only=obj_only)
    if obj_only:
        return obj, None
    byname = dict(zip(names, g))
    return obj, OrderedDict((k, float(byname[k])) for k in cov_par.keys())


def dlogp_dcov_par(cov_par, cov_fun, dcov_fun_dtheta=True, dcov_fun_dknot=None, knot_opt=None,
                   xu=None, xy=None, y=None, ff=None, mu=None, transform=True, delta=1e-6,
                   ctx=None):
    """laplace_approx_gradient.R:720-971 (FITC, knots fixed): {"gradient", "trans_par"}."""
    kind = knot_fun_kind(dcov_fun_dknot)
    if mu is None:
        mu = np.mean(np.asarray(y, dtype=np.float64))
    xu_m = np.asarray(xu, dtype=np.float64).reshape(-1, np.asarray(xy).reshape(len(y), -1).shape[1])
    if ctx is None:
        ctx = _context_for(xy, y, mu, xu_m.shape[0])
    ctx.enable_knot_grad(kind is not None)
    _, grad = fitc_eval(cov_par, cov_fun, xu, xy, y, _mu_vec(mu, y), delta, ctx=ctx)
    if not dcov_fun_dtheta:
        grad = 0
    trans_par = OrderedDict((k, float(np.log(v))) for k, v in cov_par.items())
    if kind is not None:
        gk, tk = _knot_outputs(ctx, xu_m, xy, knot_opt)
        return {"gradient": grad, "knot_gradient": gk, "trans_par": trans_par, "trans_knot": tk}
    return {"gradient": grad, "trans_par": trans_par}


def elbo_fun(cov_par, cov_fun, xu, xy, y, mu, delta=1e-6, ctx=None, r_det=False):
    """ELBO value (vi_functions.R:64-121) at (cov_par, xu)."""
    return vi_eval(cov_par, cov_fun, xu, xy, y, mu, delta, ctx=ctx, r_det=r_det,
                   obj_only=True)[0]


def delbo_dcov_par(cov_par, cov_fun, dcov_fun_dtheta=True, dcov_fun_dknot=None, knot_opt=None,
                   xu=None, xy=None, y=None, ff=None, mu=None, transform=True, delta=1e-6,
                   ctx=None):
    """vi_functions.R:126-602 with knots fixed: {"gradient", "trans_par"} like the reference."""
    kind = knot_fun_kind(dcov_fun_dknot)
    if mu is None:
        mu = np.mean(np.asarray(y, dtype=np.float64))                   # quirk Q14
    xu_m = np.asarray(xu, dtype=np.float64).reshape(-1, np.asarray(xy).reshape(len(y), -1).shape[1])
    if ctx is None:
        ctx = _context_for(xy, y, mu, xu_m.shape[0])
    ctx.enable_knot_grad(kind is not None)
    _, grad = vi_eval(cov_par, cov_fun, xu, xy, y, _mu_vec(mu, y), delta, ctx=ctx)
    if not dcov_fun_dtheta:
        grad = 0
    trans_par = OrderedDict((k, float(np.log(v))) for k, v in cov_par.items())
    if kind is not None:
        gk, tk = _knot_outputs(ctx, xu_m, xy, knot_opt)
        return {"gradient": grad, "knot_gradient": gk, "trans_par": trans_par, "trans_knot": tk}
    return {"gradient": grad, "trans_par": trans_par}
