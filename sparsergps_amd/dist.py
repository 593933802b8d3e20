"""Row-sharded multi-GPU evaluation (one process per GPU, torch.distributed over RCCL/xGMI).

The reference is single-process R; its per-eval work is row-separable:
every n-indexed quantity (K12, r, alpha, the trace-term row sums, the gradient contraction)
lives on the rank that owns the row block, and the only exchange steps are the two sums of
sgp_vi_phase1 / sgp_vi_phase2 (include/sgp.h):
  all-reduce #1  S = K^T K (m x m), t = K^T r (m), r^T r      (8.4 MB at m = 1024)
  all-reduce #2  alpha^T alpha, sum G*dK partials, coincidence sums   (L + 5 doubles)
The m x m algebra between them is replicated on every rank (no broadcast).

``backend`` is any object with phase1/phase2/finish taking and returning torch tensors:
``HipRowBackend`` (the product path, device tensors) or the numpy model used by the gloo
tests (tests/test_dist.py).
"""
from __future__ import annotations

import contextlib
import os

import numpy as np


def _force_default():
    """SGP_FORCE_COLLECTIVES=1: issue the all-reduces even at world size 1, so that a one-GPU
    run exercises the RCCL path (stream ordering included) exactly as an 8-GPU run does."""
    return os.environ.get("SGP_FORCE_COLLECTIVES") == "1"


def shard_rows(n, world, rank):
    """Contiguous row block [start, stop) of rank `rank` (C4: 8 blocks of 125 000 rows)."""
    base, extra = divmod(int(n), int(world))
    start = rank * base + min(rank, extra)
    stop = start + base + (1 if rank < extra else 0)
    return start, stop


def global_knot_bounds(X_local, group=None):
    """d x 2 [lower, upper] knot bounds over all ranks' rows: column range widened by a tenth
    on each side (vi_functions.R:175-178); one MIN and one MAX all-reduce when distributed."""
    import torch
    import torch.distributed as dist
    X_local = np.asarray(X_local, dtype=np.float64)
    lo = torch.from_numpy(X_local.min(axis=0).copy())
    hi = torch.from_numpy(X_local.max(axis=0).copy())
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        if dist.get_backend(group) == "nccl":
            lo, hi = lo.cuda(), hi.cuda()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    lo, hi = lo.cpu().numpy(), hi.cpu().numpy()
    diff = hi - lo
    return np.column_stack([lo - diff / 10, hi + diff / 10])


class HipRowBackend:
    """libsgp.so context over this rank's rows; reduction buffers are torch device tensors.
    mode "vi" (sgp_vi_*) or "fitc" (sgp_fitc_*): both are phase1 -> sum -> phase2 -> sum ->
    finish; mode "laplace" (sgp_lap_*): begin -> sum -> step -> sum -> ... -> done."""

    def __init__(self, X_local, y_local, mu_local, m_max, device_index, cov_fun, mode="vi",
                 knots=False, group=None):
        import torch

        from .vi import SparseGPContext
        self.torch = torch
        self.dev = torch.device("cuda", device_index)
        self.ctx = SparseGPContext(X_local, y_local, mu_local, m_max=m_max, device=device_index)
        self.cov_fun = cov_fun
        self.mode = mode
        L = self.ctx.d if cov_fun == "ard" else 1
        self.nparams = L + 2
        if mode == "vi":
            n1, n2 = self.ctx.vi_red1_count(m_max), self.ctx.vi_red2_count(cov_fun)
        elif mode == "fitc":
            n1, n2 = self.ctx.fitc_red1_count(m_max), self.ctx.fitc_red2_count(cov_fun, m_max)
        elif mode == "laplace":
            n1 = n2 = self.ctx.lap_red_count(cov_fun, m_max)
        else:
            raise ValueError(mode)
        if knots:     # knot-gradient partials ride along in the second reduction
            self.ctx.enable_knot_grad(True)
            n2 += self.ctx.knot_red_extra(m_max)
        self.knots = knots
        # knot bounds of the whole data set (quirk Q9, vi_functions.R:175-178): every rank
        # must use the same ones, so the per-rank column ranges are combined once here, over
        # the same process group the sharded driver reduces over
        self.knot_bounds = global_knot_bounds(X_local, group) if knots else None
        self.red1 = torch.zeros(n1, dtype=torch.float64, device=self.dev)
        self.red2 = torch.zeros(n2, dtype=torch.float64, device=self.dev)
        # A dedicated (non-null) stream shared by libsgp's launches and torch.distributed:
        # RowShardedVI issues its collectives under stream_context(), so every all-reduce is
        # ordered after the kernels that produced its buffer, with no host synchronisation.
        self.stream = torch.cuda.Stream(device=self.dev)
        self.ctx.set_stream(self.stream.cuda_stream)

    def stream_context(self):
        return self.torch.cuda.stream(self.stream)

    def set_packed_reduction(self, on=True):
        if self.mode == "vi":
            self.ctx.set_packed_reduction(on)

    def phase1(self, theta, U, delta):
        m = np.asarray(U).shape[0]
        if self.mode == "vi":
            buf = self.red1[:self.ctx.vi_red1_count(m)]
            self.ctx.vi_phase1(theta, self.cov_fun, U, delta, buf.data_ptr())
        else:
            buf = self.red1[:self.ctx.fitc_red1_count(m)]
            self.ctx.fitc_phase1(theta, self.cov_fun, U, delta, buf.data_ptr())
        self._m = m
        return buf

    def phase2(self, red1, n_global):
        extra = self.ctx.knot_red_extra(self._m) if self.knots else 0
        if self.mode == "vi":
            self.ctx.vi_phase2(red1.data_ptr(), n_global, self.red2.data_ptr())
            return self.red2[:self.ctx.vi_red2_count(self.cov_fun) + extra]
        buf = self.red2[:self.ctx.fitc_red2_count(self.cov_fun, self._m) + extra]
        self.ctx.fitc_phase2(red1.data_ptr(), n_global, buf.data_ptr())
        return buf

    def finish(self, red2):
        if self.mode == "vi":
            return self.ctx.vi_finish(red2.data_ptr(), self.nparams)
        return self.ctx.fitc_finish(red2.data_ptr(), self.nparams)

    # ---- Laplace state machine (ping-pong between red1 and red2)
    def lap_begin(self, theta, U, delta, expo, tol, maxit):
        cnt = self.ctx.lap_begin(theta, self.cov_fun, U, delta, expo, tol, maxit,
                                 self.red1.data_ptr())
        self._cur = 0
        return self.red1[:cnt]

    def lap_step(self, red):
        bufs = (self.red1, self.red2)
        src, dst = bufs[self._cur], bufs[self._cur ^ 1]
        cnt, done, obj, grad, it = self.ctx.lap_step(src.data_ptr(), dst.data_ptr(), self.nparams)
        self._cur ^= 1
        if done:
            return None, True, (obj, grad, it)
        return dst[:cnt], False, None

    def knot_gradient(self, bounds=None):
        """Row-major m*d knot gradient of the last evaluation (global bounds by default)."""
        return self.ctx.knot_gradient(self.knot_bounds if bounds is None else bounds)

    def close(self):
        self.ctx.close()


class RowShardedVI:
    """ELBO + gradient over row blocks held by the ranks of `group`.

    force_collectives: all-reduce even when the group has one rank (default: the
    SGP_FORCE_COLLECTIVES environment switch); a single rank otherwise skips them."""

    def __init__(self, backend, n_global, group=None, force_collectives=None):
        import torch.distributed as dist
        self.dist = dist
        self.backend = backend
        self.n_global = int(n_global)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        force = _force_default() if force_collectives is None else bool(force_collectives)
        if force and not dist.is_initialized():
            raise RuntimeError("force_collectives needs an initialised torch.distributed group")
        self.collective = self.world > 1 or force
        # all-reduce #1 carries S as its lower 64 x 64 blocks (8.4 -> 4.5 MB at m = 1024);
        # phase 2 unpacks on the device
        if self.collective and hasattr(backend, "set_packed_reduction"):
            backend.set_packed_reduction(True)

    def eval(self, theta, U, delta=1e-6):
        b = self.backend
        # the torch stream context orders the collectives after libsgp's kernels (and the next
        # phase's kernels after the collective), with no host synchronisation in between
        use_ctx = self.collective and hasattr(b, "stream_context")
        with (b.stream_context() if use_ctx else contextlib.nullcontext()):
            red1 = b.phase1(theta, U, delta)
            if self.collective:
                self.dist.all_reduce(red1, group=self.group)
            red2 = b.phase2(red1, self.n_global)
            if self.collective:
                self.dist.all_reduce(red2, group=self.group)
            return b.finish(red2)


class RowShardedLaplace:
    """Poisson sparse-Laplace evaluation (NR to the mode + gradient) over row blocks.

    The NR loop is the reference's (R/newtrap_sparseGP.R:76-131); each iteration has two
    exchange steps -- K^T (grad_psi / (1 - Z W)) with the stop-rule count (m + 1 doubles) and
    the objective partials S_B, t_Z, scalars (m^2 + m + 3) -- and the gradient two more.  Every
    decision is a function of summed buffers, so all ranks iterate identically.
    """

    def __init__(self, backend, group=None, force_collectives=None):
        import torch.distributed as dist
        self.dist = dist
        self.backend = backend
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        force = _force_default() if force_collectives is None else bool(force_collectives)
        if force and not dist.is_initialized():
            raise RuntimeError("force_collectives needs an initialised torch.distributed group")
        self.collective = self.world > 1 or force

    def eval(self, theta, U, delta=1e-6, expo=1.0, tol=1e-5, maxit=1000):
        """-> (objective, gradient d/dlog theta, NR iteration count).  expo: the Poisson
        exposure, a scalar or THIS rank's rows of a per-row exposure (the reference's `m` as a
        vector of cell areas, R/derivative_functions_of_data_likelihoods.R:38)."""
        b = self.backend
        with (b.stream_context() if hasattr(b, "stream_context") else contextlib.nullcontext()):
            red = b.lap_begin(theta, U, delta, expo, tol, maxit)
            while True:
                if self.collective:
                    self.dist.all_reduce(red, group=self.group)
                red, done, res = b.lap_step(red)
                if done:
                    return res
