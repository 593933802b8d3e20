"""Multi-rank row sharding on CPU: world_size 2 (and 3) over gloo.

The product backend (HipRowBackend) needs a GPU; here the same driver
(sparsergps_amd.dist.RowShardedVI) runs the numpy model of libsgp's phase protocol
(oracle/adjoint_ref.py) on each rank's row block, with the two all-reduces going through
torch.distributed/gloo, and the result must equal the single-process literal oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sparsergps_amd.dist import RowShardedLaplace, RowShardedVI, shard_rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class NumpyBackend:
    """Test backend: numpy phases, torch CPU tensors as the reduction buffers."""

    def __init__(self, X, y, mu, cov_fun, mode="vi"):
        from oracle import adjoint_ref
        self.rk = (adjoint_ref.NumpyVIRank if mode == "vi" else adjoint_ref.NumpyFITCRank)(X, y, mu)
        self.cov_fun = cov_fun

    def phase1(self, theta, U, delta):
        return torch.from_numpy(self.rk.phase1(self.cov_fun, theta, U, delta))

    def phase2(self, red1, n_global):
        return torch.from_numpy(self.rk.phase2(red1.numpy(), n_global))

    def finish(self, red2):
        return self.rk.finish(red2.numpy())


def _worker(rank, world, port, cfg, n, m, coinc, q, mode="vi"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import sgp_oracle as O
        P = O.make_gaussian_problem(cfg, n=n, m=m)
        U = P["U"].copy()
        if coinc:
            U[:3] = P["X"][[0, n // 2, n - 1]]
        s0, s1 = shard_rows(n, world, rank)
        be = NumpyBackend(P["X"][s0:s1], P["y"][s0:s1], P["mu"][s0:s1], P["cov_fun"], mode)
        runner = RowShardedVI(be, n)
        theta = np.array(list(P["cov_par"].values()))
        obj, grad = runner.eval(theta, U, P["delta"])
        if rank == 0:
            fo, fg = (O.elbo_eval, O.delbo_dcov_par) if mode == "vi" else (O.fitc_obj_eval, O.dlogp_dcov_par)
            o = fo(P["cov_par"], P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])
            g = fg(P["cov_par"], P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])
            gv = np.array(list(g["gradient"].values()))
            q.put((abs(obj - o) / abs(o), float(np.max(np.abs(grad - gv) / np.maximum(1, np.abs(gv))))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,cfg,n,m,coinc,mode", [(2, "C2", 301, 17, False, "vi"),
                                                       (2, "C3", 250, 11, True, "vi"),
                                                       (3, "C2", 200, 9, True, "vi"),
                                                       (2, "C3", 240, 10, True, "fitc"),
                                                       (3, "C2", 211, 12, False, "fitc")])
def test_row_sharded_gloo(world, cfg, n, m, coinc, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, n, m, coinc, q, mode))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    rel_obj, rel_grad = q.get(timeout=5)
    assert rel_obj < 1e-12 and rel_grad < 1e-10


def test_shard_rows_partition():
    for n in (1, 7, 1000, 1_000_000):
        for w in (1, 2, 3, 8):
            blocks = [shard_rows(n, w, r) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
    assert shard_rows(1_000_000, 8, 3) == (375_000, 500_000)    # C4: 8 blocks of 125 000


class NumpyLaplaceBackend:
    def __init__(self, X, y, mu, f0, cov_fun):
        from oracle import adjoint_ref
        self.rk = adjoint_ref.NumpyLaplaceRank(X, y, mu)
        self.rk.set_f(f0)
        self.cov_fun = cov_fun

    def lap_begin(self, theta, U, delta, expo, tol, maxit):
        return torch.from_numpy(self.rk.begin(self.cov_fun, theta, U, delta, expo, tol, maxit))

    def lap_step(self, red):
        nxt, done, res = self.rk.step(red.numpy())
        if done:
            return None, True, (res[0], res[1], len(self.rk.objs))
        return torch.from_numpy(nxt), False, None


def _lap_worker(rank, world, port, n, m, q, per_row=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import sgp_oracle as O
        P = O.make_poisson_problem(n=n, m=m, per_row_exposure=per_row)
        U = P["U"].copy()
        U[:2] = P["X"][[1, n - 2]]                      # coincident knots on both shards
        s0, s1 = shard_rows(n, world, rank)
        be = NumpyLaplaceBackend(P["X"][s0:s1], P["y"][s0:s1], P["mu"][s0:s1], P["f0"][s0:s1],
                                 "sqexp")
        theta = np.array(list(P["cov_par"].values()))
        # a per-row exposure travels with its rows: each rank passes its own slice
        expo = P["a"][s0:s1] if per_row else P["a"]
        obj, grad, it = RowShardedLaplace(be).eval(theta, U, P["delta"], expo, 1e-5, 1000)
        if rank == 0:
            nr = O.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], U, P["y"], P["mu"],
                                    P["a"], P["delta"], tol=1e-5)
            g = O.dlogq_dcov_par(P["cov_par"], "sqexp", U, P["X"], P["y"], nr["gp"], P["mu"],
                                 P["a"], P["delta"])["gradient"]
            gv = np.array(list(g.values()))
            o = nr["objective_function_values"][-1]
            q.put((abs(obj - o) / abs(o), float(np.max(np.abs(grad - gv) / np.maximum(1, np.abs(gv)))),
                   it, len(nr["objective_function_values"])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,per_row", [(2, False), (3, False), (2, True)])
def test_row_sharded_laplace_gloo(world, per_row):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lap_worker, args=(r, world, port, 301, 19, q, per_row))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    rel_obj, rel_grad, it, it_ref = q.get(timeout=5)
    assert it == it_ref
    assert rel_obj < 1e-12 and rel_grad < 1e-10
