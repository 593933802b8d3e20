"""Row-sharded evaluation through the real HIP backend (device-pointer phase API of libsgp),
2 ranks on the box's single GPU, reductions over gloo (the 8-GPU RCCL run is the driver's)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import sgp_oracle as O
        from sparsergps_amd.dist import HipRowBackend, RowShardedVI, shard_rows
        P = O.make_gaussian_problem("C3", n=3001, m=200)
        U = P["U"].copy()
        U[:2] = P["X"][[5, 2999]]                     # coincident knots on both shards
        s0, s1 = shard_rows(3001, world, rank)
        be = HipRowBackend(P["X"][s0:s1], P["y"][s0:s1], P["mu"][s0:s1], 200, 0, "ard", mode)
        theta = np.array(list(P["cov_par"].values()))
        obj, grad = RowShardedVI(be, 3001).eval(theta, U, P["delta"])
        be.close()
        if rank == 0:
            fo, fg = (O.elbo_eval, O.delbo_dcov_par) if mode == "vi" else (O.fitc_obj_eval,
                                                                            O.dlogp_dcov_par)
            o = fo(P["cov_par"], "ard", U, P["X"], P["y"], P["mu"], P["delta"])
            g = np.array(list(fg(P["cov_par"], "ard", U, P["X"], P["y"], P["mu"],
                                 P["delta"])["gradient"].values()))
            q.put((abs(obj - o) / abs(o), float(np.max(np.abs(grad - g) / np.maximum(1, np.abs(g))))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["vi", "fitc"])
def test_two_ranks_one_gpu_gloo(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    rel_obj, rel_grad = q.get(timeout=5)
    assert rel_obj < 1e-9 and rel_grad < 1e-7


def _lap_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import sgp_oracle as O
        from sparsergps_amd.dist import HipRowBackend, RowShardedLaplace, shard_rows
        n, m = 2501, 150
        P = O.make_poisson_problem(n=n, m=m)
        U = P["U"].copy()
        U[:2] = P["X"][[5, n - 3]]
        s0, s1 = shard_rows(n, world, rank)
        be = HipRowBackend(P["X"][s0:s1], P["y"][s0:s1], P["mu"][s0:s1], m, 0, "sqexp", "laplace")
        be.ctx.lap_set_f(P["f0"][s0:s1])
        theta = np.array(list(P["cov_par"].values()))
        obj, grad, it = RowShardedLaplace(be).eval(theta, U, P["delta"], P["a"], 1e-5, 1000)
        be.close()
        if rank == 0:
            nr = O.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], U, P["y"], P["mu"],
                                    P["a"], P["delta"], tol=1e-5)
            g = np.array(list(O.dlogq_dcov_par(P["cov_par"], "sqexp", U, P["X"], P["y"], nr["gp"],
                                               P["mu"], P["a"], P["delta"])["gradient"].values()))
            o = nr["objective_function_values"][-1]
            q.put((abs(obj - o) / abs(o), float(np.max(np.abs(grad - g) / np.maximum(1, np.abs(g)))),
                   it, len(nr["objective_function_values"])))
    finally:
        dist.destroy_process_group()


def test_laplace_two_ranks_one_gpu_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    rel_obj, rel_grad, it, it_ref = q.get(timeout=5)
    assert it == it_ref
    assert rel_obj < 1e-9 and rel_grad < 1e-7


def _knot_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import sgp_oracle as O
        from sparsergps_amd.dist import HipRowBackend, RowShardedVI, shard_rows
        n, m = 151, 7
        P = O.make_gaussian_problem("C2", n=n, m=m)
        s0, s1 = shard_rows(n, world, rank)
        be = HipRowBackend(P["X"][s0:s1], P["y"][s0:s1], P["mu"][s0:s1], m, 0, "sqexp", "vi",
                           knots=True)
        theta = np.array(list(P["cov_par"].values()))
        RowShardedVI(be, n).eval(theta, P["U"], P["delta"])
        g = be.ctx.knot_gradient(O.knot_bounds_of(P["X"]))      # global bounds
        be.close()
        if rank == 0:
            ref = O.delbo_dcov_par(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], P["mu"],
                                   P["delta"], dcov_fun_dknot="sqexp")["knot_gradient"]
            q.put(float(np.max(np.abs(g - ref) / np.maximum(1, np.abs(ref)))))
    finally:
        dist.destroy_process_group()


def test_knot_gradient_two_ranks_one_gpu_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_knot_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert q.get(timeout=5) < 1e-7
