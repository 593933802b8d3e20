"""RCCL rehearsal worker (launched as a child process by tests/test_gpu_rccl.py).

torch.distributed is initialised with the "nccl" backend (= RCCL on ROCm) at world size 1
BEFORE any other GPU work, and every row-sharded evaluation runs with force_collectives, so
the all-reduces of sparsergps_amd/dist.py go through RCCL on the library's stream exactly as
on an 8-GPU node.  Results are compared with the CPU oracle; one JSON line per case, exit 1 on
any failure.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"

    import numpy as np

    from oracle import adjoint_chunked as AC
    from oracle import sgp_oracle as O
    from sparsergps_amd.dist import HipRowBackend, RowShardedLaplace, RowShardedVI, shard_rows
    from sparsergps_amd.workloads import make_gaussian_problem

    def rel(a, b):
        return float(np.max(np.abs(np.asarray(a) - np.asarray(b)) /
                            np.maximum(1.0, np.abs(np.asarray(b)))))

    results = []

    def record(name, robj, rgrad, tol_obj, tol_grad, **extra):
        ok = robj < tol_obj and rgrad < tol_grad
        results.append(ok)
        print(json.dumps(dict(case=name, rel_obj=robj, rel_grad=rgrad, ok=ok, **extra)), flush=True)

    # VI and FITC through the forced collectives (coincident knots on the block)
    for mode in ("vi", "fitc"):
        P = O.make_gaussian_problem("C3", n=3001, m=200)
        U = P["U"].copy()
        U[:2] = P["X"][[5, 2999]]
        be = HipRowBackend(P["X"], P["y"], P["mu"], 200, 0, "ard", mode)
        theta = np.array(list(P["cov_par"].values()))
        runner = RowShardedVI(be, 3001, force_collectives=True)
        assert runner.collective
        obj, grad = runner.eval(theta, U, P["delta"])
        obj2, grad2 = runner.eval(theta, U, P["delta"])          # second pass: same buffers
        be.close()
        fo, fg = (O.elbo_eval, O.delbo_dcov_par) if mode == "vi" else (O.fitc_obj_eval,
                                                                        O.dlogp_dcov_par)
        o = fo(P["cov_par"], "ard", U, P["X"], P["y"], P["mu"], P["delta"])
        g = np.array(list(fg(P["cov_par"], "ard", U, P["X"], P["y"], P["mu"],
                             P["delta"])["gradient"].values()))
        record(f"{mode}_rccl", abs(obj - o) / abs(o), rel(grad, g), 1e-9, 1e-7,
               repeat_identical=bool(obj == obj2 and np.array_equal(grad, grad2)))

    # Laplace: one all-reduce per state-machine step
    n, m = 2501, 150
    P = O.make_poisson_problem(n=n, m=m)
    U = P["U"].copy()
    U[:2] = P["X"][[5, n - 3]]
    be = HipRowBackend(P["X"], P["y"], P["mu"], m, 0, "sqexp", "laplace")
    be.ctx.lap_set_f(P["f0"])
    theta = np.array(list(P["cov_par"].values()))
    obj, grad, it = RowShardedLaplace(be, force_collectives=True).eval(theta, U, P["delta"],
                                                                       P["a"], 1e-5, 1000)
    be.close()
    nr = O.newtrap_sparseGP(P["f0"], P["cov_par"], "sqexp", P["X"], U, P["y"], P["mu"], P["a"],
                            P["delta"], tol=1e-5)
    g = np.array(list(O.dlogq_dcov_par(P["cov_par"], "sqexp", U, P["X"], P["y"], nr["gp"],
                                       P["mu"], P["a"], P["delta"])["gradient"].values()))
    o = nr["objective_function_values"][-1]
    record("laplace_rccl", abs(obj - o) / abs(o), rel(grad, g), 1e-9, 1e-7,
           nr_iters=it, nr_iters_ref=len(nr["objective_function_values"]))
    results[-1] = results[-1] and it == len(nr["objective_function_values"])

    # knot gradient with the bounds combined over the group
    n, m = 151, 7
    P = O.make_gaussian_problem("C2", n=n, m=m)
    be = HipRowBackend(P["X"], P["y"], P["mu"], m, 0, "sqexp", "vi", knots=True)
    theta = np.array(list(P["cov_par"].values()))
    RowShardedVI(be, n, force_collectives=True).eval(theta, P["U"], P["delta"])
    gk = be.knot_gradient()
    be.close()
    ref = O.delbo_dcov_par(P["cov_par"], "sqexp", P["U"], P["X"], P["y"], P["mu"], P["delta"],
                           dcov_fun_dknot="sqexp")["knot_gradient"]
    record("knots_rccl", 0.0, rel(gk, ref), 1.0, 1e-7)

    # C4 shard shape: rank 3 of 8 over the C3 rows (n = 125 000, m = 1024, d = 8), checked
    # against the row-chunked adjoint model
    C = make_gaussian_problem("C3")
    s0, s1 = shard_rows(1_000_000, 8, 3)
    Xs, ys, mus = C["X"][s0:s1], C["y"][s0:s1], C["mu"][s0:s1]
    del C["X"]
    theta = np.array(list(C["cov_par"].values()))
    be = HipRowBackend(Xs, ys, mus, 1024, 0, "ard", "vi")
    obj, grad = RowShardedVI(be, s1 - s0, force_collectives=True).eval(theta, C["U"], C["delta"])
    be.close()
    o, g = AC.eval_vi("ard", theta, Xs, ys, mus, C["U"], C["delta"])
    record("c4_shard_125000_rccl", abs(obj - o) / abs(o), rel(grad, g), 1e-9, 1e-7,
           n=int(s1 - s0), m=1024, d=8)

    dist.destroy_process_group()
    return 0 if all(results) else 1


if __name__ == "__main__":
    sys.exit(main())
