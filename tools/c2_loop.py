"""Evaluation rate at a config through three host paths on one GPU: the bench's RowShardedVI
(phase1 / phase2 / finish as three ctypes calls), SparseGPContext.eval_vi (one fused
sgp_eval_vi call) with theta converted per call, and the same with the knots pre-converted.
The differences are host-side overhead between consecutive evaluations.
usage: python3 tools/c2_loop.py [C2|C3] [evals]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import sparsergps_amd as S
    from bench import make_problem
    from sparsergps_amd.dist import HipRowBackend, RowShardedVI

    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    evals = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    P = make_problem(cfg)
    names = S.param_names(P["cov_fun"], P["X"].shape[1])
    th0 = np.array([P["cov_par"][k] for k in names])
    b = HipRowBackend(P["X"], P["y"], P["mu"], P["U"].shape[0], 0, P["cov_fun"], "vi")
    vi = RowShardedVI(b, P["X"].shape[0], None, force_collectives=False)
    ctx = b.ctx
    U, delta = P["U"], P["delta"]
    Uf = np.asfortranarray(U)
    thetas = [th0 * np.exp(1e-3 * np.sin(np.arange(th0.size) + k)) for k in range(evals + 10)]

    def run(fn):
        for k in range(5):
            fn(thetas[k])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(evals):
            fn(thetas[5 + k])
        torch.cuda.synchronize()
        return evals / (time.perf_counter() - t0)

    for rep in range(2):
        r1 = run(lambda th: vi.eval(th, U, delta))
        r2 = run(lambda th: ctx.eval_vi(th, P["cov_fun"], U, delta))
        r3 = run(lambda th: ctx.eval_vi(th, P["cov_fun"], Uf, delta))
        print(f"{cfg} rep {rep}: RowShardedVI {r1:8.1f}  eval_vi {r2:8.1f}  eval_vi(fortran U) {r3:8.1f} evals/s")
    b.close()


if __name__ == "__main__":
    main()
