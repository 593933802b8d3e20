"""Host-side cost of one VI evaluation on the GPU (no profiler attached).

Times, per evaluation of the bench's loop (RowShardedVI over one HipRowBackend, as bench.py
runs it at N = 1): the host time inside sgp_vi_phase1 / sgp_vi_phase2 (launch issue only),
inside sgp_vi_finish (waits for the GPU, then the readback), and the Python time between
evaluations.  With the GPU the bottleneck, phase1 + phase2 issue time overlaps the previous
kernels; what the GPU sees as idle is finish's tail + the Python gap + phase 1's issue up to
its first launch.  usage: python3 tools/host_overhead.py [C2|C3] [n] [evals]
"""
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

    config = sys.argv[1] if len(sys.argv) > 1 else "C2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    evals = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    P = make_problem(config, n=n)
    names = S.param_names(P["cov_fun"], P["X"].shape[1])
    theta0 = np.array([P["cov_par"][k] for k in names])
    b = HipRowBackend(P["X"], P["y"], P["mu"], P["U"].shape[0], 0, P["cov_fun"], "vi")
    vi = RowShardedVI(b, P["X"].shape[0], None, force_collectives=False)
    U, delta = P["U"], P["delta"]

    t_p1, t_p2, t_fin, t_gap, t_all = [], [], [], [], []
    prev_end = None
    for k in range(evals + 5):
        th = theta0 * np.exp(1e-3 * np.sin(np.arange(theta0.size) + k))
        a = time.perf_counter()
        red1 = b.phase1(th, U, delta)
        c1 = time.perf_counter()
        red2 = b.phase2(red1, vi.n_global)
        c2 = time.perf_counter()
        b.finish(red2)
        e = time.perf_counter()
        if k >= 5:
            t_p1.append(c1 - a)
            t_p2.append(c2 - c1)
            t_fin.append(e - c2)
            t_all.append(e - a)
            if prev_end is not None:
                t_gap.append(a - prev_end)
        prev_end = e
    torch.cuda.synchronize()
    us = lambda v: f"{np.median(v) * 1e6:8.1f} us"
    print(f"{config} n={P['X'].shape[0]} m={U.shape[0]}: per evaluation (median of {evals})")
    print(f"  phase1 issue  {us(t_p1)}")
    print(f"  phase2 issue  {us(t_p2)}")
    print(f"  finish (wait + readback) {us(t_fin)}")
    print(f"  python gap between evaluations {us(t_gap)}")
    print(f"  eval wall     {us(t_all)}")
    b.close()


if __name__ == "__main__":
    main()
