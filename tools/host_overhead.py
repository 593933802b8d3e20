#!/usr/bin/env python
"""Host-side cost of one VI evaluation at C3 on one GPU: wall time of each API call of the
phase protocol (the GPU runs asynchronously except in finish), to find host gaps between
evaluations.  usage: python tools/host_overhead.py [steps] [rows]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import sparsergps_amd as S
    from sparsergps_amd.workloads import make_gaussian_problem
    from sparsergps_amd.dist import HipRowBackend
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else None
    P = make_gaussian_problem("C3", n=rows)
    n, m = P["X"].shape[0], P["U"].shape[0]
    names = S.param_names("ard", 8)
    th0 = np.array([P["cov_par"][k] for k in names])
    b = HipRowBackend(P["X"], P["y"], P["mu"], m, 0, "ard", "vi")
    U = np.asfortranarray(P["U"])
    tt = {"pre": 0.0, "phase1": 0.0, "phase2": 0.0, "finish": 0.0, "ctx": 0.0}
    for k in range(steps + 2):
        t0 = time.perf_counter()
        th = th0 * np.exp(1e-3 * np.sin(np.arange(th0.size) + k))
        t1 = time.perf_counter()
        with b.stream_context():
            t2 = time.perf_counter()
            r1 = b.phase1(th, U, P["delta"])
            t3 = time.perf_counter()
            r2 = b.phase2(r1, n)
            t4 = time.perf_counter()
            obj, g = b.finish(r2)
            t5 = time.perf_counter()
        t6 = time.perf_counter()
        if k >= 2:
            tt["pre"] += t1 - t0
            tt["ctx"] += (t2 - t1) + (t6 - t5)
            tt["phase1"] += t3 - t2
            tt["phase2"] += t4 - t3
            tt["finish"] += t5 - t4
    for k, v in tt.items():
        print(f"{k:8s} {v / steps * 1e6:10.1f} us/eval")
    torch.cuda.synchronize()
    b.close()


if __name__ == "__main__":
    main()
