"""Diagnostic: repeated VI evaluations through HipRowBackend with switchable timing/graphs.

python tools/diag_eval.py N M WARMUP STEPS TIMING   (env SGP_NO_GRAPHS=1 disables graphs)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    n, m, warm, steps, timing = (int(a) for a in sys.argv[1:6])
    import torch  # noqa: F401
    from oracle.sgp_oracle import make_gaussian_problem
    from sparsergps_amd.dist import HipRowBackend, RowShardedVI
    P = make_gaussian_problem("C3", n=n, m=m)
    be = HipRowBackend(P["X"], P["y"], P["mu"], m, 0, "ard")
    run = RowShardedVI(be, n)
    th = np.array(list(P["cov_par"].values()))
    for k in range(warm + steps):
        if k == warm and timing:
            be.ctx.enable_timing(True)
        t0 = time.perf_counter()
        obj, g = run.eval(th * np.exp(1e-3 * np.sin(np.arange(th.size) + k)), P["U"], P["delta"])
        tl = be.ctx.timings() if (timing and k >= warm) else []
        print(k, f"{(time.perf_counter() - t0) * 1e3:.1f}ms", obj, g[0], [x[0] for x in tl][:3], flush=True)
    be.close()
    print("DONE", flush=True)


if __name__ == "__main__":
    main()
