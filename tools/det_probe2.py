"""Where FITC's run-to-run differences come from: red1 / red2 of repeated phases (bitwise)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import sparsergps_amd as S
    from sparsergps_amd.dist import HipRowBackend
    from sparsergps_amd.workloads import make_gaussian_problem
    for m in (64, 200):
        P = make_gaussian_problem("C2", n=12_000, m=m)
        th = np.array(list(P["cov_par"].values()))
        b = HipRowBackend(P["X"], P["y"], P["mu"], m, 0, "sqexp", "fitc")
        ref = None
        for rep in range(4):
            with b.stream_context():
                r1 = b.phase1(th, P["U"], P["delta"])
                a1 = r1.cpu().numpy().copy()
                r2 = b.phase2(r1, P["X"].shape[0])
                a2 = r2.cpu().numpy().copy()
                o, g = b.finish(r2)
            torch.cuda.synchronize()
            cur = (a1, a2, np.array([o]), np.asarray(g))
            if ref is None:
                ref = cur
                continue
            for nm, x, y in zip(("red1", "red2", "obj", "grad"), cur, ref):
                if not np.array_equal(x, y):
                    d = np.nonzero(x != y)[0]
                    print(f"m={m} rep {rep} {nm}: {d.size} of {x.size} differ, first idx {d[:6]}, "
                          f"max abs {np.max(np.abs(x - y)):.3e}")
        b.close()
        print(f"m={m} done")


if __name__ == "__main__":
    main()
