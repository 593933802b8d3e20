"""Diagnostic: phase-by-phase comparison of libsgp's VI protocol with the numpy model
(oracle/adjoint_ref.py) for a list of (n, m) sizes.  Usage: python tools/diag_parity.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from oracle import sgp_oracle as O          # noqa: E402
from oracle import adjoint_ref as A         # noqa: E402
from sparsergps_amd.dist import HipRowBackend  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-300, np.max(np.abs(b))))


sizes = [tuple(map(int, s.split("x"))) for s in (sys.argv[1:] or
         ["20000x300", "20000x512", "20000x640", "20000x768", "20000x1024", "4000x1024", "3000x1024"])]
for n, m in sizes:
    P = O.make_gaussian_problem("C3", n=n, m=m)
    th = np.array(list(P["cov_par"].values()))
    for rep in range(int(os.environ.get("DIAG_REPS", "1"))):
        be = HipRowBackend(P["X"], P["y"], P["mu"], m, 0, "ard")
        rk = A.NumpyVIRank(P["X"], P["y"], P["mu"])
        r1 = be.phase1(th, P["U"], P["delta"])
        torch.cuda.synchronize()
        g1 = r1.cpu().numpy()
        n1 = rk.phase1("ard", th, P["U"], P["delta"])
        mm = m * m
        S_err = rel(g1[:mm], n1[:mm])
        t_err = rel(g1[mm:mm + m], n1[mm:mm + m])
        rr_err = rel(g1[mm + m:mm + m + 1], n1[mm + m:mm + m + 1])
        r2 = be.phase2(r1, n)
        torch.cuda.synchronize()
        g2 = r2.cpu().numpy()
        n2 = rk.phase2(n1, n)
        obj, grad = be.finish(r2)
        o, g = rk.finish(n2)
        if os.environ.get("SGP_DEBUG_SC"):
            print("[model sc]", {k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in rk.sc.items()},
                  file=sys.stderr, flush=True)
        print(f"n={n} m={m}: S {S_err:.2e} t {t_err:.2e} rr {rr_err:.2e} | red2 "
              f"{np.array2string(np.abs(g2[:len(n2)] - n2) / np.maximum(1, np.abs(n2)), precision=2)} | "
              f"obj {abs(obj - o) / abs(o):.2e} grad {rel(grad, g):.2e}", flush=True)
        be.close()
