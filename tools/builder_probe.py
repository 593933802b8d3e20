#!/usr/bin/env python
"""The K12 builder next to this box's plain-store ceiling, in one process.

Runs `--evals` VI evaluations at C3 (each launches k_build_knm_mfma once: 8.19 GB of K12
stores) and then `--reps` passes of sgp_diag_store_bw's builder-shaped store stream over the
same byte count (k_diag_store_tile).  Meant to run under rocprofv3 --pmc, one counter set per
run (tools/gpu_run.sh step builderpmc); prints the ceiling it measured itself.
Reference: the K12 build of every optimizer iteration, R/vi_functions.R:733-753.
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--evals", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np

    import sparsergps_amd as S
    from sparsergps_amd import _lib
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C3")
    th = np.array(list(P["cov_par"].values()))
    with S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=1024) as ctx:
        for _ in range(a.evals):
            ctx.eval_vi(th, "ard", P["U"], P["delta"])
    n_pad = -(-P["X"].shape[0] // 128) * 128
    gbs = C.c_double(0.0)
    _lib.check(_lib.lib().sgp_diag_store_bw(0, 8 * n_pad * 1024, a.reps, 1, C.byref(gbs)))
    print(f"store ceiling {gbs.value:.1f} GB/s over {8 * n_pad * 1024 / 1e9:.3f} GB", flush=True)


if __name__ == "__main__":
    main()
