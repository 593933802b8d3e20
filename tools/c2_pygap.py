"""Where the ~22 us between two C2 evaluations goes on the Python side (bench.py's one-GPU loop
shape), with the -DSGP_HOST_PROBE variant (SGP_AB_LIB=tools/ab/hprobe/libsgp.so): per
evaluation, Python before the call (theta update + wrapper up to sgp_eval_vi's entry), the call's
host time inside the library (entry -> exit), and Python after it (exit -> back in the loop).
usage: SGP_AB_LIB=tools/ab/hprobe/libsgp.so python3 tools/c2_pygap.py [evals]"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bench import make_problem
    from sparsergps_amd import _lib
    from sparsergps_amd.dist import HipRowBackend

    evals = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    P = make_problem("C2")
    n, m = P["X"].shape[0], P["U"].shape[0]
    be = HipRowBackend(P["X"], P["y"], P["mu"], m, 0, P["cov_fun"], "vi")
    ctx = be.ctx
    pt = (C.c_double * 4).in_dll(_lib.lib(), "sgp_probe_t")
    theta0 = np.array(list(P["cov_par"].values()))

    def theta_at(k):
        return theta0 * np.exp(1e-3 * np.sin(np.arange(theta0.size) + k))

    for k in range(20):
        ctx.eval_vi(theta_at(k), P["cov_fun"], P["U"], P["delta"])
    pre, inside, post, loop = [], [], [], []
    for k in range(evals):
        a = time.perf_counter()
        th = theta_at(k)
        b = time.perf_counter()
        ctx.eval_vi(th, P["cov_fun"], P["U"], P["delta"])
        c = time.perf_counter()
        pre.append(pt[0] - b)
        inside.append(pt[3] - pt[0])
        post.append(c - pt[3])
        loop.append(b - a)
    us = lambda v: 1e6 * float(np.median(v))
    print(f"theta update {us(loop):.1f} us, wrapper before entry {us(pre):.1f} us, "
          f"library {us(inside):.1f} us, wrapper after exit {us(post):.1f} us (medians)")


if __name__ == "__main__":
    main()
