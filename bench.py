#!/usr/bin/env python
"""Benchmark: sparse-GP objective+gradient evals/sec at n=1e6, m=1024, d=8 (BASELINE.json).

One step = one full evaluation of the reference's optimizer-iteration body
(norm_grad_ascent_vi, R/vi_functions.R:1089-1128): build K12/K22 at (theta, U), the Titsias
ELBO and its gradient w.r.t. all P = 10 log-hyperparameters (knots fixed), on synthetic C3
inputs already resident in HBM.  N > 1: the n rows are split into N contiguous blocks (C4),
one process per GPU, RCCL all-reduce of the two reduction buffers (sparsergps_amd/dist.py);
total work is fixed, so scaling is "strong".

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1 under torch.distributed.run, one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix peak (AMD spec)
HBM_PEAK_GBS = 8000.0


def make_problem(config, n=None, m=None):
    """Synthetic inputs of SURVEY.md 8(d) (numpy PCG64 streams); no reference files read."""
    from sparsergps_amd.workloads import make_gaussian_problem, make_poisson_problem
    if config == "C5":
        return make_poisson_problem(n=n, m=m)
    return make_gaussian_problem(config, n=n, m=m)


def cpu_baseline(sizes=(500, 1000, 2000), n_target=1_000_000, m=1024):
    """Time the literal CPU restatement of the reference (oracle/) on row samples of C3 and
    extrapolate linearly in n (the reference's per-eval cost is a + b*n at fixed m)."""
    from threadpoolctl import threadpool_info

    from oracle import sgp_oracle as O
    ts = []
    for ns in sizes:
        P = make_problem("C3", n=ns, m=m)
        t0 = time.perf_counter()
        O.elbo_eval(P["cov_par"], "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        O.delbo_dcov_par(P["cov_par"], "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        ts.append(time.perf_counter() - t0)
    A = np.vstack([np.ones(len(sizes)), np.asarray(sizes, dtype=np.float64)]).T
    (a, b), *_ = np.linalg.lstsq(A, np.asarray(ts), rcond=None)
    resid = float(np.max(np.abs(A @ np.array([a, b]) - np.asarray(ts))))
    t_target = a + b * n_target
    threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    adj = cpu_adjoint(m=m, n_target=n_target)
    return {
        "value": 1.0 / t_target,
        "unit": "evals/s",
        "cores": int(threads),
        "kind": "port",
        "sample": (f"oracle/sgp_oracle.py elbo_eval+delbo_dcov_par (literal restatement of "
                   f"vi_functions.R, numpy+OpenBLAS) on C3 rows n={list(sizes)}, m={m}, d=8: "
                   f"t={[round(t, 3) for t in ts]} s; least-squares t(n)=a+b*n, a={a:.3f}s, "
                   f"b={b:.3e}s/row, max resid {resid:.3f}s; extrapolated to n={n_target}: "
                   f"{t_target:.1f} s/eval"),
        "adjoint_cpu": adj,
    }


def cpu_adjoint(sizes=(10000, 20000, 40000), n_target=1_000_000, m=1024):
    """Second CPU bar: the same adjoint algorithm the GPU runs (one SYRK + one
    K12 P contraction per eval), as the numpy model oracle/adjoint_ref.py, timed on C3 row
    samples and extrapolated linearly in n like the literal port."""
    from oracle import adjoint_ref as A
    W = make_problem("C3", n=1000, m=m)              # warm-up (BLAS thread pool, page faults)
    A.eval_vi("ard", np.array(list(W["cov_par"].values())), W["X"], W["y"], W["mu"], W["U"],
              W["delta"])
    ts = []
    for ns in sizes:
        P = make_problem("C3", n=ns, m=m)
        theta = np.array(list(P["cov_par"].values()))
        t0 = time.perf_counter()
        A.eval_vi("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"])
        ts.append(time.perf_counter() - t0)
    Amat = np.vstack([np.ones(len(sizes)), np.asarray(sizes, dtype=np.float64)]).T
    (a, b), *_ = np.linalg.lstsq(Amat, np.asarray(ts), rcond=None)
    t_target = a + b * n_target
    return {
        "value": 1.0 / t_target,
        "unit": "evals/s",
        "kind": "port (adjoint algorithm)",
        "sample": (f"oracle/adjoint_ref.py eval_vi (numpy+OpenBLAS) on C3 rows n={list(sizes)}, "
                   f"m={m}: t={[round(t, 3) for t in ts]} s; t(n)=a+b*n, a={a:.3f}s, "
                   f"b={b:.3e}s/row; extrapolated to n={n_target}: {t_target:.1f} s/eval"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", default="vi", choices=["vi", "fitc", "laplace"],
                    help="vi = the headline metric; fitc / laplace = secondary modes (SURVEY 8(d))")
    ap.add_argument("--config", default=None, choices=["C2", "C3", "C5"])
    ap.add_argument("--tol-nr", type=float, default=1e-5)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--knots", action="store_true",
                    help="also the m*d knot gradient (xu_opt = 'simultaneous', SURVEY 8(a) a16)")
    args = ap.parse_args()
    if args.config is None:
        args.config = "C5" if args.mode == "laplace" else "C3"
    if (args.mode == "laplace") != (args.config == "C5"):
        ap.error("--mode laplace goes with --config C5 (Poisson data); vi/fitc with C2/C3")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    import sparsergps_amd as S
    from sparsergps_amd.dist import HipRowBackend, RowShardedLaplace, RowShardedVI, shard_rows

    # SGP_BENCH_REHEARSE=1: every rank on device 0 with gloo collectives -- exercises the N > 1
    # control flow (sharding, barriers, max-over-ranks timing) on a one-GPU box; never used for
    # a reported number (RCCL is the product path)
    rehearse = os.environ.get("SGP_BENCH_REHEARSE") == "1"
    dev_index = 0 if rehearse else local_rank
    if world > 1:
        torch.cuda.set_device(dev_index)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
    dev = torch.device("cuda", dev_index)

    P = make_problem(args.config, n=args.n, m=args.m)
    n, m, d = P["X"].shape[0], P["U"].shape[0], P["X"].shape[1]
    cov_fun = P["cov_fun"]
    names = S.param_names(cov_fun, d)
    theta0 = np.array([P["cov_par"][k] for k in names])
    s0, s1 = shard_rows(n, world, rank)
    n_loc = s1 - s0

    backend = HipRowBackend(P["X"][s0:s1], P["y"][s0:s1], P["mu"][s0:s1], m, dev_index, cov_fun,
                            args.mode, knots=args.knots)
    ctx = backend.ctx
    nr_iters = []
    if args.mode == "laplace":
        ctx.lap_set_f(P["f0"][s0:s1])      # optimize_gp.R:480 start, then warm starts
        lap = RowShardedLaplace(backend, None)

        class _Runner:
            def eval(self, theta, U, delta):
                o, g, it = lap.eval(theta, U, delta, P["a"], args.tol_nr, 1000)
                nr_iters.append(it)
                return o, g
        runner = _Runner()
    else:
        vi = RowShardedVI(backend, n, None)
        if args.knots:
            # the knot bounds of the whole data set, as every rank must use them
            rng = P["X"].max(axis=0) - P["X"].min(axis=0)
            kb = np.stack([P["X"].min(axis=0) - rng / 10, P["X"].max(axis=0) + rng / 10], axis=1)

            class _KnotRunner:
                def eval(self, theta, U, delta):
                    o, g = vi.eval(theta, U, delta)
                    return o, (g, ctx.knot_gradient(kb))
            runner = _KnotRunner()
        else:
            runner = vi
    del P["X"]

    # an optimizer-like trajectory: theta moves every step (no result can be reused)
    def theta_at(k):
        return theta0 * np.exp(1e-3 * np.sin(np.arange(theta0.size) + k))

    for k in range(args.warmup):
        runner.eval(theta_at(k), P["U"], P["delta"])

    # HIP events bracket every phase on its launch stream during the timed steps; they are read
    # back once, after the timed region
    ctx.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    obj = None
    for k in range(args.steps):
        obj, grad = runner.eval(theta_at(args.warmup + k), P["U"], P["delta"])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    evals = max(ctx.timing_evals(), 1)
    phase_avg = {name: ms / evals for name, ms in ctx.timings()}
    ctx.enable_timing(False)
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    timed_iters = nr_iters[args.warmup:]

    # roofline of the dominant MFMA kernel, 2 n_loc m^2 flops per launch: VI's fused GEMM +
    # gradient contraction; FITC / Laplace's row-quadratic GEMM pass diag(K12 K22^-1 K21) (their
    # gradient passes read the products the row-quadratic passes stored, no GEMM of their own)
    con_key = {"vi": "contract_knm", "fitc": "rowquad_q", "laplace": "rowquad_q"}[args.mode]
    t_con = phase_avg.get(con_key, float("nan")) * 1e-3
    flops = 2.0 * n_loc * m * m
    achieved = flops / t_con / 1e12 if t_con > 0 else float("nan")
    traffic = None
    tp = os.path.join(ROOT, "profiles", "pmc_traffic_contract_knm.json")
    if os.path.exists(tp):
        try:
            rec = json.load(open(tp))
            if rec.get("n") == n_loc and rec.get("m") == m:
                traffic = rec.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        metric = {"vi": "sparse-GP objective+gradient evals/sec at n=1e6, m=1024, d=8",
                  "fitc": "FITC objective+gradient evals/sec (secondary mode)",
                  "laplace": "Poisson sparse-Laplace NR+objective+gradient evals/sec (C5, secondary)"}
        workload = {"vi": "Titsias VI ELBO + gradient", "fitc": "FITC log-likelihood + gradient",
                    "laplace": "Poisson Laplace: NR (warm start, tol_nr=%g) + obj_fun_pois + "
                               "dlogq_dcov_par" % args.tol_nr}[args.mode]
        out = {
            "metric": metric[args.mode],
            "value": args.steps / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (SURVEY.md 8(d) {args.config} generator, numpy PCG64)",
            "config": {"workload": f"{args.config}: {workload}, n={n}, m={m}, d={d}, "
                                   f"{cov_fun}, P={len(names)}, "
                                   + ("+ knot gradient (m*d)" if args.knots else "knots fixed"),
                       "n": n, "m": m, "d": d, "kernel": cov_fun,
                       "parallelism": f"rows{world}" if world > 1 else "single"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_MFMA_PEAK_TFLOPS,
                         "traffic": traffic if args.mode == "vi" else None,
                         "kernel": con_key + " (k_contract<8>)",
                         "flops_per_launch": flops},
            "phases_ms": {k: round(v, 4) for k, v in phase_avg.items()},
            "objective": obj,
        }
        if args.mode == "laplace":
            out["nr_iters_per_eval"] = timed_iters
        if world == 1 and not args.no_cpu_baseline and args.mode == "vi":
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    backend.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
