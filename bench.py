#!/usr/bin/env python
"""Benchmark: sparse-GP objective+gradient evals/sec at n=1e6, m=1024, d=8 (BASELINE.json).

One step = one full evaluation of the reference's optimizer-iteration body
(norm_grad_ascent_vi, R/vi_functions.R:1089-1128): build K12/K22 at (theta, U), the Titsias
ELBO and its gradient w.r.t. all P = 10 log-hyperparameters (knots fixed), on synthetic C3
inputs already resident in HBM.  N > 1: the n rows are split into N contiguous blocks (C4)
and the two reduction buffers are all-reduced over RCCL; total work is fixed, so scaling is
"strong".  --gpus N always means N GPUs (plan_run):
  * under torch.distributed.run (RANK in the environment): one process per GPU
    (sparsergps_amd/dist.py); --gpus must equal WORLD_SIZE;
  * without it and N > 1: one process over devices 0..N-1 through the in-library multi-device
    context (sgp_ctx_create_multi, RCCL inside libsgp) -- the path the R drop-in takes;
  * N larger than the visible devices, or < 1, is an error: never a silent one-GPU run.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
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


def make_problem(config, n=None, m=None, d=None):
    """Synthetic inputs of SURVEY.md 8(d) (numpy PCG64 streams); no reference files read."""
    from sparsergps_amd.workloads import make_gaussian_problem, make_poisson_problem
    if config == "C5":
        return make_poisson_problem(n=n, m=m)
    return make_gaussian_problem(config, n=n, m=m, d=d)


def cpu_info():
    """Host CPU model, logical CPUs visible to this process and physical cores among them."""
    model, cores = "unknown", set()
    try:
        allowed = os.sched_getaffinity(0)
    except AttributeError:
        allowed = set(range(os.cpu_count() or 1))
    try:
        proc = phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "processor":
                proc = int(v)
            elif k == "model name":
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
                if proc in allowed:
                    cores.add((phys, core))
    except OSError:
        pass
    return {"model": model, "logical_cpus": len(allowed),
            "physical_cores": len(cores) or None, **cpu_quota()}


def cpu_quota():
    """The CPU share this process may use: the cgroup CPU quota (v2 cpu.max, or v1
    cfs_quota_us / cfs_period_us) and OMP_NUM_THREADS, which the GPU boxes set to that share.
    On those boxes affinity and /proc/cpuinfo show the whole host, not the share."""
    raw, cpus = None, None
    try:
        raw = open("/sys/fs/cgroup/cpu.max").read().strip()
        q, _, per = raw.partition(" ")
        if q != "max":
            cpus = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            raw = f"cfs_quota_us={q} cfs_period_us={per}"
            cpus = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    return {"cgroup_cpu_max": raw, "cgroup_quota_cpus": cpus,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def _blas_threads():
    from threadpoolctl import threadpool_info
    return max([i.get("num_threads", 1) for i in threadpool_info()] or [1])


def _time_literal(ns, m, threads=None):
    """One literal-port evaluation (elbo_fun + delbo_dcov_par) at C3 rows n = ns."""
    from threadpoolctl import threadpool_limits

    from oracle import sgp_oracle as O
    P = make_problem("C3", n=ns, m=m)
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        O.elbo_eval(P["cov_par"], "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        O.delbo_dcov_par(P["cov_par"], "ard", P["U"], P["X"], P["y"], P["mu"], P["delta"])
        return time.perf_counter() - t0


def _fit(sizes, ts, n_target):
    """Least squares t(n) = a + b n; with >= 3 sizes the residual tests the linear model."""
    if len(sizes) < 3:
        raise ValueError("the linear fit needs at least three sizes to have a residual")
    A = np.vstack([np.ones(len(sizes)), np.asarray(sizes, dtype=np.float64)]).T
    (a, b), *_ = np.linalg.lstsq(A, np.asarray(ts), rcond=None)
    resid = A @ np.array([a, b]) - np.asarray(ts)
    return a, b, float(np.max(np.abs(resid) / np.asarray(ts))), a + b * n_target


def literal_port(sizes, n_target=1_000_000, m=1024, threads=None):
    """The reference-faithful restatement (oracle/sgp_oracle.py: the R operation graph --
    LU solves with n right-hand sides, per-parameter GEMM chains -- on numpy + OpenBLAS) timed
    at C3 row counts; its cost is a + b n at fixed m, so it is fitted and extrapolated to n."""
    ts = []
    for ns in sizes:
        ts.append(_time_literal(ns, m, threads))
        print(f"[cpu] literal port n={ns} threads={threads or _blas_threads()}: {ts[-1]:.2f} s",
              file=sys.stderr, flush=True)
    a, b, rel, t_target = _fit(sizes, ts, n_target)
    return {"value": 1.0 / t_target, "unit": "evals/s", "sizes": list(sizes),
            "t_s": [round(t, 3) for t in ts], "fit": {"a_s": a, "b_s_per_row": b,
                                                       "max_rel_resid": rel},
            "t_target_s": t_target, "threads": threads or _blas_threads()}


def adjoint_direct(n=1_000_000, m=1024, chunk=8192):
    """The optimised CPU bar: the GPU's adjoint algorithm (oracle/adjoint_chunked.py, one SYRK
    + one K12 P contraction, row-chunked) on the host BLAS, timed directly at the full n."""
    from oracle import adjoint_chunked as AC
    P = make_problem("C3", n=n, m=m)
    theta = np.array(list(P["cov_par"].values()))
    t0 = time.perf_counter()
    AC.eval_vi("ard", theta, P["X"], P["y"], P["mu"], P["U"], P["delta"], chunk=chunk)
    t = time.perf_counter() - t0
    return {"value": 1.0 / t, "unit": "evals/s", "kind": "port (adjoint algorithm)",
            "cores": _blas_threads(),
            "sample": f"oracle/adjoint_chunked.py eval_vi (numpy + OpenBLAS, {chunk}-row chunks) "
                      f"timed once directly at C3 n={n}, m={m}, d=8: {t:.2f} s/eval "
                      f"(no extrapolation)"}


def cpu_baseline(sizes=(2000, 5000, 8000), n_target=1_000_000, m=1024, full=None):
    """cpu_baseline of the bench line (bounded: ~30-60 s of host time): a three-point fit of
    the literal port plus the adjoint bar timed directly at the full n."""
    lit = literal_port(sizes, n_target, m)
    out = {
        "value": lit["value"],
        "unit": "evals/s",
        "cores": lit["threads"],
        "kind": "port",
        "cpu": cpu_info(),
        "sample": (f"oracle/sgp_oracle.py elbo_eval+delbo_dcov_par (literal restatement of "
                   f"vi_functions.R, numpy+OpenBLAS, {lit['threads']} BLAS threads) on C3 rows "
                   f"n={list(sizes)}, m={m}, d=8: t={lit['t_s']} s; t(n)=a+b*n, "
                   f"a={lit['fit']['a_s']:.3f}s, b={lit['fit']['b_s_per_row']:.3e}s/row, max "
                   f"rel resid {lit['fit']['max_rel_resid']:.3f}; extrapolated to "
                   f"n={n_target}: {lit['t_target_s']:.1f} s/eval"),
        "adjoint_cpu": adjoint_direct(n_target, m),
    }
    if full:
        out["full_plan"] = full
    return out


def cpu_baseline_full(n_target=1_000_000, m=1024):
    """SURVEY 8(d)'s whole CPU plan: the literal port on every CPU of this process's quota
    (BLAS threads = the share, see cpu_quota) at n in {1e4, 2e4, 5e4} and on one core at n in
    {2500, 5000, 1e4}, plus the adjoint bar timed directly at n = 1e6 (several minutes of host
    time: `python bench.py --cpu-full`)."""
    share = literal_port((10_000, 20_000, 50_000), n_target, m)
    one = literal_port((2_500, 5_000, 10_000), n_target, m, threads=1)
    return {"cpu": cpu_info(), "literal_quota_cores": share, "literal_one_core": one,
            "adjoint_direct": adjoint_direct(n_target, m)}


def store_ceiling(n_loc, m, device=0):
    """This box's HBM store ceiling for the K12 builder, measured in the same run
    (sgp_diag_store_bw: plain 16-byte non-temporal stores in the builder's 4-row x 256 B shape
    over the builder's byte count, best of 5 passes).  None when it cannot be measured."""
    import ctypes as C

    from sparsergps_amd import _lib
    n_pad = -(-n_loc // 128) * 128
    m_p = -(-m // 128) * 128
    gbs = C.c_double(0.0)
    st = _lib.lib().sgp_diag_store_bw(device, int(8 * n_pad * m_p), 5, 1, C.byref(gbs))
    return gbs.value if st == _lib.SGP_OK and gbs.value > 0 else None


def kernel_rooflines(mode, phase_avg, n_loc, m, ceiling=None):
    """The other hot kernels of the step against their own bounds (same HIP-event phase
    timings as roofline.achieved): the K12 builder writes 8 B per (row, knot) pair of the
    padded n_pad x m_p matrix (HBM-write bound; also against `ceiling`, this box's measured
    store rate); the SYRK does n m^2 algorithmic flops (fp64 MFMA bound)."""
    n_pad = -(-n_loc // 128) * 128
    m_p = -(-m // 128) * 128
    out = []
    t = phase_avg.get("build_knm", 0.0) * 1e-3
    if t > 0:
        gbs = 8.0 * n_pad * m_p / t / 1e9
        row = {"kernel": "build_knm (k_build_knm_mfma)", "bound": "hbm", "achieved": gbs,
               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
               "bytes_per_launch": 8.0 * n_pad * m_p}
        if ceiling:
            row["store_ceiling_gbs"] = ceiling
            row["frac_of_store_ceiling"] = gbs / ceiling
            row["store_ceiling_note"] = ("sgp_diag_store_bw on this box in this run: plain "
                                         "non-temporal 16-byte stores, the builder's shape and "
                                         "byte count, best of 5")
        out.append(row)
    key = {"vi": "syrk", "fitc": "syrk", "laplace": "syrk_z"}.get(mode)
    t = phase_avg.get(key, 0.0) * 1e-3
    if t > 0:
        tf = float(n_loc) * m * m / t / 1e12
        out.append({"kernel": key + " (k_syrk_blk)", "bound": "mfma", "achieved": tf,
                    "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": tf / FP64_MFMA_PEAK_TFLOPS, "flops_per_launch": float(n_loc) * m * m})
    return out


class PlanError(ValueError):
    """bench.py's --gpus / --devices / launcher combination cannot run as asked."""


def plan_run(gpus, devices, env, visible):
    """How `bench.py --gpus N` runs.  Returns ("torchrun", world) when launched by
    torch.distributed.run (RANK in env), ("library", device list) for the in-library
    multi-device context, or ("single", [0]).  `visible` is a callable giving the visible GPU
    count (only asked when needed).  Raises PlanError for every request that would otherwise
    time a different number of GPUs than N."""
    if gpus < 1:
        raise PlanError(f"--gpus {gpus}: at least one GPU")
    under_torchrun = "RANK" in env
    world = int(env.get("WORLD_SIZE", "1"))
    if devices is not None:
        if under_torchrun or world > 1:
            raise PlanError("--devices runs one process over several devices (not under "
                            "torchrun)")
        if not devices:
            raise PlanError("--devices: empty list")
        distinct = len(set(devices))
        if gpus != 1 and gpus != distinct:
            raise PlanError(f"--gpus {gpus} but --devices names {distinct} distinct device(s)")
        nvis = visible()
        bad = [dv for dv in devices if dv < 0 or dv >= nvis]
        if bad:
            raise PlanError(f"--devices {bad}: {nvis} device(s) visible")
        return "library", list(devices)
    if under_torchrun:
        if gpus != world:
            raise PlanError(f"--gpus {gpus} but torchrun started WORLD_SIZE={world} rank(s)")
        return "torchrun", world
    if world > 1:
        raise PlanError(f"WORLD_SIZE={world} without RANK: launch with torch.distributed.run")
    if gpus == 1:
        return "single", [0]
    nvis = visible()
    if gpus > nvis:
        raise PlanError(f"--gpus {gpus} but only {nvis} device(s) are visible")
    return "library", list(range(gpus))


def _visible_gpus():
    import torch
    return torch.cuda.device_count()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", default="vi", choices=["vi", "fitc", "laplace"],
                    help="vi = the headline metric; fitc / laplace = secondary modes (SURVEY 8(d))")
    ap.add_argument("--config", default=None, choices=["C2", "C3", "C5"])
    ap.add_argument("--tol-nr", type=float, default=1e-5)
    # --rows: the same, for torch.distributed.run command lines (it reads "--n" as an
    # abbreviation of its own options)
    ap.add_argument("--n", "--rows", dest="n", type=int, default=None)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--d", type=int, default=None,
                    help="C3's input dimension (default 8): times the d > 8 kernels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-full", default=None, metavar="OUT_JSON",
                    help="run only SURVEY 8(d)'s full CPU plan (several minutes, no GPU) and "
                         "write it to OUT_JSON")
    ap.add_argument("--knots", action="store_true",
                    help="also the m*d knot gradient (xu_opt = 'simultaneous', SURVEY 8(a) a16)")
    ap.add_argument("--devices", default=None, metavar="LIST",
                    help="one process over the row shards on these devices (comma list, repeats "
                         "allowed): the in-library multi-device context (sgp_ctx_create_multi, "
                         "RCCL inside libsgp) -- the path an R caller of the drop-in takes.  The "
                         "driver's multi-GPU runs keep one process per GPU (torchrun)")
    args = ap.parse_args()
    if args.cpu_full:
        res = cpu_baseline_full()
        with open(args.cpu_full, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res), flush=True)
        return
    if args.config is None:
        args.config = "C5" if args.mode == "laplace" else "C3"
    if (args.mode == "laplace") != (args.config == "C5"):
        ap.error("--mode laplace goes with --config C5 (Poisson data); vi/fitc with C2/C3")
    if args.d is not None and args.config != "C3":
        ap.error("--d applies to C3 only")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        devs = None if args.devices is None else [int(v) for v in args.devices.split(",") if v]
        kind, what = plan_run(args.gpus, devs, os.environ, _visible_gpus)
    except (PlanError, ValueError) as e:
        ap.error(str(e))
    if kind == "library":
        return bench_library_shards(args, what)

    import torch
    import torch.distributed as dist

    import sparsergps_amd as S
    from sparsergps_amd.dist import HipRowBackend, RowShardedLaplace, RowShardedVI, shard_rows

    # SGP_BENCH_REHEARSE=1: every rank on device 0 with gloo collectives -- exercises the N > 1
    # control flow (sharding, barriers, max-over-ranks timing) on a one-GPU box; never used for
    # a reported number (RCCL is the product path)
    rehearse = os.environ.get("SGP_BENCH_REHEARSE") == "1"
    dev_index = 0 if rehearse else local_rank
    # launched by torch.distributed.run (RANK in the environment): one process group over RCCL,
    # and the all-reduces run even at N = 1 (the N = 1 torchrun line rehearses the RCCL path)
    distributed = world > 1 or "RANK" in os.environ
    if distributed:
        torch.cuda.set_device(dev_index)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
    dev = torch.device("cuda", dev_index)

    P = make_problem(args.config, n=args.n, m=args.m, d=args.d)
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
        lap = RowShardedLaplace(backend, None, force_collectives=distributed)

        class _Runner:
            def eval(self, theta, U, delta):
                o, g, it = lap.eval(theta, U, delta, P["a"], args.tol_nr, 1000)
                nr_iters.append(it)
                return o, g
        runner = _Runner()
    elif not distributed and not args.knots:
        # one process, one GPU: the evaluation through the one-call entry the R path uses
        # (sgp_eval_vi / sgp_eval_fitc: the same phases and kernels, one ctypes call instead of
        # three plus the Python driver between them)
        fused = ctx.eval_vi if args.mode == "vi" else ctx.eval_fitc

        class _FusedRunner:
            def eval(self, theta, U, delta):
                return fused(theta, cov_fun, U, delta)
        runner = _FusedRunner()
    else:
        vi = RowShardedVI(backend, n, None, force_collectives=distributed)
        if args.knots:
            class _KnotRunner:
                def eval(self, theta, U, delta):
                    o, g = vi.eval(theta, U, delta)
                    # knot bounds of the whole data set (quirk Q9), combined over the ranks
                    return o, (g, backend.knot_gradient())
            runner = _KnotRunner()
        else:
            runner = vi
    del P["X"]

    # an optimizer-like trajectory: theta moves every step (no result can be reused)
    def theta_at(k):
        return theta0 * np.exp(1e-3 * np.sin(np.arange(theta0.size) + k))

    for k in range(args.warmup):
        runner.eval(theta_at(k), P["U"], P["delta"])

    # roofline of the dominant MFMA kernel, 2 n_loc m^2 flops per launch: VI's fused GEMM +
    # gradient contraction; FITC / Laplace's row-quadratic GEMM pass diag(K12 K22^-1 K21) (their
    # gradient passes read the products the row-quadratic passes stored, no GEMM of their own)
    con_key = {"vi": "contract_knm", "fitc": "rowquad_q", "laplace": "rowquad_q"}[args.mode]
    # Inside the timed region HIP events bracket only that kernel's phase, on its launch
    # stream (read back once, after the region); the per-phase breakdown comes from a short
    # untimed pass afterwards, so the other phases' event records stay out of the timed steps.
    ctx.timing_filter(con_key)
    ctx.enable_timing(True)
    # the steps' theta trajectory is synthetic input: built before the timed region like the
    # data (the optimizer's own host update between evaluations is not the hot path)
    thetas = [theta_at(args.warmup + k) for k in range(args.steps)]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    obj = None
    for th in thetas:
        obj, grad = runner.eval(th, P["U"], P["delta"])
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    t1 = time.perf_counter()
    evals = max(ctx.timing_evals(), 1)
    con_avg = {name: ms / evals for name, ms in ctx.timings()}
    ctx.timing_filter(None)
    ctx.enable_timing(True)
    for k in range(min(args.steps, 3)):
        runner.eval(theta_at(args.warmup + args.steps + k), P["U"], P["delta"])
    torch.cuda.synchronize(dev)
    pevals = max(ctx.timing_evals(), 1)
    phase_avg = {name: ms / pevals for name, ms in ctx.timings()}
    ctx.enable_timing(False)
    elapsed = t1 - t0
    if distributed:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    timed_iters = nr_iters[args.warmup:args.warmup + args.steps]

    t_con = con_avg.get(con_key, float("nan")) * 1e-3
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
        if args.mode == "vi" and (n, m, d) != (1_000_000, 1024, 8):
            metric["vi"] = f"sparse-GP objective+gradient evals/sec at n={n}, m={m}, d={d}"
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
                         "kernel": con_key + (" (k_contract<8>)" if d <= 8 else " (k_contract<32>)"),
                         "flops_per_launch": flops},
            "kernel_rooflines": kernel_rooflines(args.mode, phase_avg, n_loc, m,
                                                 store_ceiling(n_loc, m, dev_index)),
            "phases_ms": {k: round(v, 4) for k, v in phase_avg.items()},
            "phases_note": "HIP-event phase times from 3 evaluations after the timed steps "
                           "(inside the timed steps only the roofline kernel's phase is timed)",
            "objective": obj,
        }
        if args.mode == "laplace":
            out["nr_iters_per_eval"] = timed_iters
        if distributed:
            out["collectives"] = "rccl" if not rehearse else "gloo (rehearsal)"
        if (world == 1 and not args.no_cpu_baseline and args.mode == "vi"
                and args.config == "C3" and n == 1_000_000):
            full = None
            fp = os.path.join(ROOT, "profiles", "r3_cpu_baseline_full.json")
            if os.path.exists(fp):
                rec = json.load(open(fp))
                full = {"source": "profiles/r3_cpu_baseline_full.json (bench.py --cpu-full on a "
                                  "GPU box's host, committed; not re-measured by this run)",
                        "cpu": rec["cpu"],
                        "literal_quota_cores": {k: rec["literal_quota_cores"][k] for k in
                                                ("value", "sizes", "t_s", "fit", "threads")},
                        "literal_one_core": {k: rec["literal_one_core"][k] for k in
                                             ("value", "sizes", "t_s", "fit", "threads")},
                        "adjoint_direct": rec["adjoint_direct"]["value"]}
            out["cpu_baseline"] = cpu_baseline(full=full)
        print(json.dumps(out), flush=True)
    backend.close()
    if distributed:
        dist.destroy_process_group()


def bench_library_shards(args, devices):
    """`--gpus N` without torchrun (devices 0..N-1) or `--devices LIST`: the in-library
    multi-device context.  The rows are split into len(devices) shards, each evaluation's
    reductions summed on the devices and over them by RCCL inside libsgp (one host worker
    thread per distinct device).  With every shard on one GPU (e.g. --devices 0,0,0,0,0,0,0,0)
    this times C4's eight-way composition on a one-GPU box; on a node, --gpus 8 is the R
    drop-in's 8-GPU path.  The line carries the same roofline / kernel_rooflines fields as the
    one-GPU line, for shard 0's kernels."""
    import torch

    import sparsergps_amd as S
    from sparsergps_amd.dist import shard_rows
    P = make_problem(args.config, n=args.n, m=args.m, d=args.d)
    n, m, d = P["X"].shape[0], P["U"].shape[0], P["X"].shape[1]
    cov_fun = P["cov_fun"]
    names = S.param_names(cov_fun, d)
    theta0 = np.array([P["cov_par"][k] for k in names])
    ctx = S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m, devices=devices)
    nshards, ndev = ctx.shards()
    U = np.asfortranarray(P["U"])
    if args.mode == "laplace":
        ctx.lap_set_f(P["f0"])
    del P["X"]
    nr_iters = []

    def run(k, th=None):
        if th is None:
            th = theta0 * np.exp(1e-3 * np.sin(np.arange(theta0.size) + k))
        if args.mode == "vi":
            return ctx.eval_vi(th, cov_fun, U, P["delta"])
        if args.mode == "fitc":
            return ctx.eval_fitc(th, cov_fun, U, P["delta"])
        o, g, it = ctx.eval_laplace(th, cov_fun, U, P["delta"], P["a"], args.tol_nr, 1000)
        nr_iters.append(it)
        return o, g

    for k in range(args.warmup):
        run(k)
    con_key = {"vi": "contract_knm", "fitc": "rowquad_q", "laplace": "rowquad_q"}[args.mode]
    ctx.timing_filter(con_key)     # shard 0's launch stream (the timing calls follow shard 0)
    ctx.enable_timing(True)
    # the theta trajectory built before the timed region, as on the one-GPU line
    thetas = [theta0 * np.exp(1e-3 * np.sin(np.arange(theta0.size) + args.warmup + k))
              for k in range(args.steps)]
    for dv in sorted(set(devices)):
        torch.cuda.synchronize(dv)
    t0 = time.perf_counter()
    obj = None
    for k in range(args.steps):
        obj, _ = run(args.warmup + k, thetas[k])
    for dv in sorted(set(devices)):
        torch.cuda.synchronize(dv)
    elapsed = time.perf_counter() - t0
    evals = max(ctx.timing_evals(), 1)
    t_con = dict(ctx.timings()).get(con_key, float("nan")) / evals * 1e-3
    # per-phase times of shard 0 from a short untimed pass (as the one-GPU line)
    ctx.timing_filter(None)
    ctx.enable_timing(True)
    for k in range(min(args.steps, 3)):
        run(args.warmup + args.steps + k)
    for dv in sorted(set(devices)):
        torch.cuda.synchronize(dv)
    pevals = max(ctx.timing_evals(), 1)
    phase_avg = {name: ms / pevals for name, ms in ctx.timings()}
    ctx.enable_timing(False)
    n0 = shard_rows(n, nshards, 0)[1]
    flops = 2.0 * n0 * m * m
    achieved = flops / t_con / 1e12 if t_con > 0 else float("nan")
    traffic = None
    tp = os.path.join(ROOT, "profiles", "pmc_traffic_contract_knm.json")
    if args.mode == "vi" and os.path.exists(tp):
        try:
            rec = json.load(open(tp))
            if rec.get("n") == n0 and rec.get("m") == m:
                traffic = rec.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    metric = {"vi": "sparse-GP objective+gradient evals/sec at n=1e6, m=1024, d=8",
              "fitc": "FITC objective+gradient evals/sec (secondary mode)",
              "laplace": "Poisson sparse-Laplace NR+objective+gradient evals/sec (C5, secondary)"}
    if args.mode == "vi" and (n, m, d) != (1_000_000, 1024, 8):
        metric["vi"] = f"sparse-GP objective+gradient evals/sec at n={n}, m={m}, d={d}"
    out = {"metric": metric[args.mode], "value": args.steps / elapsed, "unit": "evals/s",
           "n_gpus": ndev, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "f64",
           "data": f"synthetic (SURVEY.md 8(d) {args.config} generator, numpy PCG64)",
           "config": {"workload": f"{args.config} {args.mode}, n={n}, m={m}, d={d}, {cov_fun}, "
                                  f"P={len(names)}, knots fixed",
                      "n": n, "m": m, "d": d, "kernel": cov_fun,
                      "parallelism": f"library-rows{nshards}",
                      "devices": devices},
           "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": achieved / FP64_MFMA_PEAK_TFLOPS,
                        "traffic": traffic,
                        "kernel": con_key + " of shard 0"
                                  + (" (k_contract<8>)" if d <= 8 else " (k_contract<32>)"),
                        "flops_per_launch": flops},
           "kernel_rooflines": kernel_rooflines(args.mode, phase_avg, n0, m,
                                                store_ceiling(n0, m, devices[0])),
           "phases_ms": {k: round(v, 4) for k, v in phase_avg.items()},
           "phases_note": "shard 0's HIP-event phase times from 3 evaluations after the timed "
                          "steps",
           "objective": obj,
           "collectives": "rccl (in-library, ncclCommInitAll over the distinct devices)",
           "note": "in-library multi-device context (sgp_ctx_create_multi): one process, one "
                   "host worker per distinct device; shards on one device run one after another "
                   "on it"}
    if args.mode == "laplace":
        out["nr_iters_per_eval"] = nr_iters[args.warmup:args.warmup + args.steps]
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
