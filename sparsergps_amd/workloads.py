"""Synthetic workloads of SURVEY.md 8(d) (numpy PCG64 streams): C2, C3 (C4 = C3 row-sharded)
and C5.  Data generation only -- used by bench.py, the tests and tools; no reference files are
read and nothing here computes a GP quantity.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def make_gaussian_problem(config, n=None, m=None, d=None):
    """C2 / C3 (and C4 = C3 row-sharded) synthetic Gaussian regression inputs.

    C2: d=3, sqexp, theta=(sigma=1, l=1, tau=0.5); seeds X=2, U=3, y=4.
    C3: d=8, ARD,   theta=(sigma=1, l1..l8=3, tau=0.5); seeds X=5, U=6, y=7.
    `d` overrides C3's input dimension (timing of the d > 8 kernels only; not a BASELINE config).
    y = sum_c sin(x_c) [/sqrt(d) for C3] + N(0, 0.5^2); mu = mean(y) (quirk Q14).
    """
    if config == "C2":
        n = n or 100_000
        m = m or 256
        d, sx, su, sy = 3, 2, 3, 4
        X = _rng(sx).uniform(0.0, 10.0, size=(n, d))
        U = _rng(su).uniform(0.0, 10.0, size=(m, d))
        y = np.sin(X).sum(axis=1) + _rng(sy).normal(0.0, 0.5, size=n)
        cov_par = OrderedDict([("sigma", 1.0), ("l", 1.0), ("tau", 0.5)])
        cov_fun = "sqexp"
    elif config in ("C3", "C4"):
        n = n or 1_000_000
        m = m or 1024
        d, sx, su, sy = d or 8, 5, 6, 7
        X = _rng(sx).uniform(0.0, 10.0, size=(n, d))
        U = _rng(su).uniform(0.0, 10.0, size=(m, d))
        y = np.sin(X).sum(axis=1) / math.sqrt(d) + _rng(sy).normal(0.0, 0.5, size=n)
        cov_par = OrderedDict([("sigma", 1.0)] + [(f"l{c + 1}", 3.0) for c in range(d)] + [("tau", 0.5)])
        cov_fun = "ard"
    else:
        raise ValueError(config)
    mu = np.full(n, y.mean())
    return dict(X=X, U=U, y=y, mu=mu, cov_par=cov_par, cov_fun=cov_fun, delta=1e-6)


def make_poisson_problem(n=None, m=None, per_row_exposure=False):
    """C5: Poisson Laplace, n=5e5, m=512, d=5, sqexp, theta=(1, 2, 0.1); seeds X=8, U=9, y=10.

    per_row_exposure: a_i ~ U(0.5, 2) (seed 11) -- the reference's `m` as "a vector of the areas
    of each grid cell" (R/derivative_functions_of_data_likelihoods.R:38) -- instead of a = 1;
    y ~ Poisson(a_i e^f_i) and f0 = log(mean y) - log(a) per row (R/optimize_gp.R:480)."""
    n = n or 500_000
    m = m or 512
    d = 5
    X = _rng(8).uniform(0.0, 10.0, size=(n, d))
    U = _rng(9).uniform(0.0, 10.0, size=(m, d))
    f = 0.5 * np.sin(X).sum(axis=1) / math.sqrt(d) + math.log(2.0)
    a = _rng(11).uniform(0.5, 2.0, size=n) if per_row_exposure else 1.0
    y = _rng(10).poisson(a * np.exp(f)).astype(np.float64)
    mu = np.full(n, math.log(y.mean()))
    f0 = math.log(y.mean()) - np.log(a) * np.ones(n)
    cov_par = OrderedDict([("sigma", 1.0), ("l", 2.0), ("tau", 0.1)])
    return dict(X=X, U=U, y=y, mu=mu, f0=f0, a=a, cov_par=cov_par, cov_fun="sqexp", delta=1e-6)
