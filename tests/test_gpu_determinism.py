"""Run-to-run determinism of every evaluation path: repeated evaluations at the same inputs are
bit-identical (the slab + fixed-order reductions; no atomics in any sum).

Round 5 found the weighted SYRKs (FITC's S_D / S_omega, Laplace's S_B / S_a) differing in the
last bit between runs: inside a diagonal 16 x 16 fragment both elements of a symmetric pair are
computed, and with a weight on one operand they differ by rounding ((w_k K_ka) K_kb against
(w_k K_kb) K_ka); two threads then wrote the pair's two addresses in either order.  Only the lower
element writes now.  Shapes cover the packed plan (m <= 128), the fragment-balanced m_p = 256 SYRK,
and the balanced plans (m_p = 384, 640); contexts one-device and sharded.
Reference: the deterministic sums of R's own matrix products (R/vi_functions.R:87-118,
R/laplace_approx_obj_funs.R:6-52, R/newtrap_sparseGP.R:6-186).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sgp():
    import sparsergps_amd as S
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return S


def _same(a, b):
    fa = np.concatenate([np.atleast_1d(np.asarray(x, dtype=float)).ravel() for x in a])
    fb = np.concatenate([np.atleast_1d(np.asarray(x, dtype=float)).ravel() for x in b])
    return np.array_equal(fa, fb)


@pytest.mark.parametrize("m", [64, 200, 256, 384, 640])
@pytest.mark.parametrize("devices", [None, [0, 0, 0]], ids=["one", "shards3"])
def test_gaussian_paths_bit_identical(sgp, m, devices):
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C3", n=9_001, m=m, d=4)
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m, devices=devices) as c:
        runs = [(c.eval_vi(th, "ard", P["U"], P["delta"]),
                 c.eval_fitc(th, "ard", P["U"], P["delta"])) for _ in range(3)]
    for r in runs[1:]:
        assert _same(r[0], runs[0][0]), "VI"
        assert _same(r[1], runs[0][1]), "FITC"


@pytest.mark.parametrize("m", [100, 256, 384])
@pytest.mark.parametrize("devices", [None, [0, 0]], ids=["one", "shards2"])
def test_laplace_bit_identical(sgp, m, devices):
    from sparsergps_amd.workloads import make_poisson_problem
    P = make_poisson_problem(n=8_001, m=m)
    th = np.array(list(P["cov_par"].values()))
    with sgp.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m, devices=devices) as c:
        runs = []
        for _ in range(3):
            c.lap_set_f(P["f0"])
            o, g, it = c.eval_laplace(th, "sqexp", P["U"], P["delta"], P["a"], 1e-5, 1000)
            runs.append((o, g, it, c.lap_get_f()))
    for r in runs[1:]:
        assert r[2] == runs[0][2]
        assert _same(r[:2] + (r[3],), runs[0][:2] + (runs[0][3],))
