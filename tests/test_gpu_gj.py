"""The m x m SPD inverses' Gauss-Jordan chains on the GPU (k_dense.hip), pinned once.

R's chol / solve of Sigma22 and of Sigma22 + t(Sigma12) %*% ZSig12 (R/vi_functions.R:87-103,
231-239) are, in this library, two blocked Gauss-Jordan chains that phase 2 of every VI
evaluation runs side by side (K22's on the `aux` stream, Bm's on the launch stream).  Since round
5 each is ONE persistent launch whose workgroups hand tiles over through write-through stores
and per-tile flags with relaxed agent-scope atomics (k_dense.hip:472-519); before, one launch per
pivot step.  The kernel states that the two give bit-identical results (per-tile arithmetic is
k_gj_step's).  Here, through sgp_diag_gj_pair (include/sgp_diag.h), on the same SPD inputs:
* both chains in flight together (as in phase 2), at nb = 4, 16 and 64 pivot blocks
  (m = 256, 1024, 4096): the persistent and the launch-per-step results are bit-identical, the
  persistent chain is bit-identical on repeat, and both match numpy's inverse;
* the watchdog: a probe build (SGP_PROBE_BUILD, tools/ab/gj_withhold) withholds one flag publish
  once (SGP_PROBE_GJ_WITHHOLD=<ticket>); the evaluation must return SGP_EHIP naming the
  watchdog, the grid must drain (the process goes on), and the next evaluation on the same
  context must be right.
"""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    from sparsergps_amd import _lib
    _lib.require_gpu()
    return _lib.lib()


def _spd_pair(m, seed):
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((m, m))
    A = G @ G.T / m + 0.5 * np.eye(m)           # K22-like: SPD, moderate conditioning
    H = rng.standard_normal((m, 3 * m // 2))
    B = H @ H.T / m                               # S-like: PSD
    return np.asfortranarray(A), np.asfortranarray(B)


def _pair(L, A, B, beta, per_step):
    from sparsergps_amd import _lib
    m = A.shape[0]
    ia = np.zeros((m, m), order="F")
    isum = np.zeros((m, m), order="F")
    ld = np.zeros(2)
    _lib.check(L.sgp_diag_gj_pair(0, m, _lib.dptr(A), _lib.dptr(B), beta, per_step,
                                  _lib.dptr(ia), _lib.dptr(isum), _lib.dptr(ld)))
    return ia, isum, ld


@pytest.mark.parametrize("m", [256, 1024, 4096])
def test_persistent_chain_is_bit_identical_to_per_step(L, m):
    A, B = _spd_pair(m, seed=m)
    beta = 4.0
    p = _pair(L, A, B, beta, 0)
    s = _pair(L, A, B, beta, 1)
    for a, b, what in zip(p, s, ("inv(A)", "inv(A + beta B)", "log dets")):
        assert np.array_equal(a, b), f"{what}: persistent != per-step at m = {m} " \
                                     f"(max diff {np.max(np.abs(a - b)):.3e})"
    # the hand-offs under repetition: every run of the two concurrent persistent chains gives
    # the same bits (a visibility race would show as a changed tile or a failed pivot)
    for rep in range(8 if m < 4096 else 3):
        again = _pair(L, A, B, beta, 0)
        for a, c, what in zip(p, again, ("inv(A)", "inv(A + beta B)", "log dets")):
            assert np.array_equal(a, c), f"{what}: persistent chain run {rep + 2} differs at m = {m}"
    S = A + beta * B
    eye = np.eye(m)
    assert np.max(np.abs(p[0] @ A - eye)) < 1e-9
    assert np.max(np.abs(p[1] @ S - eye)) < 1e-9
    assert abs(p[2][0] - np.linalg.slogdet(A)[1]) < 1e-9 * m
    assert abs(p[2][1] - np.linalg.slogdet(S)[1]) < 1e-9 * m


def test_diag_refuses_bad_arguments(L):
    from sparsergps_amd import _lib
    A = np.eye(4, order="F")
    out = np.zeros((4, 4), order="F")
    ld = np.zeros(2)
    assert L.sgp_diag_gj_pair(0, 0, _lib.dptr(A), _lib.dptr(A), 1.0, 0, _lib.dptr(out),
                              _lib.dptr(out), _lib.dptr(ld)) == _lib.SGP_EINVAL
    assert L.sgp_diag_gj_pair(0, 5000, _lib.dptr(A), _lib.dptr(A), 1.0, 0, _lib.dptr(out),
                              _lib.dptr(out), _lib.dptr(ld)) == _lib.SGP_EINVAL   # persistent: m <= 4096
    bad = -np.eye(4, order="F")
    assert L.sgp_diag_gj_pair(0, 4, _lib.dptr(bad), _lib.dptr(A), 0.0, 0, _lib.dptr(out),
                              _lib.dptr(out), _lib.dptr(ld)) == _lib.SGP_ENOTPD


CHILD = textwrap.dedent("""
    import sys, time
    import numpy as np
    sys.path.insert(0, {root!r})
    import sparsergps_amd as S
    from sparsergps_amd import _lib
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C2", n=4000, m=256)
    th = np.array(list(P["cov_par"].values()))
    with S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=256) as ctx:
        t0 = time.time()
        try:
            ctx.eval_vi(th, "sqexp", P["U"], P["delta"])
            print("NO_ERROR")
        except _lib.SGPError as e:
            print("ERR", e.status, str(e).replace(chr(10), " "))
        print("SECONDS", time.time() - t0)
        o, g = ctx.eval_vi(th, "sqexp", P["U"], P["delta"])
        print("OBJ", repr(float(o)))
        print("GRAD", " ".join(repr(float(v)) for v in g))
""")


def test_watchdog_fault_injection(L):
    """A withheld flag publish: the evaluation fails with the watchdog's error, the grid drains
    (no hang: the child process ends), and the next evaluation on the same context equals the
    product library's."""
    from sparsergps_amd import _build, _lib
    import sparsergps_amd as S
    from sparsergps_amd.workloads import make_gaussian_problem
    lib_path = _build.build_variant("gj_withhold")   # no -D knob: the probe build's env hook
    env = dict(os.environ, SGP_AB_LIB=lib_path, SGP_PROBE_GJ_WITHHOLD="0")
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=100)
    out = r.stdout.decode(errors="replace")
    print(out)
    assert r.returncode == 0, out[-3000:]
    lines = dict(l.split(" ", 1) for l in out.splitlines() if " " in l)
    assert "ERR" in lines, out
    assert lines["ERR"].startswith(str(_lib.SGP_EHIP)) and "watchdog" in lines["ERR"], out
    P = make_gaussian_problem("C2", n=4000, m=256)
    th = np.array(list(P["cov_par"].values()))
    with S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=256) as ctx:
        o, g = ctx.eval_vi(th, "sqexp", P["U"], P["delta"])
    assert float(lines["OBJ"]) == o
    np.testing.assert_array_equal(np.array([float(v) for v in lines["GRAD"].split()]), g)
