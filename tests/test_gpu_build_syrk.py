"""K12 built inside VI's SYRK at m_p = 256 (k_build_syrk_s256) on the GPU.

At C2's knot count the builder (HBM-write bound) and the SYRK (MFMA bound) ran one after the
other; the fused kernel evaluates each 16-row slab of K12 = sig2 exp(-|x~ - u~|^2) on the VALU
into the SYRK's idle LDS buffer, stores it for the later passes and folds t = K^T r into a
per-column register.  Against the two-kernel path (SGP_BS256=0, run in a child process) the
objective, gradient and knot gradient agree to 1e-12 relative (K differs only in the exp's last
bits: direct differences against the builder's GEMM-form exponent) and the fused path is
bit-identical on repeat.  Shapes: configs[1] (C2) exactly; padding rows (n not a multiple of
16) and padding knots (m = 200); ARD at d = 4 and d = 6 (the 4- and 8-coordinate
instantiations); knots copied from data rows (the tau coincidence rule reads X and U, not K);
n small enough that every row chunk is one k-step.  The oracle checks of the fused path are the
C2 fixture (m = 256) and C2 at full n in test_gpu_configs.py, which now run through it.
Reference: R/vi_functions.R:87-103 (Sigma12, Sigma22 and t(Sigma12) %*% Sigma12 of elbo_fun).
"""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import json, sys
    import numpy as np
    sys.path.insert(0, {root!r})
    import sparsergps_amd as S
    from sparsergps_amd.workloads import make_gaussian_problem
    cfg, n, m, d, knots, coinc = {cfg!r}, {n}, {m}, {d}, {knots}, {coinc}
    P = make_gaussian_problem(cfg, n=n, m=m, d=d) if d else make_gaussian_problem(cfg, n=n, m=m)
    U = P["U"].copy()
    if coinc:
        U[::7] = P["X"][:len(U[::7])]
    th = np.array(list(P["cov_par"].values()))
    out = []
    with S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m) as ctx:
        if knots:
            ctx.enable_knot_grad(True)
        for rep in range(2):
            o, g = ctx.eval_vi(th, P["cov_fun"], U, P["delta"])
            kg = ctx.knot_gradient(None).tolist() if knots else []
            out.append([float(o)] + [float(v) for v in g] + kg)
    print("RESULT", json.dumps(out))
""")


def _run(cfg, n, m, d, knots, coinc, fused):
    env = dict(os.environ)
    env.pop("SGP_BS256", None)
    if not fused:
        env["SGP_BS256"] = "0"
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, cfg=cfg, n=n, m=m, d=d,
                                                          knots=knots, coinc=coinc)],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=250)
    out = r.stdout.decode(errors="replace")
    assert r.returncode == 0, out[-3000:]
    line = [l for l in out.splitlines() if l.startswith("RESULT ")][-1]
    return np.array(json.loads(line[7:]))


@pytest.mark.parametrize("cfg,n,m,d,knots,coinc", [
    ("C2", 100_000, 256, None, False, False),   # configs[1]
    ("C2", 12_345, 200, None, True, False),     # padding rows and knots, knot gradients
    ("C2", 20_000, 256, None, False, True),     # knots equal to data rows
    ("C3", 30_001, 256, 4, False, False),       # ARD, 4-coordinate instantiation
    ("C3", 30_000, 240, 6, True, False),        # ARD, 8-coordinate instantiation
    ("C2", 1_000, 256, None, False, False),     # one k-step per row chunk
])
def test_fused_build_syrk_matches_two_kernels(cfg, n, m, d, knots, coinc):
    from sparsergps_amd import _lib
    _lib.require_gpu()
    fused = _run(cfg, n, m, d, knots, coinc, fused=True)
    two = _run(cfg, n, m, d, knots, coinc, fused=False)
    assert np.array_equal(fused[0], fused[1]), "fused build + SYRK not bit-identical on repeat"
    assert np.array_equal(two[0], two[1])
    rel = np.abs(fused[0] - two[0]) / np.maximum(1.0, np.abs(two[0]))
    print(f"\n[bs256] {cfg} n={n} m={m} d={d} knots={knots} coinc={coinc}: max rel diff "
          f"{rel.max():.3e}")
    assert rel.max() < 1e-12
