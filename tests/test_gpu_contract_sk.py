"""The balanced (Stream-K) launch of VI's gradient contraction (k_contract_sk) on the GPU.

When the one-tile-per-workgroup grid would leave its last residency round mostly empty (C2:
1564 tiles over 512 slots = 3.05 rounds run as 4; the 8-GPU shard: 15.3 as 16), the tiles'
k-steps are split evenly over the resident workgroups and a tile cut between two workgroups is
finished by the one holding its k = 0 step (the partial product and partial K u handed over
through write-through stores and a per-slot flag).  Only the summation order of the split tiles
changes, so against the one-tile grid (the default, run in a child process) the objective,
gradient and knot gradient agree to 1e-12 relative, and the balanced launch is bit-identical on
repeat.  The launch is opt-in (SGP_CON_SK=1): it measured no faster than the grid at C2 and
slower on the shard, so the product default is the grid.  Shapes: configs[1] (C2) exactly, C4's shard (n = 125 000, m = 1024, ARD), a grid just
past one round (514 tiles: ranges barely longer than a tile), and the knot-gradient epilogue.
Reference: the contraction replaces R/vi_functions.R:259-419 (delbo_dcov_par's per-parameter
products); the oracle checks of the same shapes are in test_gpu_configs.py / test_gpu_multi.py.
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
    cfg, n, m, knots = {cfg!r}, {n}, {m}, {knots}
    P = make_gaussian_problem(cfg, n=n, m=m)
    th = np.array(list(P["cov_par"].values()))
    out = []
    with S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=m) as ctx:
        if knots:
            ctx.enable_knot_grad(True)
        for rep in range(2):
            o, g = ctx.eval_vi(th, P["cov_fun"], P["U"], P["delta"])
            kg = ctx.knot_gradient(None).tolist() if knots else []
            out.append([float(o)] + [float(v) for v in g] + kg)
    print("RESULT", json.dumps(out))
""")


def _run(cfg, n, m, knots, sk_off, dp=None):
    env = dict(os.environ)
    env.pop("SGP_CON_SK_DP", None)
    if sk_off:
        env.pop("SGP_CON_SK", None)
    else:
        env["SGP_CON_SK"] = "1"
        if dp is not None:
            env["SGP_CON_SK_DP"] = str(dp)
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, cfg=cfg, n=n, m=m,
                                                          knots=knots)],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=250)
    out = r.stdout.decode(errors="replace")
    assert r.returncode == 0, out[-3000:]
    line = [l for l in out.splitlines() if l.startswith("RESULT ")][-1]
    return np.array(json.loads(line[7:]))


@pytest.mark.parametrize("cfg,n,m,knots,dp", [
    ("C2", 100_000, 256, False, None),      # configs[1]: 1564 tiles, 3.05 rounds
    ("C3", 125_000, 1024, False, None),     # C4's shard: 7816 tiles, 15.3 rounds
    ("C2", 32_800, 256, False, None),       # 514 tiles: each range a tile and ~1 step
    ("C2", 60_000, 256, True, None),        # the knot-gradient epilogue
    ("C2", 100_000, 256, False, 0),         # every tile's k-steps balanced (SGP_CON_SK_DP=0)
    ("C2", 60_000, 256, True, 0),
    ("C3", 125_000, 1024, False, 0),
])
def test_balanced_contraction_matches_tile_grid(cfg, n, m, knots, dp):
    from sparsergps_amd import _lib
    _lib.require_gpu()
    sk = _run(cfg, n, m, knots, sk_off=False, dp=dp)
    grid = _run(cfg, n, m, knots, sk_off=True)
    assert np.array_equal(sk[0], sk[1]), "balanced launch not bit-identical on repeat"
    assert np.array_equal(grid[0], grid[1])
    rel = np.abs(sk[0] - grid[0]) / np.maximum(1.0, np.abs(grid[0]))
    print(f"\n[sk] {cfg} n={n} m={m} knots={knots} dp={dp}: max rel diff {rel.max():.3e}")
    assert rel.max() < 1e-12
