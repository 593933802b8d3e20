"""Determinism probe: repeated evaluations on one context must be bit-identical (one-device and
sharded contexts; VI / FITC evaluations and candidate scorers)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import sparsergps_amd as S
    from sparsergps_amd.workloads import make_gaussian_problem
    P = make_gaussian_problem("C2", n=12_000, m=64)
    th = np.array(list(P["cov_par"].values()))
    cand = np.random.default_rng(3).uniform(0, 10, size=(5, 3))
    for dv in (None, [0], [0] * 4):
        with S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=65, devices=dv) as c:
            out = {}
            for rep in range(3):
                r = {"vi": c.eval_vi(th, "sqexp", P["U"], P["delta"]),
                     "fitc": c.eval_fitc(th, "sqexp", P["U"], P["delta"]),
                     "fitc_oo": c.eval_fitc(th, "sqexp", P["U"], P["delta"], obj_only=True)[0],
                     "vic": c.vi_candidates(th, "sqexp", P["U"], cand, P["delta"]),
                     "fc": c.fitc_candidates(th, "sqexp", P["U"], cand, P["delta"])}
                for k, v in r.items():
                    flat = np.concatenate([np.atleast_1d(np.asarray(x, dtype=float)).ravel()
                                           for x in (v if isinstance(v, tuple) else (v,))])
                    if k in out and not np.array_equal(out[k], flat):
                        print(f"devices={dv} {k}: rep {rep} differs, max rel "
                              f"{np.max(np.abs(flat / out[k] - 1)):.3e}")
                    out.setdefault(k, flat)
            print(f"devices={dv}: done")


if __name__ == "__main__":
    main()
