"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no tests or recorded outputs and cannot be run here
(no R/Rcpp), so these vectors come from oracle/sgp_oracle.py -- the literal restatement of
the reference formulas -- after it has been pinned independently by tests/test_oracle.py
(finite differences, dense n x n formulation, closed forms).  Inputs and outputs only.

    python tests/golden/make_golden.py        # all fixtures
    python tests/golden/make_golden.py own    # only the C2 (m=256) / C5 (m=512) fixtures
    python tests/golden/make_golden.py expo   # only the per-row exposure Poisson fixture
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import sgp_oracle as O  # noqa: E402


def save(name, **arrs):
    np.savez(os.path.join(HERE, name), **arrs)
    print("wrote", name)


def gauss_case(name, cfg, n, m, coincide=False):
    P = O.make_gaussian_problem(cfg, n=n, m=m)
    U = P["U"].copy()
    if coincide:
        U[:3] = P["X"][:3]
    cp = P["cov_par"]
    names = np.array(list(cp.keys()))
    theta = np.array(list(cp.values()))
    vi_obj = O.elbo_eval(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])
    vi_grad = O.delbo_dcov_par(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    fitc_obj = O.fitc_obj_eval(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])
    fitc_grad = O.dlogp_dcov_par(cp, P["cov_fun"], U, P["X"], P["y"], P["mu"], P["delta"])["gradient"]
    save(name, X=P["X"], U=U, y=P["y"], mu=P["mu"], names=names, theta=theta,
         cov_fun=np.array(P["cov_fun"]), delta=np.array(P["delta"]),
         vi_obj=np.array(vi_obj), vi_grad=np.array([vi_grad[k] for k in cp]),
         fitc_obj=np.array(fitc_obj), fitc_grad=np.array([fitc_grad[k] for k in cp]))


def poisson_case(name, n, m, per_row_exposure=False):
    P = O.make_poisson_problem(n=n, m=m, per_row_exposure=per_row_exposure)
    cp = P["cov_par"]
    nr = O.newtrap_sparseGP(P["f0"], cp, "sqexp", P["X"], P["U"], P["y"], P["mu"], P["a"],
                            tol=1e-5)
    g = O.dlogq_dcov_par(cp, "sqexp", P["U"], P["X"], P["y"], nr["gp"], P["mu"], P["a"])["gradient"]
    save(name, X=P["X"], U=P["U"], y=P["y"], mu=P["mu"], f0=P["f0"], a=np.array(P["a"]),
         names=np.array(list(cp.keys())), theta=np.array(list(cp.values())),
         delta=np.array(P["delta"]), ff=nr["gp"], obj_trace=nr["objective_function_values"],
         grad=np.array([g[k] for k in cp]))


def fill_case(name):
    rng = np.random.default_rng(20)
    x = rng.uniform(0, 10, size=(9, 3))
    xp = np.vstack([x[:2], rng.uniform(0, 10, size=(5, 3))])
    cp = {"sigma": 1.3, "l": 1.7, "tau": 0.4}
    ln = ["l1", "l2", "l3"]
    cpa = {"sigma": 0.9, "l1": 0.8, "l2": 1.5, "l3": 2.2, "tau": 0.3}
    out = dict(x=x, xp=xp)
    for f in ("sqexp", "exp"):
        out[f"cov_{f}_sym"] = O.make_cov_matC(x, None, cp, f, 1e-6)
        out[f"cov_{f}_cross"] = O.make_cov_matC(x, xp, cp, f, 1e-6)
        for p in ("sigma", "l", "tau"):
            out[f"d_{f}_{p}_sym"] = O.dsig_dthetaC(x, None, cp, f, p)
            out[f"d_{f}_{p}_cross"] = O.dsig_dthetaC(x, xp, cp, f, p)
    out["cov_ard_sym"] = O.make_cov_mat_ardC(x, None, cpa, "ard", 1e-6, ln)
    out["cov_ard_cross"] = O.make_cov_mat_ardC(x, xp, cpa, "ard", 1e-6, ln)
    for p in ("sigma", "l1", "l2", "l3", "tau"):
        out[f"d_ard_{p}_sym"] = O.dsig_dtheta_ardC(x, None, cpa, "ard", p, ln)
        out[f"d_ard_{p}_cross"] = O.dsig_dtheta_ardC(x, xp, cpa, "ard", p, ln)
    save(name, **out)


def own_knot_counts():
    """C2 and C5 at their own knot counts (BASELINE.json configs[1], configs[4]), reduced n."""
    gauss_case("gauss_c2_m256.npz", "C2", 2000, 256)
    poisson_case("poisson_c5_m512.npz", 2000, 512)


def per_row_exposure():
    """Poisson with the exposure `m` as one value per row (a vector of cell areas,
    R/derivative_functions_of_data_likelihoods.R:38; optimize_gp.R:461-468 passes it through)."""
    poisson_case("poisson_c5_expo.npz", 400, 24, per_row_exposure=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["own"]:
        own_knot_counts()
        sys.exit(0)
    if sys.argv[1:] == ["expo"]:
        per_row_exposure()
        sys.exit(0)
    per_row_exposure()
    own_knot_counts()
    fill_case("fills.npz")
    gauss_case("gauss_c2_small.npz", "C2", 200, 16)
    gauss_case("gauss_c3_small.npz", "C3", 150, 12)
    gauss_case("gauss_c2_coincident.npz", "C2", 120, 10, coincide=True)
    poisson_case("poisson_c5_small.npz", 150, 10)
