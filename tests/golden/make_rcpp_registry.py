"""Generate tests/golden/rcpp_registry.json from the reference (run where /root/reference is
present): the .Call registry of src/RcppExports.cpp (routine name, arity, in order) and the
formals of the R hot-path functions and drivers the R shim replaces.  Interface data only (names,
arities, argument lists); tests/test_rshim.py checks rshim/ against it."""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rcpp_registry.json")

FUNCS = {
    "elbo_fun": "R/vi_functions.R",
    "delbo_dcov_par": "R/vi_functions.R",
    "obj_fun_norm": "R/laplace_approx_obj_funs.R",
    "dlogp_dcov_par": "R/laplace_approx_gradient.R",
    "newtrap_sparseGP": "R/newtrap_sparseGP.R",
    "dlogq_dcov_par": "R/laplace_approx_gradient.R",
    "norm_grad_ascent_vi": "R/vi_functions.R",
    "norm_grad_ascent": "R/laplace_gradient_ascent.R",
    "laplace_grad_ascent": "R/laplace_gradient_ascent.R",
    "predict_gp": "R/laplace_approx_prediction.R",
}


def call_entries(text):
    block = text[text.index("CallEntries[]"):]
    block = block[:block.index("{NULL, NULL, 0}")]
    return [[n, int(a)] for n, a in
            re.findall(r'\{"(\w+)",\s*\(DL_FUNC\)\s*&\w+,\s*(\d+)\}', block)]


def formals(text, name):
    m = re.search(r"^%s\s*<-\s*function\s*\(" % re.escape(name), text, re.M)
    i, depth = m.end(), 1
    j = i
    while depth:
        depth += {"(": 1, ")": -1}.get(text[j], 0)
        j += 1
    return normalise(text[i:j - 1])


def normalise(args):
    args = re.sub(r"#[^\n]*", "", args)
    return [re.sub(r"\s+", "", a) for a in args.split(",")]


def main():
    reg = call_entries(open(os.path.join(REF, "src/RcppExports.cpp")).read())
    fm = {f: formals(open(os.path.join(REF, p)).read(), f) for f, p in FUNCS.items()}
    json.dump({"source": "src/RcppExports.cpp CallEntries; R formals from " +
               ", ".join(sorted(set(FUNCS.values()))),
               "call_entries": reg, "formals": fm}, open(OUT, "w"), indent=1)
    print(f"{len(reg)} routines, {len(fm)} R functions -> {OUT}")


if __name__ == "__main__":
    main()
