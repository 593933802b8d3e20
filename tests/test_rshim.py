"""The R side of the drop-in boundary (rshim/), checked without R (absent from this image):

* the .Call registry of rshim/sparseRGPs_sgp.c starts with exactly the reference's 20 routines
  (names, arities, order of src/RcppExports.cpp:284-306; fixture tests/golden/rcpp_registry.json,
  itself compared with the reference when /root/reference is present), and every registered C
  function takes that many SEXP arguments;
* every .Call in rshim/R/sgp_hotpath.R names a registered routine with the right arity;
* the six R replacements keep the reference's formals exactly;
* every sgp_* entry point the shim calls is declared in include/sgp.h and exported by libsgp.so;
* the shim compiles (gcc -fsyntax-only -Wall -Wextra -Werror) against the R API prototypes it
  uses (tests/r_api/, declarations only).
"""
import json
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "rshim", "sparseRGPs_sgp.c")
RFILE = os.path.join(ROOT, "rshim", "R", "sgp_hotpath.R")
FIX = os.path.join(ROOT, "tests", "golden", "rcpp_registry.json")
REF = "/root/reference"


def _entries(text):
    block = text[text.index("CallEntries[]"):]
    block = block[:block.index("{NULL, NULL, 0}")]
    return [(n, f, int(a)) for n, f, a in
            re.findall(r'\{"(\w+)",\s*\(DL_FUNC\)\s*&(\w+),\s*(\d+)\}', block)]


def _c_arity(text, fn):
    m = re.search(r"^SEXP %s\(([^)]*)\)" % fn, text, re.M)
    assert m, fn
    args = m.group(1).strip()
    return 0 if args in ("", "void") else len(args.split(","))


def test_registry_matches_reference_exports():
    fix = json.load(open(FIX))
    text = open(SHIM).read()
    ent = _entries(text)
    ref = [tuple(e) for e in fix["call_entries"]]
    assert len(ref) == 20
    assert [(n, a) for n, _, a in ent[:20]] == ref
    for name, fn, arity in ent:
        assert _c_arity(text, fn) == arity, name
    assert len({n for n, _, _ in ent}) == len(ent)
    assert "void R_init_sparseRGPs(DllInfo* dll)" in text


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "RcppExports.cpp")),
                    reason="reference sources not present (GPU box)")
def test_fixture_matches_reference():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_rcpp_registry as M
    fix = json.load(open(FIX))
    assert M.call_entries(open(os.path.join(REF, "src/RcppExports.cpp")).read()) == fix["call_entries"]
    for f, p in M.FUNCS.items():
        assert M.formals(open(os.path.join(REF, p)).read(), f) == fix["formals"][f]


def _r_function_formals(text, name):
    m = re.search(r"^%s\s*<-\s*function\s*\(" % re.escape(name), text, re.M)
    assert m, name
    i = j = m.end()
    depth = 1
    while depth:
        depth += {"(": 1, ")": -1}.get(text[j], 0)
        j += 1
    args = re.sub(r"#[^\n]*", "", text[i:j - 1])
    return [re.sub(r"\s+", "", a) for a in args.split(",")]


def test_r_replacements_keep_the_formals():
    fix = json.load(open(FIX))["formals"]
    text = open(RFILE).read()
    for f, formals in fix.items():
        assert _r_function_formals(text, "sgp_" + f) == formals, f
        assert f'"{f}"' in text          # listed in sgp_install()


def _split_args(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    return [a for a in out if a.strip()]


def test_r_calls_match_registry():
    ent = {n: a for n, _, a in _entries(open(SHIM).read())}
    text = open(RFILE).read()
    calls = 0
    for m in re.finditer(r'\.Call\("(\w+)"', text):
        i = j = m.end()
        depth = 1
        while depth:
            depth += {"(": 1, ")": -1}.get(text[j], 0)
            j += 1
        nargs = len(_split_args(text[i:j - 1]))
        assert m.group(1) in ent, m.group(1)
        assert ent[m.group(1)] == nargs, (m.group(1), nargs)
        calls += 1
    assert calls >= 10


def test_shim_uses_only_declared_and_exported_entry_points():
    from sparsergps_amd import _build
    text = open(SHIM).read()
    used = set(re.findall(r"\b(sgp_[a-z0-9_]+)\s*\(", text))
    own = set(re.findall(r"^(?:SEXP|static \w+\*?)\s+(sgp_\w+)\(", text, re.M))
    used -= own
    used -= {f for _, f, _ in _entries(text)}
    header = open(os.path.join(ROOT, "include", "sgp.h")).read()
    for fn in used:
        assert re.search(r"\b%s\(" % fn, header), fn
    if not os.path.exists(_build.LIB):
        pytest.skip("libsgp.so not built")
    nm = subprocess.run(["nm", "-D", "--defined-only", _build.LIB], stdout=subprocess.PIPE,
                        check=True).stdout.decode()
    exported = set(re.findall(r" T (\w+)$", nm, re.M))
    assert used <= exported, used - exported
    assert len(used) >= 20


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_shim_compiles_against_r_api():
    res = subprocess.run(["gcc", "-fsyntax-only", "-std=c99", "-Wall", "-Wextra",
                          "-Wno-cast-function-type", "-Werror",
                          "-I" + os.path.join(ROOT, "tests", "r_api"),
                          "-I" + os.path.join(ROOT, "include"), SHIM],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    assert res.returncode == 0, res.stdout.decode()
