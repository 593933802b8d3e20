"""ctypes driver for rshim/sparseRGPs_sgp.c running on the mock R runtime (mock_rt.c).

TEST INFRASTRUCTURE.  ``build()`` links the shim, the mock runtime and libsgp.so into
tests/r_api/libsgp_rshim_mock.so (gcc; seconds); ``MockR`` builds R objects, calls registered
routines by name exactly as ``.Call`` would, and converts results back to numpy / dicts.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "libsgp_rshim_mock.so")
SRCS = [os.path.join(HERE, "mock_rt.c"), os.path.join(ROOT, "rshim", "sparseRGPs_sgp.c")]
SGP_DIR = os.path.join(ROOT, "sparsergps_amd", "lib")

REALSXP, STRSXP, VECSXP, EXTPTRSXP, INTSXP, LGLSXP, NILSXP = 14, 16, 19, 22, 13, 10, 0
NA_LOGICAL = -2 ** 31


def build(force=False):
    """Compile the mock-runtime shim library (needs libsgp.so built first)."""
    dep = SRCS + [os.path.join(ROOT, "include", "sgp.h"), os.path.join(SGP_DIR, "libsgp.so")]
    if (not force and os.path.exists(LIB)
            and os.path.getmtime(LIB) >= max(os.path.getmtime(p) for p in dep)):
        return LIB
    cmd = ["gcc", "-shared", "-fPIC", "-O1", "-g", "-std=gnu99", "-Wall", "-Wextra",
           "-Wno-cast-function-type", "-Werror", "-I", os.path.join(ROOT, "include"), "-I", HERE,
           *SRCS, "-L", SGP_DIR, "-lsgp", "-Wl,-rpath," + SGP_DIR, "-o", LIB + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


class RError(Exception):
    pass


class MockR:
    def __init__(self, path=LIB):
        L = C.CDLL(path)
        P = C.c_void_p
        for fn, res, args in [
            ("mock_load", C.c_int, []), ("mock_dynamic_symbols", C.c_int, []),
            ("mock_routine_name", C.c_char_p, [C.c_int]), ("mock_routine_arity", C.c_int, [C.c_int]),
            ("mock_real", P, [P, C.c_long]), ("mock_matrix", P, [P, C.c_int, C.c_int]),
            ("mock_int", P, [P, C.c_long]), ("mock_logical", P, [C.c_int]),
            ("mock_na_matrix", P, []), ("mock_strings", P, [P, C.c_long]),
            ("mock_list", P, [P, P, C.c_long]), ("mock_nil", P, []),
            ("mock_type", C.c_int, [P]), ("mock_length", C.c_long, [P]),
            ("mock_is_matrix", C.c_int, [P]), ("mock_nrow", C.c_int, [P]),
            ("mock_ncol", C.c_int, [P]), ("mock_real_ptr", P, [P]), ("mock_int_ptr", P, [P]),
            ("mock_elt", P, [P, C.c_long]), ("mock_name", C.c_char_p, [P, C.c_long]),
            ("mock_str", C.c_char_p, [P, C.c_long]),
            ("mock_error", C.c_char_p, []), ("mock_eprint", C.c_char_p, []),
            ("mock_protect_depth", C.c_int, []), ("mock_call", C.c_int, [C.c_char_p, C.c_int, P, P]),
            ("mock_gc", C.c_int, []), ("mock_reset", None, [])]:
            f = getattr(L, fn)
            f.restype, f.argtypes = res, args
        self.L = L
        self.n_routines = L.mock_load()
        self.routines = [(L.mock_routine_name(i).decode(), L.mock_routine_arity(i))
                         for i in range(self.n_routines)]
        self.eprint = ""
        self.called = set()

    # --------------------------------------------------------------- constructors
    # Every constructor returns a Handle; sexp() turns any Python value into a raw SEXP.
    def real(self, v):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(v, dtype=np.float64)).reshape(-1))
        return Handle(self, self.L.mock_real(a.ctypes.data, a.size))

    def mat(self, m):
        m = np.asarray(m, dtype=np.float64)
        if m.ndim == 1:
            m = m.reshape(-1, 1)
        a = np.asfortranarray(m)
        return Handle(self, self.L.mock_matrix(a.ctypes.data, m.shape[0], m.shape[1]))

    def int_(self, v):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(v, dtype=np.int32)))
        return Handle(self, self.L.mock_int(a.ctypes.data, a.size))

    def lgl(self, v):
        return Handle(self, self.L.mock_logical(NA_LOGICAL if v is None else int(bool(v))))

    def na_matrix(self):
        """R's matrix(): a 1 x 1 logical NA (the symmetric-mode sentinel)."""
        return Handle(self, self.L.mock_na_matrix())

    def str_(self, v):
        v = [v] if isinstance(v, str) else list(v)
        arr = (C.c_char_p * max(len(v), 1))(*[s.encode() for s in v])
        return Handle(self, self.L.mock_strings(C.cast(arr, C.c_void_p), len(v)))

    def list_(self, d):
        names = list(d.keys())
        vals = [self.sexp(x) for x in d.values()]
        na = (C.c_char_p * max(len(names), 1))(*[s.encode() for s in names])
        va = (C.c_void_p * max(len(vals), 1))(*vals)
        return Handle(self, self.L.mock_list(C.cast(na, C.c_void_p), C.cast(va, C.c_void_p),
                                             len(vals)))

    def nil(self):
        return Handle(self, self.L.mock_nil())

    def sexp(self, x):
        """Handle -> itself; numbers/arrays -> double vectors (2-D -> matrices); str / list of
        str -> character; dict -> named list; None -> NULL."""
        if isinstance(x, Handle):
            return x.p
        if x is None:
            return self.nil().p
        if isinstance(x, dict):
            return self.list_(x).p
        if isinstance(x, str) or (isinstance(x, (list, tuple)) and x and isinstance(x[0], str)):
            return self.str_(x).p
        a = np.asarray(x, dtype=np.float64)
        return (self.mat(a) if a.ndim == 2 else self.real(a)).p

    # --------------------------------------------------------------- .Call
    def call(self, name, *args):
        ps = [self.sexp(a) for a in args]
        arr = (C.c_void_p * max(len(ps), 1))(*ps)
        out = C.c_void_p()
        st = self.L.mock_call(name.encode(), len(ps), C.cast(arr, C.c_void_p), C.byref(out))
        self.called.add(name)
        self.eprint = self.L.mock_eprint().decode()
        if st == 1:
            raise RError(self.L.mock_error().decode())
        if st == 2:
            raise AssertionError(f"{name}: PROTECT stack unbalanced on return")
        if st in (3, 4):
            raise AssertionError(f"{name}: {'no such routine' if st == 3 else 'wrong arity'}")
        assert self.L.mock_protect_depth() == 0
        return Handle(self, out.value)

    def gc(self):
        return self.L.mock_gc()

    def reset(self):
        self.L.mock_reset()


class Handle:
    """An R object returned by a routine."""

    def __init__(self, r, p):
        self.r, self.p = r, p

    @property
    def type(self):
        return self.r.L.mock_type(self.p)

    def __len__(self):
        return self.r.L.mock_length(self.p)

    @property
    def dim(self):
        L = self.r.L
        return (L.mock_nrow(self.p), L.mock_ncol(self.p)) if L.mock_is_matrix(self.p) else None

    def py(self):
        L, t, n = self.r.L, self.type, len(self)
        if t == REALSXP:
            v = np.ctypeslib.as_array(C.cast(L.mock_real_ptr(self.p), C.POINTER(C.c_double)),
                                      (max(n, 1),))[:n].copy() if n else np.zeros(0)
            d = self.dim
            return v.reshape(d, order="F") if d else v
        if t in (INTSXP, LGLSXP):
            return np.ctypeslib.as_array(C.cast(L.mock_int_ptr(self.p), C.POINTER(C.c_int)),
                                         (max(n, 1),))[:n].copy()
        if t == STRSXP:
            return [L.mock_str(self.p, i).decode() for i in range(n)]
        if t == VECSXP:
            keys = [L.mock_name(self.p, i) for i in range(n)]
            vals = [Handle(self.r, L.mock_elt(self.p, i)).py() for i in range(n)]
            if all(k is not None for k in keys):
                return {k.decode(): v for k, v in zip(keys, vals)}
            return vals
        if t == NILSXP:
            return None
        return self
