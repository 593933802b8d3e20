"""C-ABI checks that need no GPU: libsgp.so builds for gfx950, loads, exports every symbol
include/sgp.h declares, and its host-only entry points behave (values, errors)."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

from oracle import sgp_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sgp.h")
HEADERS = sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))   # sgp.h + sgp_diag.h


@pytest.fixture(scope="module")
def lib():
    from sparsergps_amd import _lib
    return _lib.lib()


def declared_functions(paths=HEADERS):
    names = set()
    for p in paths:
        text = re.sub(r"/\*.*?\*/", "", open(p).read(), flags=re.S)
        names.update(re.findall(r"\b(sgp_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_expected_api():
    assert HEADER in HEADERS and len(HEADERS) >= 2
    names = declared_functions()
    assert "sgp_diag_gj_pair" in names and "sgp_lap_set_expo" in names
    for must in ("sgp_make_cov", "sgp_dsig_dtheta", "sgp_ctx_create", "sgp_eval_vi",
                 "sgp_vi_phase1", "sgp_vi_phase2", "sgp_vi_finish", "sgp_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    from sparsergps_amd import _lib
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in _lib.PROTOTYPES, f"{name} missing from the ctypes prototype table"


def test_lib_is_built_for_gfx950():
    from sparsergps_amd._build import LIB
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob


def test_versions_and_counts(lib):
    assert lib.sgp_abi_version() == 1
    assert lib.sgp_num_params(0, 3) == 3 and lib.sgp_num_params(1, 8) == 10
    assert lib.sgp_num_params(2, 4) == 3 and lib.sgp_num_params(7, 1) == -1
    assert lib.sgp_vi_red1_count(1024) == 1024 * 1024 + 1024 + 8
    assert lib.sgp_vi_red1_count(20) == 128 * 128 + 128 + 8
    assert lib.sgp_vi_red2_count(1, 8) == 13 and lib.sgp_vi_red2_count(0, 3) == 6


def _theta(cp, kernel, d):
    from sparsergps_amd.covariance import theta_vector
    return theta_vector(cp, kernel, d, None, need_tau=True)


@pytest.mark.parametrize("kernel", ["sqexp", "exp", "ard"])
def test_pair_functions_match_oracle(lib, kernel):
    from sparsergps_amd import _lib
    rng = np.random.default_rng(5)
    d = 3
    if kernel == "ard":
        cp = {"sigma": 1.4, "l1": 0.7, "l2": 1.1, "l3": 2.0, "tau": 0.3}
        names = ["sigma", "l1", "l2", "l3", "tau"]
    else:
        cp = {"sigma": 1.4, "l": 0.9, "tau": 0.3}
        names = ["sigma", "l", "tau"]
    th = _theta(cp, kernel, d)
    kid = _lib.KERNELS[kernel]
    for _ in range(5):
        x1 = rng.uniform(0, 3, size=d)
        x2 = x1.copy() if _ == 0 else rng.uniform(0, 3, size=d)
        a, b = x1.reshape(1, -1), x2.reshape(1, -1)
        if kernel == "ard":
            ref = O.make_cov_mat_ardC(a, b, cp, "ard", 0, ["l1", "l2", "l3"])[0, 0]
        else:
            ref = O.make_cov_matC(a, b, cp, kernel, 0)[0, 0]
        got = lib.sgp_kernel_pair(kid, _lib.dptr(x1), _lib.dptr(x2), d, _lib.dptr(th))
        assert abs(got - ref) <= 1e-14 * abs(ref)
        for p, nm in enumerate(names):
            if kernel == "ard":
                dref = O.dsig_dtheta_ardC(a, b, cp, "ard", nm, ["l1", "l2", "l3"])[0, 0]
            else:
                dref = O.dsig_dthetaC(a, b if kernel != "exp" or nm != "tau" else None, cp, kernel, nm)[0, 0] \
                    if not (kernel == "exp" and nm == "tau") else (2 * 0.09 if np.array_equal(x1, x2) else 0.0)
            dgot = lib.sgp_dkernel_pair(kid, _lib.dptr(x1), _lib.dptr(x2), d, _lib.dptr(th), p)
            assert abs(dgot - dref) <= 1e-13 * max(1e-300, abs(dref)), (nm, dgot, dref)


def test_errors_without_gpu(lib):
    from sparsergps_amd import _lib
    x = np.zeros((4, 2), order="F")
    out = np.zeros((4, 4), order="F")
    th = np.array([1.0, 1.0, 0.5])
    st = lib.sgp_make_cov(0, 9, _lib.dptr(x), 4, 4, None, 0, 0, 2, _lib.dptr(th), 1e-6, _lib.dptr(out), 4)
    assert st == _lib.SGP_EINVAL and b"invalid covariance function" in lib.sgp_last_error()
    bad = np.array([1.0, -2.0, 0.5])
    st = lib.sgp_make_cov(0, 0, _lib.dptr(x), 4, 4, None, 0, 0, 2, _lib.dptr(bad), 1e-6, _lib.dptr(out), 4)
    assert st == _lib.SGP_EINVAL and b"length scale" in lib.sgp_last_error()
    st = lib.sgp_dsig_dtheta(0, 0, _lib.dptr(x), 4, 4, None, 0, 0, 2, _lib.dptr(th), 5, _lib.dptr(out), 4)
    assert st == _lib.SGP_EINVAL and b"parameter" in lib.sgp_last_error()
    h = C.c_void_p()
    y = np.zeros(4)
    st = lib.sgp_ctx_create(C.byref(h), 0, _lib.dptr(x), 4, 4, 99, _lib.dptr(y), _lib.dptr(y), 8)
    assert st == _lib.SGP_EINVAL
    assert lib.sgp_eval_vi(None, 0, None, None, 1, 1, 1e-6, 0, None, None) == _lib.SGP_EINVAL
    assert lib.sgp_ctx_destroy(None) == _lib.SGP_OK


def test_product_path_fails_loudly_without_gpu():
    """No silent CPU fallback: on a host without a HIP device the product path raises."""
    from sparsergps_amd import _lib
    n = C.c_int(0)
    st = _lib.lib().sgp_device_count(C.byref(n))
    if st == _lib.SGP_OK and n.value > 0:
        pytest.skip("a GPU is visible")
    import sparsergps_amd as S
    with pytest.raises(RuntimeError):
        S.make_cov_matC(np.ones((3, 1)), None, {"sigma": 1, "l": 1, "tau": 0.1}, "sqexp", 1e-6)
    with pytest.raises(RuntimeError):
        S.SparseGPContext(np.ones((3, 1)), np.ones(3), 0.0, 4)


def test_multi_context_argument_validation(lib):
    """sgp_ctx_create_multi's argument checks run before any device call (SGP_EINVAL with a
    message), so they are testable here; with valid arguments and no GPU it fails loudly."""
    from sparsergps_amd import _lib
    X = np.zeros((10, 2), order="F")
    y = np.zeros(10)
    h = C.c_void_p()

    def create(devs, nshards, n=10, d=2, m_max=8, x=X):
        dv = None if devs is None else (C.c_int * len(devs))(*devs)
        return lib.sgp_ctx_create_multi(C.byref(h), dv, nshards, _lib.dptr(x), n, n, d,
                                        _lib.dptr(y), _lib.dptr(y), m_max)

    for args in ((None, 0), (None, 65), ([0] * 11, 11), (None, 2, 10, 0), (None, 2, 10, 2, 0),
                 (None, 2, 10, 33)):
        assert create(*args) == _lib.SGP_EINVAL, args
        assert b"sgp_ctx_create_multi" in lib.sgp_last_error()
    assert create([0, -1], 2) == _lib.SGP_EINVAL and b"device -1" in lib.sgp_last_error()
    assert h.value is None
    n = C.c_int(0)
    if lib.sgp_device_count(C.byref(n)) != _lib.SGP_OK or n.value == 0:
        assert create([0, 0], 2) == _lib.SGP_EHIP     # no device: no context, no fallback
        assert h.value is None
    ns, nd = C.c_int(0), C.c_int(0)
    assert lib.sgp_ctx_shards(None, C.byref(ns), C.byref(nd)) == _lib.SGP_EINVAL


def test_fast_eval_prototype_matches_the_table():
    """SparseGPContext.eval_vi / eval_fitc call sgp_eval_vi / sgp_eval_fitc through a raw-address
    CFUNCTYPE: same return type and argument count and kinds as the checked prototype table
    (pointers as c_void_p, scalars identical)."""
    from sparsergps_amd import _lib
    from sparsergps_amd.vi import SparseGPContext
    proto = SparseGPContext._EVAL_PROTO
    for name in ("sgp_eval_vi", "sgp_eval_fitc"):
        res, args = _lib.PROTOTYPES[name]
        assert proto._restype_ is res
        assert len(proto._argtypes_) == len(args)
        for fast, ref in zip(proto._argtypes_, args):
            if fast is C.c_void_p:
                assert ref is C.c_void_p or issubclass(ref, C._Pointer), (name, ref)
            else:
                assert fast is ref, (name, fast, ref)
